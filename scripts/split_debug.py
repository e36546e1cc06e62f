"""Split-K1 diagnostics (GPU box): runs small corpora through the engine and prints K1a's
chunk metadata, ordinal lists and token words next to a host tokenisation.
Usage: python scripts/split_debug.py"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-systems-mpi-tfidf_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import tfidf_abi  # noqa: E402
import tfidf_configs  # noqa: E402

L = tfidf_abi.lib()
L.tfidf_debug_split.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_uint64]


def dump(e, what, n):
    buf = np.zeros(max(n, 1), dtype=np.uint32)
    m = L.tfidf_debug_split(e.h, what, buf.ctypes.data, n)
    return buf[:max(m, 0)]


WS = set(b" \t\n\v\f\r")


def host_tokens(data, off):
    out = []
    for d in range(len(off) - 1):
        doc = bytes(data[off[d]:off[d + 1]])
        out.append([t.split(b"\0")[0] for t in doc.split() if True])
    return out


def show(name, data, off):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    N = len(off) - 1
    span = int(off[-1] - off[0])
    nch = (span + 16383) // 16384
    with tfidf_abi.Engine(0) as e:
        e.run_host(data, off)
        info = e.info()
        meta = dump(e, 1, 2 * nch).reshape(-1, 2)
        dl = dump(e, 2, N + nch + 2)
        dt = dump(e, 3, N + nch + 2)
        words = dump(e, 0, span // 2 + N + 4 * nch + 64)
    toks = host_tokens(data, off)
    print(f"== {name}: N={N} span={span} nch={nch} info.ntokens={info.get('ntokens')} V={info.get('nterms')} "
          f"host tokens={sum(len(t) for t in toks)}")
    print("meta (ntok, ndocs) per chunk:", meta[:min(nch, 12)].tolist(), "... sum ntok", int(meta[:, 0].sum()))
    print("dlist[:16]", dl[:16].tolist())
    print("dtok[:16]", dt[:16].tolist())
    print("words[:24]", [hex(x) for x in words[:24]])
    print("host docsizes[:8]", [len(t) for t in toks[:8]])


if __name__ == "__main__" and len(sys.argv) == 1:
    txt = [b"alpha beta gamma alpha", b"beta beta  delta\n", b"x", b"", b"gamma alpha y z beta"]
    data = np.frombuffer(b"".join(txt), dtype=np.uint8)
    off = np.cumsum([0] + [len(t) for t in txt]).astype(np.uint64)
    show("tiny", data, off)
    p = tfidf_configs.plan("c2", scale=0.0005)
    d, o = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    show("c2 slice", d, o)


def diff_golden(case):
    """First TF-job differences (word@doc count/docsize) of the default K1 vs the golden."""
    from helpers import load_golden, jobs_from_result
    g = load_golden(case)
    with tfidf_abi.Engine(0) as e:
        e.run_host(g["data"], g["off"])
        r = e.fetch()
        meta = dump(e, 1, 8).reshape(-1, 2)
        dl = dump(e, 2, 40)
        dt = dump(e, 3, 40)
    tf, _ = jobs_from_result(r)
    a = set(tf.split(b"\n")) - {b""}
    b = set(g["tf_jobs"].split(b"\n")) - {b""}
    print(f"== {case}: N={len(g['off']) - 1} gpu pairs {len(a)} golden {len(b)}; meta {meta.tolist()}")
    print("dlist", dl.tolist())
    print("dtok", dt.tolist())
    print("docsizes", [int(g['off'][i + 1] - g['off'][i]) for i in range(len(g['off']) - 1)])
    print("only gpu:", sorted(a - b)[:12])
    print("only golden:", sorted(b - a)[:12])


if __name__ == "__main__" and len(sys.argv) > 1:
    for case in sys.argv[1:]:
        diff_golden(case)
