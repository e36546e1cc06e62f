"""Ad-hoc GPU diagnostics (GPU box): python scripts/debug_gpu.py <what>"""
import sys
import os

sys.path[:0] = [os.path.join(os.path.dirname(__file__), d) for d in
                ("../parallel-systems-mpi-tfidf_amd/python", "../oracle", "../tests")]
import numpy as np  # noqa: E402

import oracle_py  # noqa: E402
import tfidf_abi  # noqa: E402
import tfidf_configs  # noqa: E402


def dup_report(res, tag):
    terms = res["terms"]
    seen = {}
    dups = [t for t in terms if t in seen or seen.setdefault(t, 0)]
    print(tag, "nterms", len(terms), "distinct strings", len(set(terms)), "dup examples", dups[:5])
    d, t = res["doc"], res["term"]
    same = np.flatnonzero((d[1:] == d[:-1]) & (t[1:] == t[:-1]))
    print(tag, "adjacent duplicate (doc,term) records:", len(same), same[:5])


def c2_small():
    p = tfidf_configs.plan("c2", scale=0.003)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    with tfidf_abi.Engine(0) as e:
        e.run_host(data, off, p["doc_ids"], p["ndocs_total"])
        print(e.info())
        res = e.fetch()
    ora = oracle_py.run(data, off, p["doc_ids"], p["ndocs_total"])
    dup_report(res, "gpu")
    print("oracle pairs", ora["npairs"], "gpu pairs", res["npairs"], "oracle nterms", ora["nterms"])
    # per-doc count sums vs docsize
    for name, r in (("gpu", res), ("ora", ora)):
        starts = np.flatnonzero(np.r_[True, r["doc"][1:] != r["doc"][:-1]])
        sums = np.add.reduceat(r["count"].astype(np.int64), starts)
        bad = np.flatnonzero(sums != r["docsize"][starts])
        print(name, "docs with count-sum != docsize:", [(int(r["doc"][starts[b]]), int(sums[b]),
                                                         int(r["docsize"][starts[b]])) for b in bad[:5]])
    # where are the 'aagt' records of doc106
    for name, r in (("gpu", res), ("ora", ora)):
        idx = [i for i in np.flatnonzero(r["doc"] == 106) if r["terms"][r["term"][i]] == b"aagt"]
        print(name, "doc106 aagt records", [(int(i), int(r["term"][i]), int(r["count"][i])) for i in idx])


def rccl1():
    p = tfidf_configs.plan("c2", scale=0.002)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    with tfidf_abi.Engine(0) as e:
        e.comm_init(tfidf_abi.comm_unique_id(), 0, 1)
        e.run_host(data, off, p["doc_ids"], p["ndocs_total"])
        print(e.info())
        res = e.fetch()
    ora = oracle_py.run(data, off, p["doc_ids"], p["ndocs_total"])
    print("rccl1 equal:", res["output_txt"] == ora["output_txt"])


def stamps():
    """K1 phase breakdown (diagnostic build): TFIDF_LIB=stamps TFIDF_STAMPS=1"""
    import ctypes as C
    names = ["group setup", "barrier wait (walk imbalance)", "flush tail", "docsize write", "classify", "compact",
             "round: keys+loads", "round: compare+miss", "round: docsize", "round: LDS count",
             "round: claims", "step loop top", "flush: sync+zero", "flush: pass 1", "flush: decide+alloc",
             "flush: staging", "flush: write-out"]
    NS = len(names)
    p = tfidf_configs.plan("c2", scale=float(os.environ.get("SCALE", "1.0")))
    with tfidf_abi.Engine(0) as e:
        c = e.synth_device(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"], p["ndocs_total"])
        for _ in range(2):
            e.run_corpus(c)
        info = e.info()
        buf = (C.c_uint64 * (NS + 5))()
        L = tfidf_abi.lib()
        L.tfidf_debug_k1_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        n = L.tfidf_debug_k1_stamps(e.h, buf, NS + 5)
        print("tokens", info["ntokens"], "counted", buf[NS + 1], "vocab first-probe misses", buf[NS + 2],
              "-", buf[NS + 3], "lane token-loop iterations", buf[NS + 4])
    print("k1 ms", info["ms_tokcount"], "flags", info["flags"], "stamps", n)
    wgs = buf[NS]
    tot = sum(buf[:NS])
    for k in range(NS):
        print("%-30s %12.0f cyc/WG  %5.1f%%" % (names[k], buf[k] / max(wgs, 1), 100.0 * buf[k] / max(tot, 1)))
    print("WGs", wgs, "total cyc/WG", tot / max(wgs, 1))


if __name__ == "__main__":
    globals()[sys.argv[1]]()
