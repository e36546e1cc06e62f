"""CPU-side checks of the product boundary (no GPU compute calls):
the C-ABI library loads and exports every function include/tfidf.h declares; the host
synthetic generator is deterministic and matches the config plans; document-name
ordering keys match strcmp; host ingest follows the reference's input contract."""
import ctypes as C
import os
import re
import tempfile

import numpy as np

import tfidf_abi
import tfidf_configs
from conftest import REPO


def declared_functions():
    with open(os.path.join(REPO, "include", "tfidf.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tfidf_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = tfidf_abi.lib()
    decl = declared_functions()
    assert len(decl) >= 18
    for name in decl:
        assert hasattr(lib, name), name
    assert set(tfidf_abi.EXPORTS) <= set(decl)
    assert lib.tfidf_abi_version() == tfidf_abi.ABI_VERSION == 2


def test_library_is_gfx950_code_object():
    """The shared library embeds gfx950 code objects (objdump extracts the offload
    bundles next to its input, so work on a copy in a scratch directory)."""
    import shutil
    import subprocess
    with tempfile.TemporaryDirectory() as td:
        lib_copy = os.path.join(td, "lib.so")
        shutil.copy(tfidf_abi.LIB_PATH, lib_copy)
        p = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib_copy],
                           capture_output=True, text=True, cwd=td)
    assert "gfx950" in (p.stdout + p.stderr)


def test_strerror_messages_match_reference():
    lib = tfidf_abi.lib()
    assert lib.tfidf_strerror(-6) == b"Directory failed to open"
    assert lib.tfidf_strerror(-7) == b"Error Opening File"


def test_synth_host_deterministic_and_sized():
    p = tfidf_configs.plan("c2", scale=0.001)
    a, oa = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    b, ob = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    assert np.array_equal(a, b) and np.array_equal(oa, ob)
    assert oa[-1] == len(a)
    # token count per doc == plan (separators are single ' ' or '\n')
    txt = bytes(a)
    for i in range(min(20, len(p["ntok"]))):
        doc = txt[int(oa[i]):int(oa[i + 1])]
        assert len(doc.split()) == int(p["ntok"][i])
        assert doc.endswith(b"\n")
    mean_tok_bytes = len(a) / float(p["ntok"].sum())
    assert abs(mean_tok_bytes - tfidf_configs.bytes_per_token(p["V"])) < 1.0  # Zipf weights the head terms


def test_config1_is_reference_safe():
    p = tfidf_configs.plan("c1")
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], None, p["doc_ids"], p["ntok"])
    words = set()
    pairs = set()
    for i in range(8):
        for w in bytes(data[int(off[i]):int(off[i + 1])]).split():
            words.add(w)
            pairs.add((i, w))
            assert len(w) <= 15
    assert len(pairs) == 32 and len(words) <= 29


def test_doc_name_key_is_strcmp_order():
    ids = np.arange(1, 2501, dtype=np.uint32)
    k = tfidf_configs.doc_name_key(ids)
    by_key = ids[np.argsort(k, kind="stable")].tolist()
    by_str = sorted(ids.tolist(), key=lambda i: b"doc%d@" % i)
    assert by_key == by_str


def test_shard_plan_partitions_in_name_order():
    full = tfidf_configs.plan("c2", scale=0.002)
    shards = [tfidf_configs.plan("c2", scale=0.002, rank=r, nranks=3) for r in range(3)]
    ids = np.concatenate([s["doc_ids"] for s in shards])
    assert sorted(ids.tolist()) == sorted(full["doc_ids"].tolist())
    keys = tfidf_configs.doc_name_key(ids)
    assert np.all(np.diff(keys.astype(np.int64)) > 0)
    assert all(s["ndocs_total"] == len(full["doc_ids"]) for s in shards)


def test_ingest_dir_contract():
    lib = tfidf_abi.lib()
    with tempfile.TemporaryDirectory() as td:
        pb = C.c_void_p(); nb = C.c_uint64(); po = C.c_void_p(); nd = C.c_uint32(); bad = C.c_uint32()
        args = [C.byref(pb), C.byref(nb), C.byref(po), C.byref(nd), C.byref(bad)]
        lib.tfidf_ingest_dir.argtypes = [C.c_char_p] + [C.c_void_p] * 5
        assert lib.tfidf_ingest_dir(os.path.join(td, "nope").encode(), *args) == -6
        d = os.path.join(td, "input")
        os.makedirs(d)
        for i, s in enumerate([b"a b", b"", b"c\n"], 1):
            with open(os.path.join(d, f"doc{i}"), "wb") as f:
                f.write(s)
        os.makedirs(os.path.join(d, ".hidden"))  # every entry counts in N (TFIDF.c:104-109)
        assert lib.tfidf_ingest_dir(d.encode(), *args) == -7
        assert bad.value == 4 and nd.value == 4
        os.rmdir(os.path.join(d, ".hidden"))
        assert lib.tfidf_ingest_dir(d.encode(), *args) == 0
        assert nd.value == 3 and nb.value == 5
        off = np.ctypeslib.as_array(C.cast(po, C.POINTER(C.c_uint64)), shape=(4,)).copy()
        assert off.tolist() == [0, 3, 3, 5]
        lib.tfidf_free.argtypes = [C.c_void_p]
        lib.tfidf_free(pb)
        lib.tfidf_free(po)


def test_doc_name_order_is_strcmp_order():
    """tfidf_doc_name_order (the shard plan's document order): "docN@" strcmp order."""
    for n in (1, 9, 10, 12, 100, 2345):
        got = tfidf_abi.doc_name_order(n).tolist()
        assert got == sorted(range(1, n + 1), key=lambda i: b"doc%d@" % i)


def test_shard_split_is_byte_balanced():
    """tfidf_shard_split == the Python planner's rule; every shard holds at most
    total / K + the largest document, shards are contiguous and cover all."""
    rng = np.random.default_rng(5)
    cases = [rng.integers(0, 1000, 500), rng.integers(0, 10, 50), np.array([5, 1, 1, 1, 10, 1, 1]),
             np.array([100_000_000] * 4 + [600] * 5000), np.zeros(7, np.int64), np.array([3])]
    for sizes in cases:
        sizes = sizes.astype(np.uint64)
        for K in (1, 2, 3, 4, 8):
            first = tfidf_abi.shard_split(sizes, K)
            assert first.tolist() == tfidf_configs.shard_cuts(sizes, K).tolist()
            assert first[0] == 0 and first[-1] == len(sizes) and np.all(np.diff(first.astype(np.int64)) >= 0)
            total = int(sizes.sum())
            big = int(sizes.max()) if len(sizes) else 0
            for r in range(K):
                b = int(sizes[first[r]:first[r + 1]].sum())
                assert b <= total / K + big


def test_c5_plan_balances_the_100mb_documents():
    """c5 at 8 shards (4 x 100 MB among 1e6 small documents): token-balanced shards."""
    sh = [tfidf_configs.plan("c5", scale=0.02, rank=r, nranks=8) for r in range(8)]
    tok = [int(s["ntok"].sum()) for s in sh]
    big = max(int(s["ntok"].max()) for s in sh)
    assert max(tok) <= sum(tok) / 8 + big
    ids = np.concatenate([s["doc_ids"] for s in sh])
    keys = tfidf_configs.doc_name_key(ids)
    assert np.all(np.diff(keys.astype(np.int64)) > 0)


def test_plan_dir_contract():
    """tfidf_plan_dir (host only): N counts every entry, the error contract of TFIDF.c:
    100-103 / 134-138, "docN@" order, byte-balanced shards."""
    with tempfile.TemporaryDirectory() as td:
        try:
            tfidf_abi.plan_dir(os.path.join(td, "nope"), 2)
            raise AssertionError("expected an error")
        except tfidf_abi.TfidfError as e:
            assert e.rc == -6
        d = os.path.join(td, "input")
        os.makedirs(d)
        sizes = [5, 0, 300, 7, 1, 90, 44, 3, 2, 20, 11, 8]
        for i, n in enumerate(sizes, 1):
            with open(os.path.join(d, f"doc{i}"), "wb") as f:
                f.write(b"x" * n)
        os.makedirs(os.path.join(d, ".hidden"))
        try:
            tfidf_abi.plan_dir(d, 2)
            raise AssertionError("expected an error")
        except tfidf_abi.TfidfError as e:
            assert e.rc == -7 and e.bad_doc == 13 and e.ndocs == 13
        os.rmdir(os.path.join(d, ".hidden"))
        p = tfidf_abi.plan_dir(d, 3)
        assert p["ndocs"] == 12
        assert p["doc_ids"].tolist() == sorted(range(1, 13), key=lambda i: b"doc%d@" % i)
        assert p["doc_bytes"].tolist() == [sizes[i - 1] for i in p["doc_ids"].tolist()]
        f = p["shard_first"]
        assert f.tolist() == tfidf_abi.shard_split(p["doc_bytes"], 3).tolist()
        assert [int(p["doc_bytes"][f[r]:f[r + 1]].sum()) for r in range(3)] == p["shard_bytes"].tolist()
