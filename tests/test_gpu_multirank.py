"""GPU parity of the multi-shard product path (engine.cpp exchange_df, group.cpp).

K shards of one corpus run through tfidf_group_* on K contexts.  On the one-GPU test box
the contexts share device 0 and exchange through the in-process transport (xport.h): the
engine code is the one the RCCL clique runs — the status/size agreement, the per-owner
partition of each rank's terms (a hash of the identity key picks the owner rank), the
count all-gather, the (key, df) all-to-all, the owners' hash aggregation, the all-to-all
of the global df back, and the global V.  Against the single-rank oracle (TFIDF.c:209-222,
291-326 DF combine; :253-273 gather + sort):
  * the shards' GPU-formatted texts, concatenated in rank order, are the oracle's
    output.txt byte for byte;
  * every pair's count, docSize and global DF, and every score, are bit-exact;
  * every rank reports the same global vocabulary size = the oracle's distinct terms.
The 1-rank RCCL communicator case runs the same exchange with ncclAllGather and grouped
ncclSend / ncclRecv (no `nranks > 1` shortcut)."""
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_py
import tfidf_abi
import tfidf_configs
from conftest import GOLDEN
from helpers import assert_same_result, load_golden

pytestmark = pytest.mark.gpu


def _shards(cfg, scale, K):
    shards = []
    for r in range(K):
        p = tfidf_configs.plan(cfg, scale=scale, rank=r, nranks=K)
        d, o = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
        shards.append((d, o, p["doc_ids"], p["ndocs_total"]))
    return shards


def _full(cfg, scale):
    p = tfidf_configs.plan(cfg, scale=scale)
    d, o = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    return oracle_py.run(d, o, p["doc_ids"], p["ndocs_total"])


def _concat(results):
    """rank-order concatenation of fetched shard results, terms as bytes"""
    out = {k: np.concatenate([r[k] for r in results]) for k in ("doc", "count", "docsize", "df", "score")}
    out["npairs"] = sum(r["npairs"] for r in results)
    tb = [r["terms"][t] for r in results for t in r["term"].tolist()]
    uniq = sorted(set(tb))
    gid = {t: i for i, t in enumerate(uniq)}
    out["terms"] = uniq
    out["term"] = np.array([gid[t] for t in tb], dtype=np.uint32)
    return out


def _run_group(shards, K, **kw):
    with tfidf_abi.Group(K, devices=[0] * K, **kw) as g:
        g.run_host(shards)
        texts = [e.text() for e in g.ranks]
        res = [e.fetch() for e in g.ranks]
        infos = [e.info() for e in g.ranks]
    return texts, res, infos


@pytest.mark.parametrize("xchg", ["dense", "dense_table", "owner", "owner_table"])
@pytest.mark.parametrize("cfg,scale,K", [("c2", 0.003, 2), ("c2", 0.003, 3), ("c5", 0.0005, 2), ("c5", 0.0005, 3),
                                         ("c4", 0.001, 2), ("c2", 0.003, 5), ("c4", 0.01, 4)])
def test_group_shards_equal_single_rank_oracle(cfg, scale, K, xchg, monkeypatch):
    """Both forms of the DF exchange (engine.cpp): the dense all-reduce over shared
    positions (the default up to 2^17 terms per rank; numbered by merging the ranks' term
    lists, or through a table of the gathered keys with dense_table) and the hash-owner
    all-to-all (the owners aggregate in LDS buckets, or in an HBM table with owner_table)."""
    monkeypatch.setenv("TFIDF_XCHG", xchg.replace("owner_table", "owner"))   # read by tfidf_open
    if xchg == "owner_table":
        monkeypatch.setenv("TFIDF_XAGG", "table")
    shards = _shards(cfg, scale, K)
    ora = _full(cfg, scale)
    texts, res, infos = _run_group(shards, K)
    assert b"".join(texts) == ora["output_txt"]
    assert_same_result(_concat(res), ora)
    # identical global ids on every rank: the union size is the corpus vocabulary
    assert all(i["nterms_global"] == ora["nterms"] for i in infos)
    # shards really differ in vocabulary (the 0xEE padding of the all-gather is exercised)
    assert len({i["nterms"] for i in infos}) > 1


@pytest.mark.parametrize("cfg,scale,K", [("c4", 0.01, 4), ("c2", 0.003, 3)])
def test_owner_buckets_compared_in_memory(cfg, scale, K, monkeypatch):
    """The owner form's path for a bucket too large to stage in LDS (more than 1024 records:
    not expected at a mean of <= 512, so TFIDF_XB_STAGE_MAX=0 sends every bucket there):
    keys compared in memory (finalize.hip k_xb_bucket), the same result."""
    monkeypatch.setenv("TFIDF_XCHG", "owner")
    monkeypatch.setenv("TFIDF_XB_STAGE_MAX", "0")
    shards = _shards(cfg, scale, K)
    ora = _full(cfg, scale)
    texts, res, infos = _run_group(shards, K)
    assert b"".join(texts) == ora["output_txt"]
    assert_same_result(_concat(res), ora)
    assert all(i["nterms_global"] == ora["nterms"] for i in infos)


@pytest.mark.parametrize("xchg", ["dense", "dense_table", "owner"])
def test_group_long_terms(xchg, monkeypatch):
    """Terms of >= 16 bytes (hash-tagged identity keys, not in term order) on the ranks: the
    flag travels in the agreement word and every rank numbers the dense exchange through the
    table; the same long term on two ranks gets one global DF."""
    monkeypatch.setenv("TFIDF_XCHG", xchg)
    base = _shards("c2", 0.002, 2)
    N = base[0][3] + 2
    nid = int(max(int(b[2].max()) for b in base)) + 1
    extra = [b"supercalifragilisticexpialidocious internationalization a\n",
             b"zz supercalifragilisticexpialidocious\n"]
    shards = []
    for r, (d, o, ids, _) in enumerate(base):
        x = np.frombuffer(extra[r], dtype=np.uint8)
        shards.append((np.concatenate([d, x]), np.concatenate([o, [o[-1] + len(x)]]).astype(np.uint64),
                       np.concatenate([ids, [nid + r]]).astype(np.uint32), N))
    texts, res, infos = _run_group(shards, 2)
    data = np.concatenate([shards[0][0], shards[1][0]])
    off = np.concatenate([shards[0][1], shards[0][1][-1] + shards[1][1][1:]])
    ids = np.concatenate([shards[0][2], shards[1][2]])
    ora = oracle_py.run(data, off, ids, N)
    assert sorted(b"".join(texts).split(b"\n")) == sorted(ora["output_txt"].split(b"\n"))
    assert all(i["nterms_global"] == ora["nterms"] for i in infos)


_M64 = (1 << 64) - 1


def _long_key16(t):
    """dev_common.h make_long_key's 120-bit hash truncated to the 16 bits the test build
    lib/libtfidf_hip_longtag16.so keeps"""
    def mix64(z):
        z ^= z >> 30
        z = (z * 0xBF58476D1CE4E5B9) & _M64
        z ^= z >> 27
        z = (z * 0x94D049BB133111EB) & _M64
        return z ^ (z >> 31)
    n = len(t)
    h1 = 0x243F6A8885A308D3 ^ n
    h2 = (0x13198A2E03707344 + n * 0x9E3779B97F4A7C15) & _M64
    for c in t:
        h1 = ((h1 ^ c) * 0x100000001B3) & _M64
        h2 = ((h2 + c + 1) * 0xC2B2AE3D27D4EB4F) & _M64
        h2 ^= h2 >> 29
    return mix64(h1 ^ ((h2 << 1) & _M64)) & 0xFFFF


def _colliding_long_pair():
    seen = {}
    for i in range(100000):
        t = b"crossrankcollision%05d" % i
        k = _long_key16(t)
        if k in seen:
            return seen[k], t
        seen[k] = t
    raise AssertionError("no 16-bit collision found")


def _long_pair_shards(a, b):
    """two c2 shards, rank 0 with a document holding term a, rank 1 one holding term b"""
    base = _shards("c2", 0.002, 2)
    N = base[0][3] + 2
    nid = int(max(int(s[2].max()) for s in base)) + 1
    shards = []
    for r, (d, o, ids, _) in enumerate(base):
        x = np.frombuffer(b"w " + (a, b)[r] + b" z\n", dtype=np.uint8)
        shards.append((np.concatenate([d, x]), np.concatenate([o, [o[-1] + len(x)]]).astype(np.uint64),
                       np.concatenate([ids, [nid + r]]).astype(np.uint32), N))
    return shards


_CROSS_LONG_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2]); sys.path.insert(0, sys.argv[3])
import numpy as np, tfidf_abi, test_gpu_multirank as t
a, b = t._colliding_long_pair()
# one rank holding both: the in-rank byte verification (dev_vocab.h) reports the pair
# (this also pins the test's copy of the hash to the device's)
with tfidf_abi.Engine(0) as e:
    x = b"w " + a + b" z\nq " + b + b"\n"
    try:
        e.run_host(np.frombuffer(x, dtype=np.uint8), np.array([0, 5 + len(a), len(x)], dtype=np.uint64))
        print("RESULT one merged")
    except tfidf_abi.TfidfError as ex:
        print("RESULT one rc=%d" % ex.rc)
# one term on each rank: only the exchange meets them, and its check reports them
for xchg in ("dense", "owner"):
    import os
    os.environ["TFIDF_XCHG"] = xchg
    with tfidf_abi.Group(2, devices=[0, 0]) as g:
        try:
            g.run_host(t._long_pair_shards(a, b))
            print("RESULT two %s merged" % xchg)
        except tfidf_abi.TfidfError as ex:
            print("RESULT two %s rc=%d" % (xchg, ex.rc))
"""


def test_cross_rank_long_term_collision_is_reported():
    """Cross-rank identity of terms of >= 16 bytes is byte-exact (engine.cpp
    exchange_long_check): the DF exchange meets long terms by their 120-bit hash keys, so every
    key two ranks share is then compared byte by byte, as TFIDF.c:229's strcmp would.  The
    test library truncates the keys to 16 bits: two distinct long terms with one 16-bit key,
    one per rank, fail the run with TFIDF_E_CAPACITY on both exchange forms (never merged);
    on one rank the in-rank verification reports the same pair."""
    here = os.path.dirname(os.path.abspath(__file__))
    pydir = os.path.join(os.path.dirname(here), "parallel-systems-mpi-tfidf_amd", "python")
    env = dict(os.environ, TFIDF_LIB="longtag16")
    import sys
    r = subprocess.run([sys.executable, "-c", _CROSS_LONG_CHILD, pydir, here, os.path.join(os.path.dirname(here), "oracle")],
                       env=env, capture_output=True, text=True, timeout=240, cwd=here)
    out = [l for l in r.stdout.splitlines() if l.startswith("RESULT")]
    assert out == ["RESULT one rc=-9", "RESULT two dense rc=-9", "RESULT two owner rc=-9"], r.stdout + r.stderr[-3000:]
    assert "on different ranks share their 120-bit identity key" in r.stderr


@pytest.mark.parametrize("xchg", ["dense", "owner"])
def test_cross_rank_distinct_long_terms_equal_oracle(xchg, monkeypatch):
    """The same pair under the product library's full 120-bit keys: two distinct terms, the
    check passes and the shards equal the single-rank oracle."""
    monkeypatch.setenv("TFIDF_XCHG", xchg)
    shards = _long_pair_shards(*_colliding_long_pair())
    texts, res, infos = _run_group(shards, 2)
    data = np.concatenate([shards[0][0], shards[1][0]])
    off = np.concatenate([shards[0][1], shards[0][1][-1] + shards[1][1][1:]])
    ids = np.concatenate([shards[0][2], shards[1][2]])
    ora = oracle_py.run(data, off, ids, shards[0][3])
    assert sorted(b"".join(texts).split(b"\n")) == sorted(ora["output_txt"].split(b"\n"))
    assert all(i["nterms_global"] == ora["nterms"] for i in infos)


def test_group_retry_is_collective(monkeypatch):
    """A 1024-slot starting vocabulary makes every rank grow its table and repeat the run;
    the repeats are agreed at the exchange (no rank re-enters the collectives alone)."""
    monkeypatch.setenv("TFIDF_VCAP", "1024")
    monkeypatch.setenv("TFIDF_VLOAD", "50")
    shards = _shards("c2", 0.003, 3)
    ora = _full("c2", 0.003)
    texts, res, infos = _run_group(shards, 3)
    assert b"".join(texts) == ora["output_txt"]
    assert all(i["vocab_capacity"] > 1024 for i in infos)


def test_group_one_rank_retries_alone(monkeypatch):
    """Only one rank's shard outgrows the starting table: the others repeat with it."""
    monkeypatch.setenv("TFIDF_VCAP", "4096")
    monkeypatch.setenv("TFIDF_VLOAD", "50")
    big = _shards("c2", 0.003, 1)[0]
    tiny_doc = (np.frombuffer(b"a b c\n", dtype=np.uint8).copy(), np.array([0, 6], dtype=np.uint64),
                np.array([int(big[2].max()) + 1], dtype=np.uint32))
    N = len(big[2]) + 1
    shards = [(big[0], big[1], big[2], N), (tiny_doc[0], tiny_doc[1], tiny_doc[2], N)]
    texts, res, infos = _run_group(shards, 2)
    # oracle over the same two shards as one corpus ("doc301@" is not after every id of
    # shard 0 in strcmp order, so the lines are compared as sorted sets)
    data = np.concatenate([big[0], tiny_doc[0]])
    off = np.concatenate([big[1], big[1][-1] + tiny_doc[1][1:]])
    ids = np.concatenate([big[2], tiny_doc[2]])
    ora = oracle_py.run(data, off, ids, N)
    assert sorted(b"".join(texts).split(b"\n")) == sorted(ora["output_txt"].split(b"\n"))
    # rank 0 grew its table; rank 1 repeated the run with it, at its own size
    assert infos[0]["vocab_capacity"] > 4096 and infos[1]["vocab_capacity"] == 4096


def test_group_empty_shard():
    """A shard with no documents still takes part in the exchange (V = 0)."""
    full = _shards("c2", 0.002, 1)[0]
    N = len(full[2])
    empty = (np.zeros(0, np.uint8), np.zeros(1, np.uint64), np.zeros(0, np.uint32), N)
    texts, res, infos = _run_group([full, empty], 2)
    ora = oracle_py.run(full[0], full[1], full[2], N)
    assert b"".join(texts) == ora["output_txt"]
    assert infos[1]["npairs"] == 0 and infos[0]["nterms_global"] == ora["nterms"]


def test_group_error_releases_peers():
    """A rank whose corpus is invalid fails; its peer returns TFIDF_E_PEER instead of
    waiting in the exchange."""
    full = _shards("c2", 0.001, 1)[0]
    bad = (full[0], full[1][:-1] * 0 + np.uint64(1 << 40), full[2][:-1], len(full[2]))   # offsets past the bytes
    with tfidf_abi.Group(2, devices=[0, 0]) as g:
        with pytest.raises(tfidf_abi.TfidfError) as ei:
            g.run_host([full, bad])
        assert ei.value.rc == -1   # rank 1's own error is reported first... (rank 0 is E_PEER)
        # the group is usable again afterwards
        g.run_host(_shards("c2", 0.001, 2))


@pytest.mark.parametrize("xchg", ["dense", "owner"])
@pytest.mark.parametrize("failing", [0, 1, 2])
def test_exchange_failure_after_allgather_aborts_peers(failing, xchg, monkeypatch):
    """A rank-local failure INSIDE the exchange (after the per-owner count all-gather, past
    the agreement: TFIDF_TEST_XFAIL_RANK) aborts the transport; the peers, already on their
    way into the next collective, return TFIDF_E_PEER instead of waiting, the group reports the
    failing rank's own error, and the next run of the group starts afresh (the in-process
    hub is reset).  The same engine path (exchange_df -> Xport::abort) aborts every RCCL
    communicator of a clique."""
    shards = _shards("c2", 0.001, 3)
    monkeypatch.setenv("TFIDF_XCHG", xchg)
    monkeypatch.setenv("TFIDF_TEST_XFAIL_RANK", str(failing))   # read by tfidf_open; fires once
    with tfidf_abi.Group(3, devices=[0, 0, 0]) as g:
        with pytest.raises(tfidf_abi.TfidfError) as ei:
            g.run_host(shards)
        assert ei.value.rc == -3   # TFIDF_E_HIP, the failing rank's own error (the others: E_PEER)
        g.run_host(shards)         # the same group again: the hub's poison was reset
        ora = _full("c2", 0.001)
        assert b"".join(g.ranks[r].text() for r in range(3)) == ora["output_txt"]


def test_failed_run_then_other_n_gets_its_own_idf_table(monkeypatch):
    """A run that fails inside the exchange may leave its idf-table upload (stream3, queued
    before the exchange) in flight.  The next run of the same contexts has another document
    count N, so its idf table differs in every entry: a stale upload landing after the new
    one, or a rewrite of the pinned table under the old copy, would change its scores.  The
    second run must match the oracle byte for byte (engine.cpp idf_pin_quiesce)."""
    monkeypatch.setenv("TFIDF_XCHG", "dense")
    monkeypatch.setenv("TFIDF_TEST_XFAIL_RANK", "1")   # read by tfidf_open; fires once
    first = _shards("c2", 0.002, 2)
    second = _shards("c2", 0.0013, 2)
    with tfidf_abi.Group(2, devices=[0, 0]) as g:
        with pytest.raises(tfidf_abi.TfidfError):
            g.run_host(first)
        g.run_host(second)
        ora = _full("c2", 0.0013)
        assert b"".join(g.ranks[r].text() for r in range(2)) == ora["output_txt"]
        g.run_host(first)
        assert b"".join(g.ranks[r].text() for r in range(2)) == _full("c2", 0.002)["output_txt"]


@pytest.mark.parametrize("xchg", ["dense", "owner"])
@pytest.mark.parametrize("failing", [0, 2])
def test_exchange_agreed_alloc_failure_keeps_group_usable(failing, xchg, monkeypatch):
    """A receive-side allocation failure inside the exchange is agreed between the ranks
    (TFIDF_TEST_XNOMEM_RANK): every rank returns an error before the (key, df) all-to-all,
    the transport is NOT aborted (tfidf.h: an agreed failure needs no action from the
    caller), and the next run of the same group succeeds with the oracle's output."""
    shards = _shards("c2", 0.001, 3)
    monkeypatch.setenv("TFIDF_XCHG", xchg)
    monkeypatch.setenv("TFIDF_TEST_XNOMEM_RANK", str(failing))   # read by tfidf_open; fires once
    with tfidf_abi.Group(3, devices=[0, 0, 0]) as g:
        with pytest.raises(tfidf_abi.TfidfError) as ei:
            g.run_host(shards)
        assert ei.value.rc == -2   # TFIDF_E_NOMEM, the failing rank's own error (the others: E_PEER)
        g.run_host(shards)
        ora = _full("c2", 0.001)
        assert b"".join(g.ranks[r].text() for r in range(3)) == ora["output_txt"]


def test_dense_prealloc_failure_falls_back_to_owner_form(monkeypatch):
    """Auto form: one rank cannot allocate the dense form's buffers (TFIDF_TEST_XNOMEM_RANK
    fires at their pre-allocation).  The failure travels as a flag of the first agreement,
    every rank takes the hash-owner form instead (which sizes its own buffers), and the run
    succeeds with the oracle's output — the group does not fail with NOMEM."""
    shards = _shards("c2", 0.001, 3)
    monkeypatch.delenv("TFIDF_XCHG", raising=False)
    monkeypatch.setenv("TFIDF_TEST_XNOMEM_RANK", "1")
    with tfidf_abi.Group(3, devices=[0, 0, 0]) as g:
        g.run_host(shards)
        assert not (g.ranks[0].info()["flags"] & tfidf_abi.RUN_XCHG_DENSE)
        ora = _full("c2", 0.001)
        assert b"".join(g.ranks[r].text() for r in range(3)) == ora["output_txt"]
        g.run_host(shards)   # the next run: every rank allocates, the dense form again
        assert g.ranks[0].info()["flags"] & tfidf_abi.RUN_XCHG_DENSE
        assert b"".join(g.ranks[r].text() for r in range(3)) == ora["output_txt"]


@pytest.mark.parametrize("xchg", ["dense", "owner"])
def test_rccl_single_rank_runs_the_exchange(xchg, monkeypatch):
    """A 1-rank RCCL communicator: exchange_df runs (agreement; dense: the key ncclAllGather
    and the DF ncclAllReduce; owner: the count ncclAllGather, the self all-to-alls by
    ncclSend / ncclRecv, the owner aggregation) and the results are unchanged."""
    monkeypatch.setenv("TFIDF_XCHG", xchg)
    p = tfidf_configs.plan("c2", scale=0.002)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    with tfidf_abi.Engine(0) as e:
        e.comm_init(tfidf_abi.comm_unique_id(), 0, 1)
        e.run_host(data, off, p["doc_ids"], p["ndocs_total"])
        res = e.fetch()
        assert e.info()["nterms_global"] == res["nterms"]
        e.run_host(data, off, p["doc_ids"], p["ndocs_total"])   # repeat on the same communicator
        assert e.fetch()["output_txt"] == res["output_txt"]
    assert_same_result(res, oracle_py.run(data, off, p["doc_ids"], p["ndocs_total"]))


def test_rccl_group_one_gpu():
    """tfidf_group_open with one rank on its own GPU builds an RCCL clique (ncclCommInitAll)."""
    shards = _shards("c5", 0.0005, 1)
    ora = _full("c5", 0.0005)
    with tfidf_abi.Group(1, devices=[0]) as g:
        g.run_host(shards)
        assert g.ranks[0].text() == ora["output_txt"]


@pytest.mark.parametrize("case", ["g2_twelve_docs", "g5_w1", "g5_w3", "g3_bytes"])
@pytest.mark.parametrize("shards", [1, 2, 3])
def test_cli_shards_drop_in(case, shards):
    """`tfidf --gpus 1 --shards K`: byte-balanced shards of input/ on one GPU, the same
    output.txt as the reference for every K (as the reference's is for every -np), and
    the --debug-jobs lines, split into their blocks and sorted, equal tf_jobs.txt /
    idf_jobs.txt."""
    g = load_golden(case)
    with tempfile.TemporaryDirectory() as td:
        shutil.copytree(os.path.join(GOLDEN, case, "input"), os.path.join(td, "input"))
        p = subprocess.run([tfidf_abi.CLI_PATH, "--gpus", "1", "--shards", str(shards), "--debug-jobs"], cwd=td,
                           capture_output=True, timeout=120)
        assert p.returncode == 0, p.stderr
        with open(os.path.join(td, "output.txt"), "rb") as f:
            assert f.read() == g["output"]
    tf, idf = split_jobs(p.stdout)
    assert tf == g["tf_jobs"] and idf == g["idf_jobs"]


def split_jobs(stdout: bytes):
    """TF Job / IDF Job lines of the CLI's stdout (TFIDF.c:200-204,237-239), each block
    kind sorted (the reference interleaves ranks, so only the sorted sets compare)."""
    tf, idf, cur = [], [], None
    for line in stdout.split(b"\n"):
        if line == b"-------------TF Job-------------":
            cur = tf
        elif line == b"------------IDF Job-------------":
            cur = idf
        elif line and cur is not None:
            cur.append(line)
    return b"".join(x + b"\n" for x in sorted(tf)), b"".join(x + b"\n" for x in sorted(idf))


def test_c3_sharded_over_8_equals_single_rank_oracle():
    """BASELINE config 3's shape (Zipf V = 5e4, ~4 KB documents) sharded over 8 ranks as the
    8-GPU run shards it (byte-balanced, docN@-ordered), at 5000 documents: the 8 shards'
    texts concatenated are the single-rank oracle's output.txt byte for byte."""
    K = 8
    shards = _shards("c3", 0.0005, K)
    ora = _full("c3", 0.0005)
    texts, res, infos = _run_group(shards, K)
    assert b"".join(texts) == ora["output_txt"]
    assert_same_result(_concat(res), ora)
    assert all(i["nterms_global"] == ora["nterms"] for i in infos)


def test_c3_sharded_over_8_properties():
    """Config 3 at 1e5 documents (~400 MB) over 8 shards, device-generated: the rank-order
    concatenation obeys the size-independent properties of the single-rank path — counts
    sum to the tokens, per-document sums = docSize, global DF = pairs per term across all
    shards, strict strcmp order across shard boundaries, scores recomputed with the global
    N (<= 1e-12 relative)."""
    K = 8
    with tfidf_abi.Group(K, devices=[0] * K) as g:
        plans = [tfidf_configs.plan("c3", scale=0.01, rank=r, nranks=K) for r in range(K)]
        corpora = [e.synth_device(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"], p["ndocs_total"])
                   for e, p in zip(g.ranks, plans)]
        g.run(corpora)
        infos = [e.info() for e in g.ranks]
        res = [e.fetch() for e in g.ranks]
    ntok = sum(int(p["ntok"].sum()) for p in plans)
    assert sum(i["ntokens"] for i in infos) == ntok
    cat = _concat(res)
    cnt = cat["count"].astype(np.int64)
    assert cnt.sum() == ntok and cat["npairs"] > 1_000_000
    starts = np.flatnonzero(np.r_[True, cat["doc"][1:] != cat["doc"][:-1]])
    assert np.array_equal(np.add.reduceat(cnt, starts), cat["docsize"][starts].astype(np.int64))
    # global DF: pairs per term over every shard
    dfc = np.bincount(cat["term"], minlength=len(cat["terms"]))
    assert np.array_equal(cat["df"], dfc[cat["term"]])
    assert all(i["nterms_global"] == len(cat["terms"]) for i in infos)
    # strict order across the concatenation: (document name key, term bytes)
    dk = tfidf_configs.doc_name_key(cat["doc"]).astype(np.uint64)
    tr = cat["term"]   # ids of the sorted union: byte order of the terms
    assert np.all((dk[1:] > dk[:-1]) | ((dk[1:] == dk[:-1]) & (tr[1:] > tr[:-1])))
    N = plans[0]["ndocs_total"]
    ref = (cnt / cat["docsize"].astype(np.float64)) * np.log(N / cat["df"].astype(np.float64))
    np.testing.assert_allclose(cat["score"], ref, rtol=1e-12, atol=1e-300)


_INIT_TIMEOUT_CHILD = r"""
import sys, time
sys.path.insert(0, sys.argv[1])
import tfidf_abi
with tfidf_abi.Engine(0) as e:
    t0 = time.time()
    try:
        e.comm_init(tfidf_abi.comm_unique_id(), 0, 2)   # rank 1 never joins
        print("RESULT joined")
    except tfidf_abi.TfidfError as ex:
        print("RESULT rc=%d after %.1f s" % (ex.rc, time.time() - t0))
"""


def test_rccl_init_peer_never_joins_times_out():
    """Process-per-GPU mode: rank 0 of a 2-rank job whose peer never calls tfidf_comm_init.
    The communicator is created non-blocking and polled (comm_rank.h), so the call gives up
    at TFIDF_COMM_TIMEOUT_S with TFIDF_E_PEER and aborts it, instead of blocking forever the
    way the reference's ranks wait for mpirun to kill them (TFIDF.c:122,137).  Run in a child
    process with its own time limit, so a regression fails this test instead of hanging."""
    import subprocess
    import sys
    env = dict(os.environ, TFIDF_COMM_TIMEOUT_S="3")
    pydir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "parallel-systems-mpi-tfidf_amd", "python")
    r = subprocess.run([sys.executable, "-c", _INIT_TIMEOUT_CHILD, pydir], env=env, capture_output=True,
                       text=True, timeout=90)
    out = [l for l in r.stdout.splitlines() if l.startswith("RESULT")]
    assert out, r.stdout + r.stderr
    assert out[0].startswith("RESULT rc=-11"), out[0]   # TFIDF_E_PEER
    secs = float(out[0].split("after ")[1].split(" ")[0])
    assert 2.5 <= secs < 30, out[0]


@pytest.mark.parametrize("xchg", ["dense", "owner"])
def test_rccl_clique_failure_releases_peers(xchg, monkeypatch):
    """An RCCL clique over distinct GPUs (skipped on a 1-GPU box): a rank-local failure
    inside the exchange (TFIDF_TEST_XFAIL_RANK, after the first collective) releases the peer
    waiting in the next collective: every rank aborts its own communicator at its next poll
    (comm_rank.h), the group reports the failing rank's error, and nobody hangs."""
    if tfidf_abi.device_count() < 2:
        pytest.skip("needs two GPUs for an RCCL clique")
    shards = _shards("c2", 0.001, 2)
    monkeypatch.setenv("TFIDF_XCHG", xchg)
    monkeypatch.setenv("TFIDF_TEST_XFAIL_RANK", "1")
    with tfidf_abi.Group(2, devices=[0, 1]) as g:
        with pytest.raises(tfidf_abi.TfidfError) as ei:
            g.run_host(shards)
        assert ei.value.rc == -3   # TFIDF_E_HIP from rank 1; rank 0 returned TFIDF_E_PEER
        with pytest.raises(tfidf_abi.TfidfError) as ei2:
            g.run_host(shards)     # the clique was aborted: unusable until reopened
        assert ei2.value.rc in (-11, -10)
