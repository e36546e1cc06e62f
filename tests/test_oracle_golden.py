"""Pins the oracle (C restatement of TFIDF.c) to the reference program's own outputs.

Every fixture under tests/golden/ was produced by running oracle/_ref/TFIDF (built from
/root/reference/TFIDF.c) under MPICH mpirun (tests/golden/make_golden.py).  The
restatement must reproduce output.txt byte for byte and the TF/IDF Job lines as sets.
"""
import os
import subprocess
import tempfile
import shutil

import numpy as np
import pytest

import oracle_py
from conftest import golden_cases, GOLDEN
from helpers import check_full_properties, load_golden, sorted_lines


@pytest.mark.parametrize("case", golden_cases())
def test_oracle_matches_reference(case):
    g = load_golden(case)
    r = oracle_py.run(g["data"], g["off"], n_total=0)
    assert r["output_txt"] == g["output"]
    assert sorted_lines(r["tf_jobs"]) == g["tf_jobs"]
    assert sorted_lines(r["idf_jobs"]) == g["idf_jobs"]


@pytest.mark.parametrize("case", ["g1_whitespace", "g3_bytes", "g4_config1"])
def test_oracle_cli_process_contract(case):
    """The oracle CLI mirrors `mpirun -np 2 ./TFIDF` run inside the fixture directory."""
    oracle_py.build()
    with tempfile.TemporaryDirectory() as td:
        shutil.copytree(os.path.join(GOLDEN, case, "input"), os.path.join(td, "input"))
        p = subprocess.run([oracle_py.CLI], cwd=td, capture_output=True, timeout=60)
        assert p.returncode == 0
        with open(os.path.join(td, "output.txt"), "rb") as f:
            assert f.read() == load_golden(case)["output"]


def test_oracle_cli_errors():
    oracle_py.build()
    with tempfile.TemporaryDirectory() as td:
        p = subprocess.run([oracle_py.CLI], cwd=td, capture_output=True, timeout=60)
        assert p.returncode == 1 and p.stdout == b"Directory failed to open\n"     # TFIDF.c:100-103
        os.makedirs(os.path.join(td, "input"))
        with open(os.path.join(td, "input", "doc2"), "wb") as f:
            f.write(b"x")
        p = subprocess.run([oracle_py.CLI], cwd=td, capture_output=True, timeout=60)
        assert p.returncode == 0 and p.stdout.startswith(b"Error Opening File: input/doc1")  # TFIDF.c:134-138


def test_golden_fixture_inventory():
    cases = golden_cases()
    for need in ("g1_whitespace", "g2_twelve_docs", "g3_bytes", "g4_config1", "g6_common_word"):
        assert need in cases
    assert sum(c.startswith("g5_") for c in cases) >= 4
    g = load_golden("g4_config1")
    assert g["meta"]["npairs"] == 32 and g["meta"]["ndocs"] == 8


def test_sharded_cpu_baseline_equals_oracle():
    """oracle_run_sharded (bench.py's CPU baseline: threads per shard + DF combine +
    shard-order concatenation) produces the single-rank oracle's output.txt."""
    import numpy as np
    import tfidf_abi
    import tfidf_configs
    p = tfidf_configs.plan("c2", scale=0.002)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    ref = oracle_py.run(data, off, p["doc_ids"], p["ndocs_total"], arrays=False)["output_txt"]
    order = np.argsort(tfidf_configs.doc_name_key(p["doc_ids"]), kind="stable").astype(np.uint32)
    sizes = np.diff(off.astype(np.int64))[order]
    for k in (1, 3, 8):
        first = tfidf_configs.shard_cuts(sizes, k)
        txt, npairs = oracle_py.run_sharded(data, off, p["doc_ids"], p["ndocs_total"], order, first)
        assert txt == ref and npairs == ref.count(b"\n")


def _as_views(r: dict, doc_off, ids) -> dict:
    """the oracle's result in the layout of tfidf_abi.Engine.fetched()"""
    V = r["nterms"]
    order = sorted(range(V), key=lambda i: r["terms"][i] + b"\t")   # term ids in strcmp("word\t") order
    rank = np.zeros(V, dtype=np.uint32)
    rank[order] = np.arange(V, dtype=np.uint32)
    terms = [r["terms"][i] for i in order]
    pool = b"".join(terms)
    toff = np.zeros(V + 1, dtype=np.uint64)
    toff[1:] = np.cumsum([len(t) for t in terms])
    term = rank[r["term"]]
    sizes = np.zeros(len(ids), dtype=np.uint32)
    first = {}
    for i, d in enumerate(r["doc"].tolist()):
        first.setdefault(d, i)
    for k, d in enumerate(ids.tolist()):
        sizes[k] = r["docsize"][first[d]] if d in first else 0
    return dict(npairs=r["npairs"], nterms=V, ndocs=len(ids), ndocs_total=len(ids), doc=r["doc"], term=term,
                count=r["count"], docsize=r["docsize"], df=r["df"], score=r["score"], doc_id=ids, doc_size=sizes,
                term_df=np.bincount(term, minlength=V).astype(np.uint32), term_off=toff,
                term_bytes=np.frombuffer(pool, dtype=np.uint8))


def test_full_size_checker_on_oracle():
    """helpers.check_full_properties — the checker the full-size GPU tests (c2..c5 at
    BASELINE size) rely on — accepts the oracle's result at chunk sizes that split it into
    many document-aligned chunks, and rejects a changed count, a changed score and two
    documents out of order."""
    rng = np.random.default_rng(7)
    words = [b"w%d" % i for i in range(300)] + [b"x" * 20 + b"%d" % i for i in range(5)]
    docs = [b" ".join(words[j] for j in rng.integers(0, len(words), int(rng.integers(0, 60)))) for _ in range(120)]
    data = np.frombuffer(b"".join(docs), dtype=np.uint8)
    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs])
    ids = np.arange(1, len(docs) + 1, dtype=np.uint32)
    r = oracle_py.run(data, off)
    ntok = sum(len(d.split()) for d in docs)
    for chunk in (1, 37, 1 << 20):
        check_full_properties(_as_views(r, off, ids), ntok, threads=3, chunk=chunk)
    bad = _as_views(r, off, ids)
    bad["count"] = bad["count"].copy()
    bad["count"][5] += 1
    with pytest.raises(AssertionError):
        check_full_properties(bad, ntok, chunk=37)
    bad = _as_views(r, off, ids)
    bad["score"] = bad["score"].copy()
    bad["score"][11] *= 1 + 1e-9
    with pytest.raises(AssertionError):
        check_full_properties(bad, ntok, chunk=37)
    v = _as_views(r, off, ids)
    st = np.flatnonzero(np.r_[True, v["doc"][1:] != v["doc"][:-1]])
    a, b, c = int(st[3]), int(st[4]), int(st[5])   # swap documents 3 and 4 (whole runs)
    perm = np.r_[np.arange(a), np.arange(b, c), np.arange(a, b), np.arange(c, v["npairs"])]
    for k in ("doc", "term", "count", "docsize", "df", "score"):
        v[k] = v[k][perm]
    with pytest.raises(AssertionError):
        check_full_properties(v, ntok, chunk=37)
