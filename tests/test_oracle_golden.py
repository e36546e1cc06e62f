"""Pins the oracle (C restatement of TFIDF.c) to the reference program's own outputs.

Every fixture under tests/golden/ was produced by running oracle/_ref/TFIDF (built from
/root/reference/TFIDF.c) under MPICH mpirun (tests/golden/make_golden.py).  The
restatement must reproduce output.txt byte for byte and the TF/IDF Job lines as sets.
"""
import os
import subprocess
import tempfile
import shutil

import pytest

import oracle_py
from conftest import golden_cases, GOLDEN
from helpers import load_golden, sorted_lines


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
