"""GPU tests of the streaming ingest (tfidf_ingest_dir_device):
input/doc1..N read by host threads into pinned 8 MiB segments and copied to HBM with the
copies overlapping the reads.  The device corpus must be byte-identical to the files
(and to the host ingest tfidf_ingest_dir), the run on it must give the reference's
output.txt, and the error contract must follow TFIDF.c:98-110,130-138."""
import json
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

import tfidf_abi
import tfidf_configs
from conftest import golden_cases, GOLDEN
from helpers import load_golden

pytestmark = pytest.mark.gpu


def write_docs(d, docs):
    os.makedirs(d, exist_ok=True)
    for i, b in enumerate(docs, 1):
        with open(os.path.join(d, f"doc{i}"), "wb") as f:
            f.write(b)


@pytest.mark.parametrize("case", golden_cases())
def test_ingest_golden_dirs(engine, case):
    g = load_golden(case)
    c, info = engine.ingest_dir(os.path.join(GOLDEN, case, "input"))
    data, off = engine.corpus_bytes(c)
    assert np.array_equal(data, g["data"]) and np.array_equal(off, g["off"])
    assert info["ndocs"] == len(g["off"]) - 1 and info["nbytes"] == len(g["data"])
    engine.run_corpus(c)
    assert engine.fetch()["output_txt"] == g["output"]
    assert engine.text() == g["output"]


def test_ingest_multi_segment_ragged(engine):
    """~40 MB over 5 segments: documents straddling segment edges, one document larger than
    two segments, empty documents, 3 reader threads (so slots are reused)."""
    p = tfidf_configs.plan("c2", scale=0.03)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    docs = [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(len(off) - 1)]
    big = b"".join(docs[:2000])            # ~20 MB: spans three segments
    docs = docs[:5] + [b"", big, b""] + docs[5:]
    with tempfile.TemporaryDirectory() as td:
        d = os.path.join(td, "input")
        write_docs(d, docs)
        c, info = engine.ingest_dir(d, threads=3)
        assert info["segments"] >= 5 and info["threads"] == 3
        got, goff = engine.corpus_bytes(c)
    want = np.frombuffer(b"".join(docs), dtype=np.uint8)
    assert np.array_equal(got, want)
    assert np.array_equal(goff, np.concatenate([[0], np.cumsum([len(x) for x in docs])]).astype(np.uint64))
    engine.run_corpus(c)
    dev_txt = engine.fetch()["output_txt"]
    engine.run_host(want, goff)
    assert engine.fetch()["output_txt"] == dev_txt


def test_ingest_error_contract(engine):
    with tempfile.TemporaryDirectory() as td:
        with pytest.raises(tfidf_abi.TfidfError) as e:
            engine.ingest_dir(os.path.join(td, "nope"))
        assert e.value.rc == -6                       # TFIDF.c:100-103
        d = os.path.join(td, "input")
        write_docs(d, [b"a b", b"", b"c\n"])
        os.makedirs(os.path.join(d, ".hidden"))       # every entry counts in N (TFIDF.c:104-109)
        with pytest.raises(tfidf_abi.TfidfError) as e:
            engine.ingest_dir(d)
        assert e.value.rc == -7 and e.value.bad_doc == 4 and e.value.ndocs == 4   # TFIDF.c:134-138
        os.rmdir(os.path.join(d, ".hidden"))
        c, info = engine.ingest_dir(d)
        assert c.ndocs == 3 and c.nbytes == 5 and c.flags == tfidf_abi.TFIDF_CORPUS_DEVICE
        empty = os.path.join(td, "empty")
        os.makedirs(empty)
        c, info = engine.ingest_dir(empty)
        assert c.ndocs == 0 and c.nbytes == 0


def test_cli_streaming_ingest_stats():
    """The CLI on a multi-segment input/: output equals the engine's host-ingest run, and
    --stats reports the ingest and run times."""
    p = tfidf_configs.plan("c2", scale=0.01)
    data, off = tfidf_abi.synth_host(p["seed"], p["V"], p["mode"], p["cdf"], p["doc_ids"], p["ntok"])
    with tempfile.TemporaryDirectory() as td:
        write_docs(os.path.join(td, "input"), [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(len(off) - 1)])
        r = subprocess.run([tfidf_abi.CLI_PATH, "--stats"], cwd=td, capture_output=True, timeout=120)
        assert r.returncode == 0, r.stderr
        st = json.loads(r.stderr.decode().strip().splitlines()[-1])
        assert st["docs"] == len(off) - 1 and st["corpus_bytes"] == len(data)
        with open(os.path.join(td, "output.txt"), "rb") as f:
            cli_out = f.read()
    with tfidf_abi.Engine(0) as e:
        e.run_host(data, off)
        assert e.fetch()["output_txt"] == cli_out
