#!/usr/bin/env python3
"""Generates the golden fixtures under tests/golden/<case>/ by running the REFERENCE
program itself (oracle/_ref/TFIDF, compiled from /root/reference/TFIDF.c by
oracle/Makefile; oracle/_ref/TFIDF_w4096 is the "widened oracle" of SURVEY §8c) under
MPICH mpirun.  Run in the development container only (the reference, MPICH and this
script's outputs never need to exist on the GPU box; the fixtures are committed data).

Each fixture directory holds:
  input/docN        the corpus (inputs)
  output.txt        the reference's output.txt (TFIDF.c:274-282)
  tf_jobs.txt       sorted "word@docN\\twc/ds" lines of the TF Job blocks (TFIDF.c:199-205)
  idf_jobs.txt      sorted "word@docN\\tN/df" lines of the IDF Job blocks (TFIDF.c:236-239)
  meta.json         binary, -np, case description

Cases follow SURVEY §8c: G1 whitespace, G2 doc10 < doc1 ordering, G3 byte classes /
NUL truncation / empty doc, G4 config 1, G5 widened-oracle corpora at -np 2/4/5,
G6 a word in every document (score 0).
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "parallel-systems-mpi-tfidf_amd", "python"))
import tfidf_abi  # noqa: E402  (host synthetic generator only; no GPU)
import tfidf_configs  # noqa: E402

MPIRUN = "/opt/conda/bin/mpirun"
REF = os.path.join(REPO, "oracle", "_ref", "TFIDF")
REF_W = os.path.join(REPO, "oracle", "_ref", "TFIDF_w4096")


def run_reference(docs: list[bytes], np_: int, binary: str):
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, "input"))
        for i, d in enumerate(docs, 1):
            with open(os.path.join(td, "input", f"doc{i}"), "wb") as f:
                f.write(d)
        env = dict(os.environ, MPICH_CC="gcc", PATH="/opt/conda/bin:" + os.environ.get("PATH", ""))
        p = subprocess.run([MPIRUN, "-prepend-rank", "-np", str(np_), binary], cwd=td, env=env,
                           capture_output=True, timeout=120)
        if p.returncode != 0:
            raise RuntimeError(f"reference failed rc={p.returncode}: {p.stderr.decode(errors='replace')[:500]}")
        with open(os.path.join(td, "output.txt"), "rb") as f:
            out = f.read()
    tf, idf = [], []
    state = {}
    for line in p.stdout.split(b"\n"):
        if not line.startswith(b"["):
            continue
        rk, _, rest = line.partition(b"] ")
        if rest.startswith(b"-------------TF Job"):
            state[rk] = "tf"
            continue
        if rest.startswith(b"------------IDF Job"):
            state[rk] = "idf"
            continue
        (tf if state.get(rk) == "tf" else idf).append(rest)
    return out, sorted(tf), sorted(idf)


def write_case(name: str, docs: list[bytes], np_: int, binary: str, desc: str):
    d = os.path.join(HERE, name)
    if os.path.exists(d):
        shutil.rmtree(d)
    os.makedirs(os.path.join(d, "input"))
    for i, doc in enumerate(docs, 1):
        with open(os.path.join(d, "input", f"doc{i}"), "wb") as f:
            f.write(doc)
    out, tf, idf = run_reference(docs, np_, binary)
    with open(os.path.join(d, "output.txt"), "wb") as f:
        f.write(out)
    with open(os.path.join(d, "tf_jobs.txt"), "wb") as f:
        f.write(b"".join(x + b"\n" for x in tf))
    with open(os.path.join(d, "idf_jobs.txt"), "wb") as f:
        f.write(b"".join(x + b"\n" for x in idf))
    meta = dict(case=name, np=np_, binary=os.path.basename(binary), description=desc, ndocs=len(docs),
                npairs=out.count(b"\n"))
    with open(os.path.join(d, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{name}: {len(docs)} docs, {meta['npairs']} pairs, -np {np_}, {meta['binary']}")


def synth_docs(seed, V, mode, cdf, ntok):
    data, off = tfidf_abi.synth_host(seed, V, mode, cdf, None, ntok)
    return [bytes(data[int(off[i]):int(off[i + 1])]) for i in range(len(ntok))]


def main():
    if not (os.path.exists(REF) and os.path.exists(MPIRUN)):
        sys.exit("oracle/_ref/TFIDF or MPICH missing: run `make -C oracle ref` in the dev container")
    write_case("g1_whitespace", [
        b"hello world\thello\n",
        b"  world\t\tfoo\r\nfoo\vbar\fbaz  \n\n",
        b"x",
    ], 3, REF, "mixed C-locale whitespace, double separators, no trailing newline")
    docs = [b"alpha beta\n" if i % 2 else b"beta gamma gamma\n" for i in range(1, 13)]
    write_case("g2_twelve_docs", docs, 4, REF, "doc10..doc12 sort before doc1 (strcmp of 'docN@')")
    write_case("g3_bytes", [
        b"a\x01 a a\n",
        b"\xc2\xa0x x\n",
        b"ab\x00cd ab zz\n",
        b"",
        b"a\x01 zz\n",
    ], 3, REF, "a\\x01 vs a, NBSP is not whitespace, NUL truncates the term, empty doc counts in N")
    p = tfidf_configs.plan("c1")
    write_case("g4_config1", synth_docs(p["seed"], p["V"], p["mode"], None, p["ntok"]), 4, REF,
               "config 1: 8 docs x 2000 tokens, 4 distinct words per doc, 22-word vocabulary")
    write_case("g6_common_word", [b"the cat\n", b"the dog the\n", b"the\n", b"the end\n"], 2, REF,
               "a word in every document scores 0.0000000000000000")
    # widened oracle corpora (MAX_WORDS_IN_CORPUS 4096; valid while P <= ~3700)
    wide = [("g5_w1", 12, 300, 2000, 1.07, 11, 2), ("g5_w2", 8, 600, 1000, 1.0, 12, 4),
            ("g5_w3", 20, 150, 3000, 1.1, 13, 5), ("g5_w4", 5, 1000, 800, 0.9, 14, 4)]
    for name, N, T, V, s, seed, np_ in wide:
        cdf = tfidf_configs.zipf_cdf(V, s)
        rng = np.random.Generator(np.random.PCG64(seed))
        ntok = np.maximum(1, rng.integers(T // 2, T * 3 // 2, size=N)).astype(np.uint64)
        docs = synth_docs(seed, V, 0, cdf, ntok)
        write_case(name, docs, np_, REF_W, f"widened oracle: {N} docs ~{T} tokens, V={V}, zipf {s}")


if __name__ == "__main__":
    main()
