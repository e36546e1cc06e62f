"""Shared test helpers: golden fixture loading and result comparison."""
from __future__ import annotations

import json
import os

import numpy as np

from conftest import GOLDEN


def read_dir_corpus(input_dir: str):
    """Reference input contract (TFIDF.c:98-110,130-139): N = entries, docs doc1..docN."""
    names = [n for n in os.listdir(input_dir) if n not in (".", "..")]
    n = len(names)
    docs = []
    for i in range(1, n + 1):
        with open(os.path.join(input_dir, f"doc{i}"), "rb") as f:
            docs.append(f.read())
    return docs_to_arrays(docs)


def docs_to_arrays(docs):
    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in docs], dtype=np.uint64)
    data = np.frombuffer(b"".join(docs), dtype=np.uint8).copy()
    return data, off


def load_golden(case: str):
    d = os.path.join(GOLDEN, case)
    data, off = read_dir_corpus(os.path.join(d, "input"))
    with open(os.path.join(d, "output.txt"), "rb") as f:
        out = f.read()
    with open(os.path.join(d, "tf_jobs.txt"), "rb") as f:
        tf = f.read()
    with open(os.path.join(d, "idf_jobs.txt"), "rb") as f:
        idf = f.read()
    with open(os.path.join(d, "meta.json")) as f:
        meta = json.load(f)
    return dict(data=data, off=off, output=out, tf_jobs=tf, idf_jobs=idf, meta=meta)


def sorted_lines(b: bytes) -> bytes:
    lines = [x for x in b.split(b"\n") if x]
    return b"".join(x + b"\n" for x in sorted(lines))


def jobs_from_result(res: dict):
    """TF Job / IDF Job lines (TFIDF.c:204,239) rebuilt from a fetched GPU result."""
    terms = res["terms"]
    tf, idf = [], []
    N = res["ndocs_total"]
    for d, t, c, ds, df in zip(res["doc"].tolist(), res["term"].tolist(), res["count"].tolist(),
                               res["docsize"].tolist(), res["df"].tolist()):
        w = terms[t]
        tf.append(w + b"@doc%d\t%d/%d" % (d, c, ds))
        idf.append(w + b"@doc%d\t%d/%d" % (d, N, df))
    return b"".join(x + b"\n" for x in sorted(tf)), b"".join(x + b"\n" for x in sorted(idf))


def describe_diff(gpu: dict, ora: dict) -> str:
    """First document whose pairs differ, for the failure message."""
    def by_doc(r):
        out = {}
        for d, t, c, ds in zip(r["doc"].tolist(), r["term"].tolist(), r["count"].tolist(), r["docsize"].tolist()):
            out.setdefault(d, []).append((r["terms"][t], c, ds))
        return out
    g, o = by_doc(gpu), by_doc(ora)
    for d in sorted(set(g) | set(o)):
        if g.get(d) != o.get(d):
            gs, os_ = g.get(d, []), o.get(d, [])
            extra = sorted(set(gs) - set(os_))[:10]
            missing = sorted(set(os_) - set(gs))[:10]
            return (f"doc{d}: gpu {len(gs)} pairs, oracle {len(os_)}; gpu-only {extra}; oracle-only {missing}; "
                    f"docsize gpu {gs[0][2] if gs else None} oracle {os_[0][2] if os_ else None}")
    return "no per-document difference"


def assert_same_result(gpu: dict, ora: dict, exact_scores: bool = True):
    """Field-by-field parity: integers bit-exact, scores exact (or <= 1e-12 relative)."""
    assert gpu["npairs"] == ora["npairs"], describe_diff(gpu, ora)
    np.testing.assert_array_equal(gpu["doc"], ora["doc"])
    gterms = [gpu["terms"][t] for t in gpu["term"].tolist()]
    oterms = [ora["terms"][t] for t in ora["term"].tolist()]
    assert gterms == oterms
    np.testing.assert_array_equal(gpu["count"], ora["count"])
    np.testing.assert_array_equal(gpu["docsize"], ora["docsize"])
    np.testing.assert_array_equal(gpu["df"], ora["df"])
    if exact_scores:
        np.testing.assert_array_equal(gpu["score"].view(np.uint64), ora["score"].view(np.uint64))
    else:
        np.testing.assert_allclose(gpu["score"], ora["score"], rtol=1e-12, atol=0)
