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


def _chunk_bounds(doc: np.ndarray, chunk: int):
    """pair ranges of about `chunk` pairs, each starting at a document's first pair"""
    P = len(doc)
    b = [0]
    for t in range(chunk, P, chunk):
        if t <= b[-1]:
            continue
        j, w = t, 1 << 16
        while j < P:
            seg = doc[j - 1:j + w]
            ch = np.flatnonzero(seg[1:] != seg[:-1])
            if len(ch):
                j += int(ch[0])
                break
            j += w
        if j < P:
            b.append(j)
    b.append(P)
    return b


def check_full_properties(r: dict, ntokens: int, threads: int = 8, chunk: int = 1 << 26):
    """Size-independent properties of a result (the views of Engine.fetched(), any size),
    checked in document-aligned chunks on a thread pool so that full-size configurations
    need no copy of the pairs:
      counts sum to the tokens; per document (a contiguous run of pairs): sum of counts =
      docSize (TFIDF.c:141-167), docSize as the run's documents report it; terms strictly
      increasing inside a document and documents strictly increasing in "docN@" strcmp
      order, each document one run (TFIDF.c:245,273); DF = pairs per term (TFIDF.c:169-234);
      score = count/docSize * log(N/df) within 1e-12 relative (TFIDF.c:202,243-244)."""
    from concurrent.futures import ThreadPoolExecutor
    import tfidf_configs
    P, V, N = r["npairs"], r["nterms"], r["ndocs_total"]
    doc, term, cnt, dsz, df, score, tdf = (r[k] for k in ("doc", "term", "count", "docsize", "df", "score", "term_df"))
    assert P > 0 and len(doc) == P
    bounds = _chunk_bounds(doc, chunk)

    def one(i):
        a, b = bounds[i], bounds[i + 1]
        d, t, c = doc[a:b], term[a:b], cnt[a:b].astype(np.int64)
        st = np.flatnonzero(np.r_[True, d[1:] != d[:-1]])
        assert np.array_equal(np.add.reduceat(c, st), dsz[a:b][st].astype(np.int64)), "per-document sums"
        same = d[1:] == d[:-1]
        assert np.all(~same | (t[1:] > t[:-1])), "term order inside a document"
        assert np.all(~same | (dsz[a + 1:b] == dsz[a:b - 1])), "docSize constant inside a document"
        assert np.array_equal(df[a:b], tdf[t]), "df = the term's df"
        ds = dsz[a:b].astype(np.float64)
        ref = (c / ds) * np.log(N / df[a:b].astype(np.float64))
        err = np.abs(score[a:b] - ref)
        assert np.all(err <= 1e-12 * np.abs(ref) + 1e-300), "scores"
        return int(c.sum()), np.bincount(t, minlength=V), d[st].copy(), dsz[a:b][st].copy()

    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(one, range(len(bounds) - 1)))
    assert sum(p[0] for p in parts) == ntokens
    dfc = np.zeros(V, dtype=np.int64)
    for p in parts:
        dfc += p[1]
    assert np.array_equal(dfc, tdf.astype(np.int64)), "DF = pairs per term"
    runs = np.concatenate([p[2] for p in parts])
    run_ds = np.concatenate([p[3] for p in parts])
    key = tfidf_configs.doc_name_key(runs)
    assert np.all(key[1:] > key[:-1]), "documents strictly increasing, one run each"
    # the run's docSize is the document's (tfidf_result doc_id/doc_size); empty documents have no run
    ids, sizes = r["doc_id"], r["doc_size"]
    o = np.argsort(ids, kind="stable")
    pos = np.searchsorted(ids[o], runs)
    assert np.array_equal(ids[o][pos], runs) and np.array_equal(sizes[o][pos], run_ds)
    assert int(sizes.astype(np.int64).sum()) == ntokens
    # term table in strcmp("word\t") order
    toff, tb = r["term_off"], r["term_bytes"]
    step = max(1, V // 200_000)
    for i in range(0, V - 1, step):
        x = bytes(tb[int(toff[i]):int(toff[i + 1])]) + b"\t"
        y = bytes(tb[int(toff[i + 1]):int(toff[i + 2])]) + b"\t"
        assert x < y, (i, x, y)
