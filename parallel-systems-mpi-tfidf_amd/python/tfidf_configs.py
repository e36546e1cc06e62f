"""Synthetic Zipfian corpus plans for BASELINE.json's configs.

A plan fixes, per document, its global id ("docN") and token count, plus the Zipf CDF
table; the bytes themselves come from csrc/synth.h (host or device, byte-identical).

  c1  8 docs x 2000 tokens, 4 distinct words per doc from a 22-word vocabulary (seed 1):
      32 (doc, word) pairs, inside the reference's 32-pair capacity (TFIDF.c:16)
  c2  1e5 docs, V = 5e4, Zipf s = 1.07, lognormal(sigma 0.5) lengths, mean 10 KB -> ~1 GB
  c3  1e7 docs, V = 5e4, s = 1.07, mean 4 KB -> ~40 GB
  c4  1e5 docs, V = 1e7, s = 0.8, mean 10 KB (high-cardinality vocabulary)
  c5  4 docs x 100 MB at seeded ids + 1e6 docs x ~600 B, V = 5e4, s = 1.07 (skew)
`scale` shrinks N (and the big documents of c5) for tests.
"""
from __future__ import annotations

import numpy as np

MODE_ZIPF = 0
MODE_C1 = 1

CONFIGS = {
    "c1": dict(N=8, V=22, mode=MODE_C1, tokens=2000, seed=1),
    "c2": dict(N=100_000, V=50_000, s=1.07, mean_bytes=10_000, sigma=0.5, seed=2),
    "c3": dict(N=10_000_000, V=50_000, s=1.07, mean_bytes=4_000, sigma=0.5, seed=3),
    "c4": dict(N=100_000, V=10_000_000, s=0.8, mean_bytes=10_000, sigma=0.5, seed=4),
    "c5": dict(N=1_000_004, V=50_000, s=1.07, mean_bytes=600, sigma=0.5, seed=5, big=4, big_bytes=100_000_000),
}


def digits26(V: int) -> int:
    m, cap = 1, 26
    while cap < V:
        cap *= 26
        m += 1
    return m


def bytes_per_token(V: int) -> float:
    """mean term length (m + uniform{0..5}, clamped to [3, 12]) + one separator"""
    m = digits26(V)
    lens = [min(12, max(3, m + e)) for e in range(6)]
    return sum(lens) / 6.0 + 1.0


def zipf_cdf(V: int, s: float) -> np.ndarray:
    w = np.arange(1, V + 1, dtype=np.float64) ** (-s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    cdf[-1] = 1.0
    return cdf


def doc_name_key(ids: np.ndarray) -> np.ndarray:
    """strcmp order of "docN@" (TFIDF.c:245,273): digits right-padded with 10, base 11"""
    ids = np.asarray(ids, dtype=np.uint64)
    nd = np.ones(len(ids), dtype=np.int64)
    for k in range(1, 10):
        nd += (ids >= np.uint64(10 ** k)).astype(np.int64)
    key = np.zeros(len(ids), dtype=np.uint64)
    for p in range(10):
        # digit p (from the left) of each id, or 10 past its length
        shift = nd - 1 - p
        dig = np.where(shift >= 0, (ids // (10 ** np.maximum(shift, 0)).astype(np.uint64)) % 10, 10)
        key = key * np.uint64(11) + dig.astype(np.uint64)
    return key


def shard_cuts(weights, nshards: int) -> np.ndarray:
    """Balanced contiguous cut of a sequence (the rule of tfidf_shard_split in
    csrc/ingest.cpp): cut r is the prefix-sum position nearest to r * total / nshards, so
    every shard weighs at most total / nshards + the heaviest element."""
    w = np.asarray(weights, dtype=np.uint64)
    pre = np.zeros(len(w) + 1, dtype=np.uint64)
    pre[1:] = np.cumsum(w, dtype=np.uint64)
    total = int(pre[-1])
    first = np.zeros(nshards + 1, dtype=np.int64)
    for r in range(1, nshards):
        target = (total * r) // nshards
        i = int(np.searchsorted(pre, np.uint64(target), side="left"))
        i = min(i, len(w))
        if i > 0 and target - int(pre[i - 1]) < int(pre[i]) - target:
            i -= 1
        first[r] = max(i, first[r - 1])
    first[nshards] = len(w)
    return first


def plan(name: str, scale: float = 1.0, rank: int = 0, nranks: int = 1, weak: bool = False, vocab: int = 0):
    """Returns dict(doc_ids, ntok, cdf, V, mode, seed, ndocs_total).

    nranks > 1: documents are sharded in contiguous "docN" strcmp-order ranges, so the
    concatenation of the shards' outputs is the global output, balanced by bytes (SURVEY
    §8e; a document's bytes are its token count times the generator's bytes per token,
    so the cut is taken over token counts).  weak=True grows the corpus with nranks
    (fixed per-GPU work); otherwise (strong) the config's corpus is split.
    """
    cfg = dict(CONFIGS[name])
    seed = cfg["seed"]
    V = vocab or cfg["V"]   # vocab: diagnostic override of the vocabulary size
    if cfg.get("mode") == MODE_C1:
        N = cfg["N"] * (nranks if weak else 1)
        ids = np.arange(1, N + 1, dtype=np.uint32)
        ntok = np.full(N, cfg["tokens"], dtype=np.uint64)
        cdf = None
        mode = MODE_C1
    else:
        mode = MODE_ZIPF
        N = max(1, int(round(cfg["N"] * scale)))
        if weak:
            N *= nranks
        rng = np.random.Generator(np.random.PCG64(seed))
        mean_tok = cfg["mean_bytes"] / bytes_per_token(V)
        sig = cfg["sigma"]
        z = rng.standard_normal(N)
        ntok = np.maximum(1, np.rint(mean_tok * np.exp(sig * z - 0.5 * sig * sig))).astype(np.uint64)
        if cfg.get("big"):
            nb = cfg["big"]
            big_tok = int(cfg["big_bytes"] * scale / bytes_per_token(V))
            where = rng.choice(N, size=min(nb, N), replace=False)
            ntok[where] = max(1, big_tok)
        ids = np.arange(1, N + 1, dtype=np.uint32)
        cdf = zipf_cdf(V, cfg["s"])
    ndocs_total = len(ids)
    if nranks > 1:
        order = np.argsort(doc_name_key(ids), kind="stable")
        first = shard_cuts(ntok[order], nranks)
        sel = order[first[rank]:first[rank + 1]]
        ids, ntok = ids[sel], ntok[sel]
    return dict(doc_ids=ids, ntok=ntok, cdf=cdf, V=V, mode=mode, seed=seed, ndocs_total=ndocs_total)
