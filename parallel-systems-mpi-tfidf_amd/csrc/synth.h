/*
 * synth.h — deterministic synthetic Zipfian corpus generator.
 *
 * One definition, compiled both by gcc (host generation: fixtures, CPU baseline
 * samples) and by hipcc (device generation straight into HBM for bench.py), so the
 * two produce byte-identical corpora from the same inputs.
 *
 * Floating point never enters the byte stream: per-document token counts and the
 * Zipf CDF table are computed by the caller (numpy) and passed in; the generator
 * only does integer splitmix64 arithmetic, exact double compares against the CDF
 * table, and table lookups.
 *
 * Corpus shape:
 *   - term t has a unique lowercase string of 3..12 bytes: (L-m) hash-derived filler
 *     letters followed by the m-digit base-26 spelling of t (m = digits needed for V),
 *     so the last m letters identify t and strings are unique by construction;
 *   - zipf mode: token rank drawn from the CDF by inverse transform, mapped to a term
 *     through the bijection term = (rank * perm_a + perm_b) mod V;
 *   - c1 mode: each document draws uniformly from 4 fixed distinct words
 *     (config 1: 8 docs x 2000 tokens -> 32 (doc, word) pairs, reference-safe);
 *   - separators: ' ' after each token, '\n' after every 12th token and after the
 *     last token of a document.
 *   - tokens are generated in blocks of SYN_BLOCK_TOKENS with an independent
 *     splitmix64 stream per (doc, block), so a 100 MB document generates in parallel.
 */
#ifndef TFIDF_SYNTH_H
#define TFIDF_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define SYN_HD __host__ __device__ __forceinline__
#else
#define SYN_HD static inline
#endif

#define SYN_BLOCK_TOKENS 1024u
#define SYN_MODE_ZIPF 0u
#define SYN_MODE_C1 1u

typedef struct syn_spec {
    uint64_t seed;
    uint32_t V;        /* vocabulary size (terms 0..V-1) */
    uint32_t m;        /* base-26 digits identifying a term */
    uint64_t perm_a;   /* rank -> term bijection, gcd(perm_a, V) == 1 */
    uint64_t perm_b;
    uint32_t mode;     /* SYN_MODE_ZIPF / SYN_MODE_C1 */
    uint32_t pad_;
    const double* cdf; /* zipf mode: V entries, non-decreasing, cdf[V-1] == 1.0 */
} syn_spec;

SYN_HD uint64_t syn_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* splitmix64 stream for (seed, doc, block) */
SYN_HD uint64_t syn_stream_seed(uint64_t seed, uint64_t doc_id, uint64_t block) {
    return syn_mix64(seed ^ syn_mix64(doc_id * 0x2545F4914F6CDD1Dull + 0x1234567ull)) ^
           syn_mix64(block + 0xABCDEF01ull);
}

SYN_HD uint64_t syn_next(uint64_t* s) {
    *s += 0x9E3779B97F4A7C15ull;
    uint64_t z = *s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

SYN_HD uint32_t syn_digits26(uint32_t V) {
    uint32_t m = 1;
    uint64_t cap = 26;
    while (cap < (uint64_t)V) { cap *= 26; ++m; }
    return m;
}

SYN_HD uint32_t syn_term_len(const syn_spec* s, uint32_t t) {
    uint64_t h = syn_mix64(s->seed ^ 0x7E57000000000000ull ^ (uint64_t)t);
    uint32_t L = s->m + (uint32_t)(h % 6u);
    if (L < 3u) L = 3u;
    if (L > 12u) L = 12u;
    return L;
}

/* writes syn_term_len(s,t) bytes */
SYN_HD void syn_term_bytes(const syn_spec* s, uint32_t t, uint8_t* out) {
    uint32_t L = syn_term_len(s, t);
    uint32_t fill = L - s->m;
    uint64_t h = syn_mix64(s->seed ^ 0xF111000000000000ull ^ (uint64_t)t);
    for (uint32_t i = 0; i < fill; ++i) {
        out[i] = (uint8_t)('a' + (uint32_t)(h % 26u));
        h = h / 26u ^ (h << 59);
    }
    uint32_t v = t;
    for (uint32_t i = 0; i < s->m; ++i) {
        out[L - 1u - i] = (uint8_t)('a' + v % 26u);
        v /= 26u;
    }
}

/* term of the next token of document doc_id (1-based) */
SYN_HD uint32_t syn_draw(const syn_spec* s, uint64_t* rng, uint64_t doc_id) {
    uint64_t x = syn_next(rng);
    if (s->mode == SYN_MODE_C1) {
        uint32_t j = (uint32_t)(x % 4u);
        return (uint32_t)((doc_id * 3u + (uint64_t)j * 5u) % s->V);
    }
    double u = (double)(x >> 11) * (1.0 / 9007199254740992.0);
    uint32_t lo = 0, hi = s->V - 1u; /* first k with cdf[k] > u */
    while (lo < hi) {
        uint32_t mid = lo + ((hi - lo) >> 1);
        if (s->cdf[mid] > u) hi = mid; else lo = mid + 1u;
    }
    return (uint32_t)(((uint64_t)lo * s->perm_a + s->perm_b) % s->V);
}

SYN_HD uint8_t syn_sep(uint64_t tok_idx, uint64_t ntok) {
    return (tok_idx + 1u == ntok || ((tok_idx + 1u) % 12u) == 0u) ? (uint8_t)'\n' : (uint8_t)' ';
}

/* bytes produced by block `b` of a document with `ntok` tokens */
SYN_HD uint64_t syn_block_bytes(const syn_spec* s, uint64_t doc_id, uint64_t ntok, uint64_t b) {
    uint64_t t0 = b * SYN_BLOCK_TOKENS;
    uint64_t t1 = t0 + SYN_BLOCK_TOKENS;
    if (t1 > ntok) t1 = ntok;
    uint64_t rng = syn_stream_seed(s->seed, doc_id, b);
    uint64_t n = 0;
    for (uint64_t i = t0; i < t1; ++i) n += syn_term_len(s, syn_draw(s, &rng, doc_id)) + 1u;
    return n;
}

/* writes block `b` of the document at out; returns syn_block_bytes() */
SYN_HD uint64_t syn_block_fill(const syn_spec* s, uint64_t doc_id, uint64_t ntok, uint64_t b, uint8_t* out) {
    uint64_t t0 = b * SYN_BLOCK_TOKENS;
    uint64_t t1 = t0 + SYN_BLOCK_TOKENS;
    if (t1 > ntok) t1 = ntok;
    uint64_t rng = syn_stream_seed(s->seed, doc_id, b);
    uint64_t n = 0;
    for (uint64_t i = t0; i < t1; ++i) {
        uint32_t t = syn_draw(s, &rng, doc_id);
        uint32_t L = syn_term_len(s, t);
        syn_term_bytes(s, t, out + n);
        out[n + L] = syn_sep(i, ntok);
        n += L + 1u;
    }
    return n;
}

#endif /* TFIDF_SYNTH_H */
