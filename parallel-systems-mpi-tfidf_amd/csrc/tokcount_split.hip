/*
 * tokcount_split.hip — K1 as two kernels: K1a resolves every token to its vocabulary slot,
 * K1b counts the (document, slot) pairs.  Together they replace the reference's per-rank hot
 * loop TFIDF.c:130-196: fscanf("%s") tokenising (:141-147), the strcmp search/append of
 * (word, doc) records (:151-167) and the per-rank word table (:169-188).
 *
 * Why split.  The fused kernel (tokcount_st.hip) holds the walk state, the token rounds and
 * the LDS count table in one wave: 128 VGPRs plus 131 SGPR spills (every spill a VALU
 * v_writelane/v_readlane), 16 waves per CU, a workgroup barrier per chunk.  Split, each
 * kernel keeps only its own state:
 *
 *   K1a k_tok_resolve  one WAVE per chunk (no workgroup barrier anywhere): the LDS-staged
 *        walk of tokcount_st (SWAR isspace per 16-byte group, document starts, one 32-bit
 *        token entry per token), then rounds of 64 tokens: the exact 128-bit identity key
 *        by one unaligned ds_read_b128 + four v_perm, the vocabulary hash, two adjacent
 *        slots loaded in one go, the lock-free insert on a miss.  Each token's slot goes to
 *        a token stream in corpus order: 4 bytes per token, written as 256-byte rows.
 *        Tokens of one chunk occupy [tbase(c), tbase(c) + ntok(c)) where
 *          tbase(c) = (chunk_start[c] - lo) / 2 + chunk_doc[c] + 4c
 *        (a chunk of B bytes holding D document starts has at most B/2 + D + 1 tokens: every
 *        token that is not at a document start follows a whitespace byte of its own), and
 *        the word is  (document ordinal in the chunk mod G) << sb | slot.  The k-th
 *        document of the chunk that has tokens gets dlist[lb + k] = its index and
 *        dtok[lb + k] = the chunk index of its first token (lb = chunk_doc[c] + c).
 *
 *   K1b k_count_slots  one workgroup per chunk: the stream rows of a group of G documents
 *        are counted in the bucketed LDS table of tokcount_st (4 u32 keys + counts per
 *        bucket, ONE ds_read_b128 per probe), 256 tokens per wave and dwordx4 load, then
 *        flushed as records exactly like tokcount_st (complete documents to the record
 *        stream, split or overflowing ones to the partial stream for K2).  docSize is the
 *        distance between consecutive dtok entries.
 *
 * The stream costs 8 bytes per token of HBM traffic (c2: 1.06 GB) and C/2 words of space.
 *
 * Measured on c2 (round 2, profiles/r02_s1_*), bit-exact with the oracle and the fused
 * kernel (tests: test_k1_variants_agree, the goldens), but SLOWER: K1a 3.1 ms + K1b 1.6 ms
 * against tokcount_st's 2.2 ms, so it is opt-in (TFIDF_K1=split).  What it showed:
 *   - K1a issues 4.3e8 VALU wave-instructions per launch (tokcount_st: 9.95e8 for walk +
 *     resolve + count), i.e. the resolve half does halve the per-token instruction count;
 *   - its waves wait 85 % of their cycles, and the walk alone (timing build K1A_ABL=24) takes
 *     2.46 ms at 20 waves/CU but 1.15 ms at 4 waves/CU: ~5000 independent 16 KiB chunk
 *     streams in flight (one per wave) read the corpus far slower than tokcount_st's ~1000
 *     (four waves per chunk) — the cost is the number of concurrent streams, not the work;
 *   - K1b issues another 4.3e8 VALU and keeps a ~17 us fixed cost per chunk (0.95 ms with a
 *     single key per chunk) with the next chunk's metadata, ordinals, bounds and first row
 *     all prefetched; one record-allocation atomic per chunk on a single counter remains.
 * A faster split needs the four waves of a workgroup on one chunk (ordinals across waves)
 * and batched record allocation; see DESIGN.md §8.
 */
#include "dev_common.h"
#include "dev_vocab.h"
#include "kernels.h"

namespace {

/* ------------------------------------------------------------------ K1a ---------- */

#ifndef K1A_WGCU
#define K1A_WGCU 8                        /* workgroups of 4 waves per CU requested */
#endif
#ifndef K1A_WAVES_PER_SIMD
#define K1A_WAVES_PER_SIMD 5              /* launch bound: <= 96 VGPRs */
#endif
/* timing-only ablations (make variant NAME=a1 DEFS=-DK1A_ABL=1; results invalid): 1 no
 * vocabulary gathers (every short key hits its home slot), 2 no token rounds (walk + entries
 * only), 4 no stream/ordinal stores, 8 no token entries (walk only), 16 no rare pass (misses
 * dropped: no call, no scratch) */
#ifndef K1A_ABL
#define K1A_ABL 0
#endif
constexpr int A_NT = 256;
constexpr int A_NW = A_NT / 64;
constexpr int WSTEP = 992;                /* bytes a wave step owns: lanes 1..62 (lane 0: the 16
                                             bytes before, lane 63: the 16 after) */
constexpr int TLW = 1024;                 /* token entries per wave: a whole step (<= 992 tokens) */
constexpr uint32_t LEN_LONG = 31u;
constexpr uint32_t GA = 63;               /* documents per walk group: lane k holds doc_off[gd0 + k] */
constexpr uint32_t TOK_NONE = 0xFFFFFFFFu;

struct AShared {
    uint4 stage[A_NW][64];                /* the step's 64 groups: [sb - 16, sb + 1008) */
    uint32_t tl[A_NW][TLW];
    uint16_t ml[A_NW][TLW];               /* the step's tokens left to the rare pass */
    uint4 sel[16];                        /* v_perm selectors of a term of length n */
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));

__device__ __forceinline__ uint4 ld16c(const uint8_t* __restrict__ bytes, uint64_t last_blk, uint64_t pos) {
    const uint64_t p = pos < last_blk ? pos : last_blk;
    const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(bytes + p));
    return make_uint4(r.x, r.y, r.z, r.w);
}

__device__ __forceinline__ uint32_t bounds_ws(uint64_t pos, uint64_t lo, uint64_t hi) {
    const uint32_t a = pos < lo ? (uint32_t)min(lo - pos, (uint64_t)16) : 0u;
    const uint32_t b = hi > pos ? (uint32_t)min(hi - pos, (uint64_t)16) : 0u;
    const uint32_t in = b > a ? (((1u << b) - 1u) & ~((1u << a) - 1u)) : 0u;
    return ~in & 0xFFFFu;
}

__device__ __forceinline__ uint32_t zero_bits(uint32_t x) { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u; }
__device__ __forceinline__ uint32_t compress4(uint32_t m) {
    m >>= 7;
    m |= m >> 7;
    m |= m >> 14;
    return m & 0xFu;
}

__device__ __forceinline__ uint32_t perm_sel(uint32_t n, uint32_t k) {
    uint32_t s = 0;
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t p = 4 * k + j;
        const uint32_t b = p < n ? j : (p == n ? 4u : 12u);
        s |= b << (8 * j);
    }
    return s;
}

__device__ __forceinline__ uint32_t ufirst(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t ufirst64(uint64_t x) {
    return ((uint64_t)ufirst((uint32_t)(x >> 32)) << 32) | ufirst((uint32_t)x);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t x, uint32_t k) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), (int)k) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)k);
}
__device__ __forceinline__ uint32_t lane_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

/* The next chunk of the 8 sharded counters (tokcount_st.hip: one device counter saturates
 * at ~88 claims/us); wave-uniform, lane 0 issues the atomics.  Returns n when none is left. */
__device__ __forceinline__ uint64_t claim_chunk_w(unsigned long long* ctr, uint32_t& sh, uint64_t n) {
    const int lane = threadIdx.x & 63;
    for (int t = 0; t < 8; ++t) {
        const uint64_t lo = n * sh / 8, hi = n * (sh + 1) / 8;
        if (hi > lo) {
            unsigned long long v = 0;
            if (lane == 0) v = atomicAdd(&ctr[sh], 1ull);
            v = ufirst64(v);
            if (lo + v < hi) return lo + v;
        }
        sh = (sh + 1) & 7u;
    }
    return n;
}

/* slot of a token whose term is >= 16 bytes (or runs past the 32-byte window): re-read from
 * HBM (rare for text); same keys as tokcount_st.hip */
__device__ __forceinline__ uint32_t slow_slot_a(const uint8_t* __restrict__ bytes, const VocabDev& v, uint64_t p0,
                                             uint64_t dend, uint32_t* status) {
    uint64_t p = p0;
    while (p < dend && !is_ws(bytes[p])) ++p;
    uint64_t n = 0;
    while (p0 + n < p && bytes[p0 + n] != 0) ++n;
    uint64_t klo, khi;
    if (n < 16) {
        uint64_t lo = 0, hi = 0;
        for (uint32_t k = 0; k < n; ++k) {
            const uint64_t b = bytes[p0 + k];
            if (k < 8) lo |= b << (8 * k); else hi |= b << (8 * (k - 8));
        }
        make_short_key(lo, hi, (uint32_t)n, &klo, &khi);
        return vocab_insert(v, klo, khi, 0, status);
    }
    make_long_key(bytes + p0, n, &klo, &khi);
    if (n >= 0xFFFFFFull) atomicOr(status, ST_TERM_LONG);
    const uint64_t rep = ((n < 0xFFFFFFull ? n : 0xFFFFFFull) << 40) | p0;
    return vocab_insert(v, klo, khi, rep, status);
}

/* The rare pass of a K1a step, out of line so that the walk and the rounds carry no insert
 * code (inlined, vocab_insert and the long-term path cost ~100 spilled VGPRs): every token
 * queued in ml (a new term, a key displaced past the two loaded slots, a term of >= 16
 * bytes) is inserted / looked up and its stream word written.  p0 = corpus offset of stage
 * byte 0, out0 = stream index of the step's token 0. */
__device__ __noinline__ void k1a_rare(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ doc_off, VocabDev v,
                                      uint32_t* __restrict__ tok, uint64_t tok_words, uint32_t* status, uint32_t sb,
                                      const uint8_t* stage, uint32_t* tl, const uint16_t* ml, const uint4* sel,
                                      uint32_t nmiss, uint64_t p0, uint64_t out0, uint32_t gd0) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t j0 = 0; j0 < nmiss; j0 += 64) {
        const uint32_t j = j0 + lane;
        if (j < nmiss) {
            const uint32_t t = ml[j];
            const uint32_t e = tl[t];
            const uint32_t pos = e & 1023u, len = (e >> 10) & 31u, rel = (e >> 16) & 63u;
            const uint32_t word = (e >> 22) << sb;
            uint32_t slot;
            if (len != LEN_LONG) {
                const u32x4u raw = *reinterpret_cast<const u32x4u*>(stage + pos);
                const uint4 sl = sel[len];
                const uint32_t k0 = __builtin_amdgcn_perm(0x09090909u, raw.x, sl.x);
                const uint32_t k1 = __builtin_amdgcn_perm(0x09090909u, raw.y, sl.y);
                const uint32_t k2 = __builtin_amdgcn_perm(0x09090909u, raw.z, sl.z);
                const uint32_t k3 = __builtin_amdgcn_perm(0x09090909u, raw.w, sl.w);
                slot = vocab_insert(v, ((uint64_t)k1 << 32) | k0, ((uint64_t)k3 << 32) | k2, 0, status);
            } else {
                slot = slow_slot_a(bytes, v, p0 + pos, gload(doc_off + gd0 + rel + 1), status);
            }
            const uint64_t out = out0 + t;
            if (out < tok_words) gstore(tok + out, slot == INVALID_SLOT ? TOK_NONE : (word | slot));
            else atomicOr(status, ST_BOUNDS);
        }
    }
}

}  // namespace

/* an offset from the chunk frame, clamped to +-2^30 (beyond the chunk either way) */
__device__ __forceinline__ int32_t clamp_frame(int64_t d) {
    return d < -(1ll << 30) ? -(1 << 30) : d > (1ll << 30) ? (1 << 30) : (int32_t)d;
}

/* tbase(c): first stream word of chunk c (see the header) */
__device__ __forceinline__ uint64_t split_tbase(uint64_t cs, uint64_t lo, uint32_t dfirst, uint64_t c) {
    return ((cs - lo) >> 1) + dfirst + 4ull * c;
}

__global__ __launch_bounds__(A_NT, K1A_WAVES_PER_SIMD) void k_tok_resolve(
    CorpusDev c, const uint64_t* __restrict__ chunk_start, const uint32_t* __restrict__ chunk_doc, uint64_t nch,
    VocabDev v, K1Split sp, uint32_t* status, uint32_t sb, uint32_t G) {
    __shared__ __attribute__((aligned(16))) AShared S;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid < 64) {
        const uint32_t n = (uint32_t)tid >> 2, k = (uint32_t)tid & 3u;
        (&S.sel[n].x)[k] = perm_sel(n, k);
    }
    __syncthreads();   /* the only workgroup barrier: the waves are independent from here */
    const uint64_t last_blk = c.nbytes ? ((c.nbytes - 1) & ~(uint64_t)15) : 0;
    uint8_t* const stage = reinterpret_cast<uint8_t*>(&S.stage[wid][0]);
    uint32_t* const tl = S.tl[wid];
    const int32_t lane_off = 16 * lane - 16;
    uint32_t sh = (blockIdx.x * A_NW + wid) & 7u;
    const uint64_t lb_cap = (uint64_t)c.ndocs + nch + 1;

    /* Positions inside a chunk are int32 offsets from cb = chunk start & ~15 (a chunk and its
     * documents' starts that matter lie within +-2^30 of it): fewer 64-bit scalars. */
    uint64_t cb = 0, tbase = 0;   /* the current chunk's frame */
    uint16_t* const ml = S.ml[wid];

    uint64_t cur = claim_chunk_w(sp.shard_a, sh, nch);
    uint64_t nxt = claim_chunk_w(sp.shard_a, sh, nch);
    uint64_t cs = 0, ce = 0;
    uint32_t dfirst = 0, dlast = 0;
    if (cur < nch) {
        cs = chunk_start[cur]; ce = chunk_start[cur + 1];
        dfirst = chunk_doc[cur]; dlast = chunk_doc[cur + 1];
    }
    /* corpus prefetch ring: pfA holds the step at absolute address pa, pfB the one at pb */
    uint4 pfA = make_uint4(0, 0, 0, 0), pfB = make_uint4(0, 0, 0, 0);
    uint64_t pa = ~0ull, pb = ~0ull;
    uint64_t pre_gd = 0;
    bool pre_ok = false;
    while (cur < nch) {
        unsigned long long pend_v = 0;   /* the claim after next, used at the chunk end */
        if (lane == 0) pend_v = atomicAdd(&sp.shard_a[sh], 1ull);
        uint64_t ncs = 0, nce = 0;
        uint32_t ndf = 0, ndl = 0;
        if (nxt < nch) {
            ncs = chunk_start[nxt]; nce = chunk_start[nxt + 1];
            ndf = chunk_doc[nxt]; ndl = chunk_doc[nxt + 1];
        }
        cb = cs & ~(uint64_t)15;
        tbase = split_tbase(cs, c.lo, dfirst, cur);
        const uint64_t lb = (uint64_t)dfirst + cur;
        const int32_t span_r = (int32_t)(ce - cb);
        /* shard bounds in the frame (bytes outside [lo, hi) read as whitespace) */
        const int32_t lo_r = clamp_frame((int64_t)c.lo - (int64_t)cb);
        const int32_t hi_r = clamp_frame((int64_t)c.hi - (int64_t)cb);
        uint32_t run = 0, kord = 0, last_d = 0xFFFFFFFFu;
        /* the next chunk's first group offsets, fetched during the previous chunk (an empty
         * chunk, cs == ce, fetches none: the flag is consumed here either way) */
        const bool have_pre = pre_ok;
        pre_ok = false;
        if (cs < ce)
        for (uint32_t gd0 = dfirst;; gd0 += GA) {
            const uint32_t ng = (dlast + 1 - gd0) < GA ? (dlast + 1 - gd0) : GA;
            uint64_t gd;
            if (gd0 == dfirst && have_pre) gd = pre_gd;
            else gd = (uint32_t)lane <= ng ? gload(c.doc_off + gd0 + lane) : ~0ull;
            const bool last_group = gd0 + GA > dlast;
            if (last_group && nxt < nch) {   /* the next chunk's first group, in flight during this one */
                const uint32_t nng = (ndl + 1 - ndf) < GA ? (ndl + 1 - ndf) : GA;
                pre_gd = (uint32_t)lane <= nng ? gload(c.doc_off + ndf + lane) : ~0ull;
                pre_ok = true;
            }
            /* lane k <= ng: start of document gd0 + k in the frame, clamped; others past all */
            const int32_t gdr = (uint32_t)lane > ng ? (1 << 30) : clamp_frame((int64_t)gd - (int64_t)cb);
            const int32_t g0 = __builtin_amdgcn_readlane(gdr, 0), gn = __builtin_amdgcn_readlane(gdr, (int)ng);
            const int32_t gs = g0 > (int32_t)(cs - cb) ? g0 : (int32_t)(cs - cb);
            const int32_t ge = gn < span_r ? gn : span_r;
            if (gs < ge) {
                const int32_t b0 = gs & ~15;
                const uint32_t nsteps = (uint32_t)((ge - b0 + WSTEP - 1) / WSTEP);
                const bool ahead = last_group && nxt < nch && ncs < nce;
                const uint64_t nb0 = ncs & ~(uint64_t)15;
                for (uint32_t s = 0; s < nsteps; ++s) {
                    const int32_t sbase = b0 + (int32_t)s * WSTEP;
                    const int32_t gpos = sbase + lane_off;
                    uint4 cur4;
                    if (pa == cb + (uint64_t)sbase) cur4 = pfA;
                    else cur4 = ld16c(c.bytes, last_blk, cb + (uint64_t)(int64_t)gpos);
                    pfA = pfB;
                    pa = pb;
                    {
                        uint64_t nx = ~0ull;
                        if (s + 2 < nsteps) nx = cb + (uint64_t)(b0 + (int32_t)(s + 2) * WSTEP);
                        else if (ahead) nx = nb0 + (uint64_t)(s + 2 - nsteps) * WSTEP;
                        if (nx != ~0ull) pfB = ld16c(c.bytes, last_blk, nx + (uint64_t)(int64_t)lane_off);
                        pb = nx;
                    }
                    reinterpret_cast<uint4*>(stage)[lane] = cur4;
                    uint32_t ws = ws_mask16_swar(cur4);
                    if (!(sbase >= lo_r + 16 && sbase + WSTEP + 16 <= hi_r)) {
                        const int32_t a = gpos < lo_r ? min(lo_r - gpos, 16) : 0;
                        const int32_t b = hi_r > gpos ? min(hi_r - gpos, 16) : 0;
                        const uint32_t in = b > a ? (((1u << b) - 1u) & ~((1u << a) - 1u)) : 0u;
                        ws |= ~in & 0xFFFFu;
                    }
                    /* document starts in the window [sbase - 16, sbase + WSTEP + 16) and the
                     * document of each lane's first byte (long documents: none per step) */
                    const int32_t wlo = sbase - 16, whi = sbase + WSTEP + 16;
                    const uint64_t inwin = __ballot(gdr >= wlo && gdr < whi);
                    const uint32_t nbefore = (uint32_t)__popcll(__ballot(gdr < wlo));
                    uint32_t base = nbefore ? nbefore - 1u : 0u;
                    uint32_t ds = 0;
                    for (uint64_t m = inwin; m; m &= m - 1) {
                        const uint32_t k = (uint32_t)__builtin_ctzll(m);
                        const int32_t sk = __builtin_amdgcn_readlane(gdr, (int)k);
                        if (sk <= gpos) base = k;
                        if (sk >= gpos && sk < gpos + 16) ds |= 1u << (uint32_t)(sk - gpos);
                    }
                    const uint32_t prev = (lane_prev(ws) >> 15) & 1u;
                    uint32_t own = (lane >= 1 && lane <= 62) ? 0xFFFFu : 0u;
                    if (!(sbase >= gs && sbase + WSTEP <= ge) && own) {
                        own = 0;
                        if (gpos + 16 > gs && gpos < ge) {
                            const int32_t a = gpos < gs ? gs - gpos : 0;
                            const int32_t b = gpos + 16 > ge ? ge - gpos : 16;
                            own = ((1u << b) - 1u) & ~((1u << a) - 1u);
                        }
                    }
                    const uint32_t starts = ~ws & ((ws << 1) | prev | ds) & own & 0xFFFFu;
                    uint32_t nul = 0;
                    if (__ballot((zero_bits(cur4.x) | zero_bits(cur4.y) | zero_bits(cur4.z) | zero_bits(cur4.w)) != 0u) != 0ull)
                        nul = compress4(zero_bits(cur4.x)) | (compress4(zero_bits(cur4.y)) << 4) |
                              (compress4(zero_bits(cur4.z)) << 8) | (compress4(zero_bits(cur4.w)) << 12);
                    const uint32_t stop = ws | ds;
                    const uint32_t stop32 = stop | (lane_next(stop) << 16), nul32 = nul | (lane_next(nul) << 16);
                    const uint32_t nmine = (uint32_t)__popc(starts);
                    const uint32_t incl = wave_incl_scan(nmine);
                    const uint32_t ntok = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                    if (ntok == 0) continue;
                    if (K1A_ABL & 8) { run += ntok; continue; }
                    /* every token entry of the step (at most 992), then the rounds: no walk
                     * state stays live across them */
                    {
                        uint32_t sm = starts, idx = incl - nmine;
                        while (sm) {
                            const uint32_t i = (uint32_t)__builtin_ctz(sm);
                            sm &= sm - 1;
                            const uint32_t e = ((stop32 >> i) & ~1u) | (nul32 >> i);
                            const uint32_t len = e ? (uint32_t)__builtin_ctz(e) : LEN_LONG;
                            /* the document of byte i: the last one starting at or before it */
                            uint32_t rel = base;
                            if (ds & ((2u << i) - 2u)) {
                                for (uint64_t m = inwin; m; m &= m - 1) {
                                    const uint32_t k = (uint32_t)__builtin_ctzll(m);
                                    if (__builtin_amdgcn_readlane(gdr, (int)k) <= gpos + (int32_t)i) rel = k;
                                }
                            }
                            tl[idx] = ((uint32_t)lane << 4 | i) | ((len < 16u ? len : LEN_LONG) << 10) | (rel << 16);
                            ++idx;
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    /* Rounds of 64 tokens.  A token whose key is in neither of the two slots
                     * loaded (a new term, a displaced key) or whose term is long only queues
                     * its entry index; the rare pass below resolves those, so the round loop
                     * holds no insert code (no spills) */
                    uint32_t nmiss = 0;
                    for (uint32_t t0 = 0; t0 < ntok && !(K1A_ABL & 2); t0 += 64) {
                        const uint32_t t = t0 + (uint32_t)lane;
                        const bool val = t < ntok;
                        const uint32_t e = val ? tl[t] : 0u;
                        const uint32_t pos = e & 1023u, len = (e >> 10) & 31u, rel = e >> 16;
                        const bool shrt = val && len != LEN_LONG;
                        const uint32_t dabs = gd0 + rel;
                        const u32x4u raw = *reinterpret_cast<const u32x4u*>(stage + pos);
                        const uint4 sl = S.sel[len & 15u];
                        const uint32_t k0 = __builtin_amdgcn_perm(0x09090909u, raw.x, sl.x);
                        const uint32_t k1 = __builtin_amdgcn_perm(0x09090909u, raw.y, sl.y);
                        const uint32_t k2 = __builtin_amdgcn_perm(0x09090909u, raw.z, sl.z);
                        const uint32_t k3 = __builtin_amdgcn_perm(0x09090909u, raw.w, sl.w);
                        const uint32_t hv = shrt ? (uint32_t)(key_hash(((uint64_t)k1 << 32) | k0, ((uint64_t)k3 << 32) | k2) &
                                                              v.mask)
                                                 : 0u;
#if K1A_ABL & 1
                        const uint4 s4 = make_uint4(k0, k1, k2, k3), t4 = s4;
#else
                        const uint4 s4 = gload(v.keys + hv);
                        const uint4 t4 = gload(v.keys + ((hv + 1) & (uint32_t)v.mask));
#endif
                        /* the document ordinal: a token whose document differs from the
                         * previous token's starts the next ordinal */
                        /* lane i-1's document; lane 0 (no source lane) keeps `old` = the
                         * previous round's last.  One DPP move: written as a select, the
                         * compiler masked lane 0 off around the DPP, and a DPP read of an
                         * inactive lane returns the reader's own value */
                        const uint32_t pd = (uint32_t)__builtin_amdgcn_update_dpp((int)last_d, (int)dabs, DPP_WAVE_SHR1,
                                                                                  0xF, 0xF, false);
                        const bool flag = val && dabs != pd;
                        const uint64_t fm = __ballot(flag);
                        const uint32_t ord = kord + lane_below(fm) - (flag ? 0u : 1u);
                        const uint32_t ti = run + t;
                        if (flag && !(K1A_ABL & 4)) {
                            if (lb + ord < lb_cap) {
                                gstore(sp.dlist + lb + ord, dabs);
                                gstore(sp.dtok + lb + ord, ti);
                            } else {
                                atomicOr(status, ST_BOUNDS);
                            }
                        }
                        kord += (uint32_t)__popcll(fm);
                        const uint32_t lastl = (ntok - t0) < 64u ? (ntok - t0 - 1u) : 63u;
                        last_d = (uint32_t)__builtin_amdgcn_readlane((int)dabs, (int)lastl);
                        const uint32_t word = (ord & (G - 1u)) << sb;
                        const bool hit0 = s4.x == k0 && s4.y == k1 && s4.z == k2 && s4.w == k3;
                        const bool hit1 = t4.x == k0 && t4.y == k1 && t4.z == k2 && t4.w == k3;
                        const bool miss = val && !(shrt && (hit0 || hit1));
                        if (val && !miss && !(K1A_ABL & 4)) {
                            const uint64_t out = tbase + ti;
                            const uint32_t slot = hit0 ? hv : ((hv + 1) & (uint32_t)v.mask);
                            if (out < sp.tok_words) gstore(sp.tok + out, word | slot);
                            else atomicOr(status, ST_BOUNDS);
                        }
                        const uint64_t mm = __ballot(miss);
                        if (miss) {
                            ml[nmiss + lane_below(mm)] = (uint16_t)t;
                            tl[t] = e | ((ord & (G - 1u)) << 22);   /* the ordinal field for the rare pass */
                        }
                        nmiss += (uint32_t)__popcll(mm);
                    }
                    if (nmiss && !(K1A_ABL & 16)) {   /* the rare pass (stage and entries are still this step's) */
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        k1a_rare(c.bytes, c.doc_off, v, sp.tok, sp.tok_words, status, sb, stage, tl, ml, S.sel, nmiss,
                                 cb + (uint64_t)(int64_t)(sbase - 16), tbase + run, gd0);
                    }
                    run += ntok;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            }
            if (last_group) break;
        }
        if (lane == 0) sp.chunk_meta[cur] = make_uint2(run, kord);
        {
            const uint64_t lo = nch * sh / 8, hi = nch * (sh + 1) / 8;
            const uint64_t pv = ufirst64(pend_v);
            const uint64_t nn = lo + pv < hi ? lo + pv : claim_chunk_w(sp.shard_a, sh, nch);
            cur = nxt;
            nxt = nn;
        }
        cs = ncs; ce = nce; dfirst = ndf; dlast = ndl;
    }
}

/* ------------------------------------------------------------------ K1b ---------- */

namespace {

#ifndef K1B_NT
#define K1B_NT 256
#endif
#ifndef K1B_TB
#define K1B_TB 3584
#endif
#ifndef K1B_WGCU
#define K1B_WGCU (1024 / K1B_NT)
#endif
constexpr int B_NT = K1B_NT;
constexpr int B_NW = B_NT / 64;
constexpr int TB = K1B_TB;                /* LDS table entries (u32 key + u32 count) */
constexpr int EPT = TB / B_NT;
constexpr uint32_t FILL_LIMIT = TB - B_NT * 2 - 64;
constexpr int GCAP = 256;                 /* documents per group at most */
constexpr uint32_t BW = 4;
constexpr uint32_t NB = TB / BW;

struct BShared {
    uint32_t TK[TB];                      /* key32 = 1 << 31 | ordinal << sb | slot (0: empty) */
    uint32_t TC[TB];
    uint32_t gid[GCAP];                   /* document index of each ordinal of the group */
    uint32_t ts[GCAP + 1];                /* chunk token index of each ordinal's first token */
    uint32_t dcnt[GCAP];                  /* flush: entries per document */
    uint32_t doff[GCAP];
    uint32_t drun[GCAP];
    uint8_t dstate[GCAP];                 /* 0 none, 1 partial, 2 complete */
    uint8_t gcomp[GCAP];                  /* document lies inside the chunk */
    uint8_t dpart[GCAP];                  /* document has overflow records */
    uint64_t fbase[8];
    uint32_t fill;
    uint64_t cur_chunk, nxt_chunk;
    uint32_t wsum[B_NW];
    unsigned long long rec_base, part_base;
};

struct BktK {
    uint4 a;
};
__device__ __forceinline__ uint32_t bkt_hash(uint32_t key) {
    return (uint32_t)(((uint64_t)(key * 0x9E3779B1u) * (uint64_t)NB) >> 32);
}
__device__ __forceinline__ uint32_t bkt_next(uint32_t b) { return b + 1 == NB ? 0u : b + 1; }
__device__ __forceinline__ BktK bkt_read(BShared& S, uint32_t b) {
    BktK k;
    k.a = reinterpret_cast<const uint4*>(S.TK)[b];
    return k;
}
__device__ __forceinline__ uint32_t bkt_match(const BktK& kk, uint32_t key) {
    return kk.a.x == key ? 0u : kk.a.y == key ? 1u : kk.a.z == key ? 2u : kk.a.w == key ? 3u : 4u;
}
__device__ __forceinline__ uint32_t bkt_empty(const BktK& kk, uint32_t key) {
    const uint32_t em = (kk.a.x == 0u ? 1u : 0u) | (kk.a.y == 0u ? 2u : 0u) | (kk.a.z == 0u ? 4u : 0u) | (kk.a.w == 0u ? 8u : 0u);
    if (!em) return BW;
    const uint32_t r0 = key & (BW - 1u);
    const uint32_t rot = ((em | (em << BW)) >> r0) & ((1u << BW) - 1u);
    return ((uint32_t)__builtin_ctz(rot) + r0) & (BW - 1u);
}

__device__ __forceinline__ void overflow_rec(const K1Out& o, uint32_t doc, uint32_t slot) {
    const uint64_t am = __ballot(1);
    const uint32_t rank = lane_below(am);
    unsigned long long b = 0;
    if (rank == 0u) b = atomicAdd(o.part_alloc, (unsigned long long)__popcll(am));
    const unsigned long long q = ufirst64(b) + rank;
    if (q < o.part_cap) { o.part_doc[q] = doc; o.part_slot[q] = slot; o.part_cnt[q] = 1u; }
    else atomicOr(o.status, ST_PART_FULL);
}

/* the slow count (tokcount_st.hip bkt_slow): full home bucket, a lost claim, overflow mode */
constexpr int PMAX = 16;
__device__ uint32_t bkt_slow_b(BShared& S, const K1Out& o, uint32_t key, uint32_t b, bool over, uint32_t sb) {
    for (int probe = 0, tries = 0; probe < PMAX && tries < 64; ++tries) {
        const BktK kk = bkt_read(S, b);
        const uint32_t j = bkt_match(kk, key);
        if (j < BW) { atomicAdd(&S.TC[BW * b + j], 1u); return 0u; }
        const uint32_t e = bkt_empty(kk, key);
        if (e < BW) {
            if (over) break;
            const uint32_t old = atomicCAS(&S.TK[BW * b + e], 0u, key);
            if (old == 0u || old == key) {
                atomicAdd(&S.TC[BW * b + e], 1u);
                return old == 0u ? 1u : 0u;
            }
            continue;
        }
        b = bkt_next(b);
        ++probe;
    }
    const uint32_t rel = (key & 0x7FFFFFFFu) >> sb;
    S.dpart[rel] = 1;
    overflow_rec(o, S.gid[rel], key & ((1u << sb) - 1u));
    return 0u;
}

__device__ __forceinline__ void wave_agg_add(uint32_t* ctr, uint32_t idx) {
    const uint32_t i0 = ufirst(idx);
    const uint64_t am = __ballot(1);
    if (__ballot(idx != i0) == 0ull) {
        if (lane_below(am) == 0u) atomicAdd(&ctr[i0], (uint32_t)__popcll(am));
    } else {
        atomicAdd(&ctr[idx], 1u);
    }
}
__device__ __forceinline__ uint32_t wave_agg_add_rtn(uint32_t* ctr, uint32_t idx) {
    const uint32_t i0 = ufirst(idx);
    const uint64_t am = __ballot(1);
    uint32_t k;
    if (__ballot(idx != i0) == 0ull) {
        const uint32_t rank = lane_below(am);
        uint32_t b = 0;
        if (rank == 0u) b = atomicAdd(&ctr[i0], (uint32_t)__popcll(am));
        k = ufirst(b) + rank;
    } else {
        k = atomicAdd(&ctr[idx], 1u);
    }
    return k;
}

/* Emits the group's table entries as records and clears the table (tokcount_st.hip
 * st_flush): complete documents to the record stream, documents crossing a chunk edge,
 * over K5's in-LDS sort size or overflowed, to the partial stream. */
__device__ void b_flush(BShared& S, const K1Out& o, uint32_t ng, uint32_t sb) {
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    if (tid < GCAP) { S.dcnt[tid] = 0; S.drun[tid] = 0; }
    __syncthreads();
    const uint32_t smask = (1u << sb) - 1u;
    uint32_t ek[EPT], ec[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        ek[j] = S.TK[j * B_NT + tid];
        ec[j] = S.TC[j * B_NT + tid];
        if (ek[j]) wave_agg_add(&S.dcnt[0], (ek[j] & 0x7FFFFFFFu) >> sb);
    }
    lds_barrier();
    uint32_t packed = 0;
    if ((uint32_t)tid < ng) {
        uint8_t st = 0;
        const uint32_t cnt = S.dcnt[tid];
        const bool part = S.dpart[tid] != 0;
        if (cnt) {
            const bool complete = !part && S.gcomp[tid] && cnt <= (uint32_t)K5_MAX_PAIRS;
            st = complete ? 2 : 1;
            packed = complete ? cnt : (cnt << 16);
        }
        if (st == 1 || part) o.doc_flags[S.gid[tid]] = DF_PARTIAL;
        S.dstate[tid] = st;
    }
    uint32_t tot;
    const uint32_t off = block_excl_scan<B_NT, true>(packed, S.wsum, &tot);
    if ((uint32_t)tid < ng) S.doff[tid] = off;
    const uint32_t nrec = tot & 0xFFFFu, npart = tot >> 16;
    if (tid == 0) {
        const unsigned long long rb = nrec ? atomicAdd(o.rec_alloc, (unsigned long long)nrec) : 0ull;
        if (rb + nrec > o.rec_cap) atomicOr(o.status, ST_REC_FULL);
        S.rec_base = rb;
    } else if (tid == 64) {
        const unsigned long long pb = npart ? atomicAdd(o.part_alloc, (unsigned long long)npart) : 0ull;
        if (pb + npart > o.part_cap) atomicOr(o.status, ST_PART_FULL);
        S.part_base = pb;
    }
    lds_barrier();
    const unsigned long long rb = S.rec_base, pb = S.part_base;
    const bool rec_ok = rb + nrec <= o.rec_cap, part_ok = pb + npart <= o.part_cap;
    if ((uint32_t)tid < ng && S.dstate[tid] == 2) {
        o.doc_recoff[S.gid[tid]] = rb + (off & 0xFFFFu);
        o.doc_npairs[S.gid[tid]] = S.dcnt[tid];
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const uint32_t key = ek[j];
        if (key) {
            const uint32_t rel = (key & 0x7FFFFFFFu) >> sb;
            const uint32_t k = wave_agg_add_rtn(&S.drun[0], rel);
            const uint32_t dof = S.doff[rel];
            if (S.dstate[rel] == 2) {
                const uint64_t q = rb + (dof & 0xFFFFu) + k;
                if (rec_ok) { o.rec_slot[q] = key & smask; o.rec_cnt[q] = ec[j]; }
            } else {
                const uint64_t q = pb + (dof >> 16) + k;
                if (part_ok) { o.part_doc[q] = S.gid[rel]; o.part_slot[q] = key & smask; o.part_cnt[q] = ec[j]; }
            }
            S.TK[j * B_NT + tid] = 0u;
            S.TC[j * B_NT + tid] = 0u;
        }
    }
}

/* the flush of a group of at most FEW documents (tokcount_st.hip st_flush_few): per-thread
 * 16-bit document counters, one block scan, no LDS atomics */
constexpr uint32_t FEW = 8;
__device__ void b_flush_few(BShared& S, const K1Out& o, uint32_t ng, uint32_t sb) {
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, w = tid >> 6;
    const uint32_t smask = (1u << sb) - 1u;
    uint32_t ek[EPT], ec[EPT];
    uint32_t pk[FEW / 2] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        ek[j] = S.TK[j * B_NT + tid];
        ec[j] = S.TC[j * B_NT + tid];
        if (ek[j]) {
            const uint32_t rel = (ek[j] & 0x7FFFFFFFu) >> sb;
#pragma unroll
            for (uint32_t q = 0; q < FEW / 2; ++q) pk[q] += (rel >> 1) == q ? (1u << (16 * (rel & 1u))) : 0u;
        }
    }
    uint32_t inc[FEW / 2];
#pragma unroll
    for (uint32_t q = 0; q < FEW / 2; ++q) {
        inc[q] = wave_incl_scan(pk[q]);
        if (lane == 63) S.dcnt[w * (FEW / 2) + q] = inc[q];
    }
    lds_barrier();
    uint32_t rank[FEW / 2], tot[FEW / 2];
#pragma unroll
    for (uint32_t q = 0; q < FEW / 2; ++q) {
        uint32_t base = 0, t = 0;
#pragma unroll
        for (int k = 0; k < B_NW; ++k) {
            const uint32_t x = S.dcnt[k * (FEW / 2) + q];
            base += k < w ? x : 0u;
            t += x;
        }
        rank[q] = base + inc[q] - pk[q];
        tot[q] = t;
    }
    if (w == 0) {
        const uint32_t d = (uint32_t)lane;
        uint32_t cnt = 0, packed = 0;
        uint8_t st = 0;
        if (d < ng) {
#pragma unroll
            for (uint32_t q = 0; q < FEW / 2; ++q)
                if ((d >> 1) == q) cnt = (tot[q] >> (16 * (d & 1u))) & 0xFFFFu;
            const bool part = S.dpart[d] != 0;
            if (cnt) {
                const bool complete = !part && S.gcomp[d] && cnt <= (uint32_t)K5_MAX_PAIRS;
                st = complete ? 2 : 1;
                packed = complete ? cnt : (cnt << 16);
            }
            if (st == 1 || part) o.doc_flags[S.gid[d]] = DF_PARTIAL;
        }
        const uint32_t incl = wave_incl_scan(packed);
        const uint32_t all = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t off = incl - packed;
        const uint32_t nrec = all & 0xFFFFu, npart = all >> 16;
        unsigned long long a0 = 0, a1 = 0;
        if (lane == 0 && nrec) a0 = atomicAdd(o.rec_alloc, (unsigned long long)nrec);
        if (lane == 32 && npart) a1 = atomicAdd(o.part_alloc, (unsigned long long)npart);
        const unsigned long long rb = readlane64(a0, 0), pb = readlane64(a1, 32);
        const bool rec_ok = rb + nrec <= o.rec_cap, part_ok = pb + npart <= o.part_cap;
        if (lane == 0 && !rec_ok) atomicOr(o.status, ST_REC_FULL);
        if (lane == 0 && !part_ok) atomicOr(o.status, ST_PART_FULL);
        if (d < ng) {
            uint64_t fb = ~0ull;
            if (st == 2) {
                fb = rec_ok ? rb + (off & 0xFFFFu) : ~0ull;
                o.doc_recoff[S.gid[d]] = rb + (off & 0xFFFFu);
                o.doc_npairs[S.gid[d]] = cnt;
            } else if (st == 1) {
                fb = part_ok ? pb + (off >> 16) : ~0ull;
            }
            S.fbase[d] = fb;
            S.dstate[d] = st;
        }
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const uint32_t key = ek[j];
        if (key) {
            const uint32_t rel = (key & 0x7FFFFFFFu) >> sb;
            uint32_t r = 0;
#pragma unroll
            for (uint32_t q = 0; q < FEW / 2; ++q)
                if ((rel >> 1) == q) {
                    r = (rank[q] >> (16 * (rel & 1u))) & 0xFFFFu;
                    rank[q] += 1u << (16 * (rel & 1u));
                }
            const uint64_t fb = S.fbase[rel];
            if (fb != ~0ull) {
                const uint64_t qq = fb + r;
                if (S.dstate[rel] == 2) { o.rec_slot[qq] = key & smask; o.rec_cnt[qq] = ec[j]; }
                else { o.part_doc[qq] = S.gid[rel]; o.part_slot[qq] = key & smask; o.part_cnt[qq] = ec[j]; }
            }
            S.TK[j * B_NT + tid] = 0u;
            S.TC[j * B_NT + tid] = 0u;
        }
    }
}

__device__ __forceinline__ uint64_t claim_chunk_b(unsigned long long* ctr, uint32_t& sh, uint64_t n) {
    for (int t = 0; t < 8; ++t) {
        const uint64_t lo = n * sh / 8, hi = n * (sh + 1) / 8;
        if (hi > lo) {
            const uint64_t v = atomicAdd(&ctr[sh], 1ull);
            if (lo + v < hi) return lo + v;
        }
        sh = (sh + 1) & 7u;
    }
    return n;
}

}  // namespace

__global__ __launch_bounds__(B_NT, K1B_WGCU) void k_count_slots(CorpusDev c, const uint64_t* __restrict__ chunk_start,
                                                                const uint32_t* __restrict__ chunk_doc, uint64_t nch,
                                                                K1Split sp, K1Out o, uint32_t sb, uint32_t G) {
    __shared__ __attribute__((aligned(16))) BShared S;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int j = 0; j < EPT; ++j) { S.TK[j * B_NT + tid] = 0u; S.TC[j * B_NT + tid] = 0u; }
    uint32_t shard = blockIdx.x & 7u;
    if (tid == 0) {
        S.cur_chunk = claim_chunk_b(sp.shard_b, shard, nch);
        S.nxt_chunk = claim_chunk_b(sp.shard_b, shard, nch);
    }
    __syncthreads();
    uint64_t chunk = ufirst64(S.cur_chunk), nxt = ufirst64(S.nxt_chunk);

    /* one LDS count (tokcount_st.hip count()): ONE ds_read_b128 of the home bucket, a
     * match adds, a new key claims a free slot with one CAS; the rest takes bkt_slow_b */
    auto count = [&](uint32_t key) {
        const bool over = S.fill >= FILL_LIMIT;
        const uint32_t b = bkt_hash(key);
        uint32_t claims = 0u;
        bool slow = false;
        if (key) {
            const BktK kk = bkt_read(S, b);
            const uint32_t j = bkt_match(kk, key);
            if (j < BW) {
                atomicAdd(&S.TC[BW * b + j], 1u);
            } else {
                const uint32_t e = bkt_empty(kk, key);
                if (e < BW && !over) {
                    const uint32_t old = atomicCAS(&S.TK[BW * b + e], 0u, key);
                    if (old == 0u || old == key) {
                        atomicAdd(&S.TC[BW * b + e], 1u);
                        claims = old == 0u ? 1u : 0u;
                    } else {
                        slow = true;
                    }
                } else {
                    slow = true;
                }
            }
        }
        if (__ballot(slow) != 0ull) {
            if (slow) claims = bkt_slow_b(S, o, key, b, over, sb);
        }
        const uint32_t wc = (uint32_t)__popcll(__ballot(claims != 0u));
        if (wc && lane == 0) (void)atomicAdd(&S.fill, wc);
    };

    /* What a chunk needs before its first count — its metadata, the first group's ordinal
     * lists, those documents' bounds and each wave's first stream row — is fetched during
     * the previous chunk in three dependent stages (metadata at its start, lists and row
     * before its flush, bounds after it), so a chunk starts without an HBM round trip. */
    struct Meta {
        uint32_t ntok, nd, df;
        uint64_t cs, ce;
    };
    auto load_meta = [&](uint64_t ch) {
        Meta m{0, 0, 0, 0, 0};
        if (ch < nch) {
            const uint2 mt = sp.chunk_meta[ch];
            m.ntok = mt.x;
            m.nd = mt.y;
            m.cs = chunk_start[ch];
            m.ce = chunk_start[ch + 1];
            m.df = chunk_doc[ch];
        }
        return m;
    };
    /* stage 2: this thread's ordinal of group g0 (document, first token) and, thread 0, the
     * group's token end; the wave's first stream row */
    uint32_t p_id = 0, p_ts = 0, p_tend = 0;
    uint4 p_wv = make_uint4(TOK_NONE, TOK_NONE, TOK_NONE, TOK_NONE);
    auto load_lists = [&](uint64_t ch, const Meta& m, uint32_t g0) {
        const uint32_t ng = (m.nd - g0) < G ? (m.nd - g0) : G;
        const uint64_t lb = (uint64_t)m.df + ch;
        if ((uint32_t)tid < ng) {
            p_id = gload(sp.dlist + lb + g0 + tid);
            p_ts = gload(sp.dtok + lb + g0 + tid);
        }
        if (tid == 0) p_tend = g0 + ng < m.nd ? gload(sp.dtok + lb + g0 + ng) : m.ntok;
    };
    auto load_row = [&](uint64_t ch, const Meta& m) {   /* group 0's first row (its t0 is 0) */
        const uint64_t tb = split_tbase(m.cs, c.lo, m.df, ch);
        const uint64_t ra = (tb & ~3ull) + 256ull * wid + 4ull * lane;
        p_wv = ra < tb + m.ntok ? gload(reinterpret_cast<const uint4*>(sp.tok + ra))
                                : make_uint4(TOK_NONE, TOK_NONE, TOK_NONE, TOK_NONE);
    };
    /* stage 3: the document lies inside the chunk */
    uint32_t p_comp = 0;
    auto load_bounds = [&](const Meta& m, uint32_t g0) {
        const uint32_t ng = (m.nd - g0) < G ? (m.nd - g0) : G;
        if ((uint32_t)tid < ng) p_comp = (gload(c.doc_off + p_id) >= m.cs && gload(c.doc_off + p_id + 1) <= m.ce) ? 1u : 0u;
    };

    Meta cm = load_meta(chunk);
    if (chunk < nch) {
        load_lists(chunk, cm, 0);
        load_row(chunk, cm);
        load_bounds(cm, 0);
    }
    while (chunk < nch) {
        unsigned long long pend_v = 0;
        if (tid == 0) pend_v = atomicAdd(&sp.shard_b[shard], 1ull);
        const Meta nm = load_meta(nxt);   /* stage 1 of the next chunk */
        const uint64_t cs = cm.cs, ce = cm.ce;
        const uint64_t tbase = split_tbase(cs, c.lo, cm.df, chunk);
        const uint64_t lb = (uint64_t)cm.df + chunk;
        const uint32_t ntok = cm.ntok, nd = cm.nd;
        if (tid == 0 && ntok) atomicAdd(o.ntokens, (unsigned long long)ntok);
        for (uint32_t g0 = 0; g0 < nd; g0 += G) {
            const uint32_t ng = (nd - g0) < G ? (nd - g0) : G;
            const bool last = g0 + G >= nd;
            if (g0) {   /* chunks of more than G documents with tokens: later groups unprefetched */
                load_lists(chunk, cm, g0);
                load_bounds(cm, g0);
            }
            if ((uint32_t)tid < ng) {
                S.gid[tid] = p_id;
                S.ts[tid] = p_ts;
                S.gcomp[tid] = (uint8_t)p_comp;
                S.dpart[tid] = 0;
            }
            if (tid == 0) {
                S.ts[ng] = p_tend;
                S.fill = 0;
            }
            __syncthreads();
            const uint32_t t0 = S.ts[0], t1 = S.ts[ng];
            /* stream rows: each lane loads 4 consecutive words (one dwordx4 per 256 tokens
             * per wave), the next row in flight while this one is counted */
            const uint64_t a0 = (tbase + t0) & ~3ull, aend = tbase + t1;
            uint64_t ra = a0 + 256ull * wid + 4ull * lane;
            uint4 wv = p_wv;
            if (g0) wv = ra < aend ? gload(reinterpret_cast<const uint4*>(sp.tok + ra))
                                   : make_uint4(TOK_NONE, TOK_NONE, TOK_NONE, TOK_NONE);
            for (uint64_t r0 = a0 + 256ull * wid; r0 < aend; r0 += 256ull * B_NW) {
                const uint4 w = wv;
                const uint64_t rw = ra;
                ra += 256ull * B_NW;
                if (ra < aend) wv = gload(reinterpret_cast<const uint4*>(sp.tok + ra));
                const uint32_t wa[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint64_t idx = rw + j;
                    const bool ok = idx >= tbase + t0 && idx < aend && wa[j] != TOK_NONE;
                    count(ok ? (0x80000000u | wa[j]) : 0u);
                }
            }
            if (last && nxt < nch) {   /* stage 2 of the next chunk, in flight during the flush */
                load_lists(nxt, nm, 0);
                load_row(nxt, nm);
            }
            lds_barrier();
            if (ng <= FEW) b_flush_few(S, o, ng, sb);
            else b_flush(S, o, ng, sb);
            if (last && nxt < nch) load_bounds(nm, 0);   /* stage 3 */
            /* docSize = the distance between the ordinals' first tokens */
            if ((uint32_t)tid < ng) {
                const uint32_t n = S.ts[tid + 1] - S.ts[tid];
                if (n) {
                    const uint32_t d = S.gid[tid];
                    if (S.gcomp[tid]) o.doc_size[d] = n;
                    else atomicAdd(&o.doc_size[d], n);
                }
            }
            __syncthreads();
        }
        if (nd == 0 && nxt < nch) {   /* a chunk without tokens: the next chunk's stages now */
            load_lists(nxt, nm, 0);
            load_row(nxt, nm);
            load_bounds(nm, 0);
        }
        (void)lb;
        if (tid == 0) {
            const uint64_t lo = nch * shard / 8, hi = nch * (shard + 1) / 8;
            const uint64_t claim = lo + pend_v < hi ? lo + pend_v : claim_chunk_b(sp.shard_b, shard, nch);
            S.cur_chunk = nxt;
            S.nxt_chunk = claim;
        }
        __syncthreads();
        chunk = nxt;
        nxt = ufirst64(S.nxt_chunk);
        cm = nm;
    }
}

int launch_tokcount_split(const CorpusDev& c, const uint64_t* chunk_start, const uint32_t* chunk_doc, uint64_t nch,
                          const VocabDev& v, const K1Out& o, const K1Split& sp, hipStream_t s) {
    if (nch == 0) return 0;
    if (v.mask >= (1ull << 28)) return -3;
    static_assert(sizeof(BShared) * K1B_WGCU <= 163840, "LDS of K1B_WGCU workgroups per CU");
    static_assert(TB % B_NT == 0 && TB % BW == 0, "table rows");
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const uint32_t sb = (uint32_t)__builtin_popcountll(v.mask);
    /* ordinal field: key32 = 1 << 31 | ordinal << sb | slot */
    const uint32_t G = (1u << (31u - sb)) >= (uint32_t)GCAP ? (uint32_t)GCAP : (1u << (31u - sb));
    const uint64_t wa = (uint64_t)ncu * K1A_WGCU * A_NW;
    const uint64_t ga = ((nch < wa ? nch : wa) + A_NW - 1) / A_NW;
    k_tok_resolve<<<(unsigned)ga, A_NT, 0, s>>>(c, chunk_start, chunk_doc, nch, v, sp, o.status, sb, G);
    if (hipGetLastError() != hipSuccess) return -1;
    const uint64_t wb = (uint64_t)ncu * K1B_WGCU;
    const uint64_t gb = nch < wb ? nch : wb;
    k_count_slots<<<(unsigned)gb, B_NT, 0, s>>>(c, chunk_start, chunk_doc, nch, sp, o, sb, G);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* token-stream words needed for a corpus span of `span` bytes, N documents, nch chunks */
uint64_t tokcount_split_words(uint64_t span, uint64_t ndocs, uint64_t nch) { return span / 2 + ndocs + 4 * nch + 64; }
