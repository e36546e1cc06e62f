/*
 * tokcount_win.hip — K1: fused tokenize + per-document term counting over block-wide
 * 8 KiB windows.  Replaces the reference's per-rank hot loop TFIDF.c:130-196: fscanf("%s")
 * tokenising (:141-147), the O(P) strcmp search/append of (word, doc) records (:151-167)
 * and the per-rank word table (:169-188).
 *
 * Structure (one workgroup of 256 threads per chunk at a time, four per CU):
 *   chunks   a persistent grid takes K0's chunks (~16 KiB of whole documents, or a piece
 *            of a document longer than BIG_DOC) from 8 sharded counters; a chunk's
 *            documents are processed in groups of <= gcap (as tokcount_lean.hip).
 *   window   the group's bytes in 8 KiB windows.  Every thread owns 32 bytes (two 16-byte
 *            loads, issued one window ahead into registers, across chunk boundaries too);
 *            thread 0 also loads the 16 bytes before the window, thread 255 the 16 after.
 *            Per thread: SWAR C-locale isspace (TFIDF.c:142,147), NUL bytes (a term ends at
 *            its first NUL: strcmp, TFIDF.c:152,172), document starts from an LDS bitmap,
 *            token starts = not-ws and (previous byte ws or document start), one block scan
 *            of (tokens, document starts) per window; every token start becomes one 32-bit
 *            entry (window offset | term length | document in group) in an LDS list.  The
 *            term length comes from the owner's stop mask and its right neighbour's (DPP
 *            within a wave, LDS across waves).
 *   resolve  each thread takes list entries tid, tid + 256, ... in batches of BATCH: per
 *            entry ONE unaligned ds_read_b128 of the term and four v_perm_b32 build the
 *            exact 128-bit identity key (dev_common.h), a two-multiply hash, and the home
 *            vocabulary slot plus the next one are loaded — all BATCH tokens' loads are in
 *            flight together (the round-based kernels had one token per lane in flight).
 *            Misses and terms of >= 16 bytes go to the out-of-line rare paths.
 *   count    the batch's (document, slot) keys: all bucket reads issued, then add on a
 *            match or claim a free slot by CAS (a stale bucket view is harmless: the CAS
 *            arbitrates, keys never move).  Past FILL_LIMIT claims the group is in overflow
 *            mode: absent pairs become partial records of count 1, merged by finalize.hip.
 *   flush    per group: every (document, slot) entry becomes a record (complete documents)
 *            or a partial record (documents split across chunks, or overflowing the table).
 *
 * LDS: 22 KiB table + 18 KiB window/list/state -> four workgroups (16 waves) per CU.
 * Requires a 16-byte aligned corpus base.
 */
#include "dev_common.h"
#include "dev_vocab.h"
#include "kernels.h"

namespace {

constexpr int NT = 256;                   /* threads per workgroup */
constexpr int WG_PER_CU = 4;
constexpr int NWAVE = NT / 64;
constexpr uint32_t W = 8192;              /* window bytes: 32 per thread */
constexpr uint32_t LCAP = 1536;           /* token entries per pass (c2 windows hold ~1100 tokens) */
constexpr int GCAP = 128;                 /* documents per group at most */
constexpr uint32_t LEN_LONG = 16u;        /* entry length: term of >= 16 bytes */
constexpr uint32_t BW = 4;                /* LDS table bucket width */
constexpr int TB = 2816;                  /* LDS table entries (u32 key + u32 count): 11 per thread */
constexpr uint32_t NB = TB / BW;
constexpr int EPT = TB / NT;
constexpr uint32_t FILL_LIMIT = TB - NT * 2 - 64;  /* claims after which overflow mode starts */
constexpr int BATCH = 4;                  /* tokens per thread with vocabulary loads in flight together */
constexpr uint32_t ENT_NONE = 0xFFFFFFFFu;
static_assert(W == NT * 32, "one 32-bit mask per thread");
static_assert(GCAP < NT, "one thread per group document offset");

struct WShared {
    uint32_t TK[TB];                      /* key32 = 1 << 31 | doc-in-group << sb | slot (0: empty) */
    uint32_t TC[TB];                      /* its count */
    uint4 wb[W / 16 + 2];                 /* [ws - 16, ws + W + 16): head, window, tail */
    union {
        uint32_t list[LCAP];              /* token entries of the window (pass) */
        struct {                          /* flush */
            uint32_t dcnt[GCAP];
            uint32_t doff[GCAP];
            uint32_t drun[GCAP];
            uint8_t dstate[GCAP];
        } f;
    };
    uint32_t dsb[NT + 1];                 /* document-start bits of the window (+ the tail's 16) */
    uint64_t gdoc[GCAP + 1];              /* doc_off of the group's documents */
    uint32_t dsz[GCAP];                   /* docSize accumulators */
    uint4 sel[16];                        /* v_perm selectors of a term of length n */
    uint64_t fbase[8];
    uint8_t dpart[GCAP];                  /* document has overflow records */
    uint32_t xs[NWAVE + 1];               /* each wave's lane-0 stop mask; the tail's */
    uint32_t wsum[NWAVE];
    uint32_t fill;
    uint32_t dup;                         /* two documents start at one position in this window */
    uint32_t cur_chunk, nxt_chunk;
    unsigned long long rec_base, part_base;
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));   /* unaligned LDS read */

__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
    const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(r.x, r.y, r.z, r.w);
}

/* bits of the bytes [gp, gp + 32) that lie inside [lo, hi) */
__device__ __forceinline__ uint32_t in_mask32(int32_t gp, int32_t lo, int32_t hi) {
    const int32_t a = min(max(lo - gp, 0), 32);
    const int32_t b = min(max(hi - gp, 0), 32);
    const uint64_t m = ((1ull << b) - 1ull) & ~((1ull << a) - 1ull);
    return b > a ? (uint32_t)m : 0u;
}

__device__ __forceinline__ uint32_t zero_bits(uint32_t x) { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u; }
__device__ __forceinline__ uint32_t compress4(uint32_t m) {   /* bits 7, 15, 23, 31 -> bits 0-3 */
    m >>= 7;
    m |= m >> 7;
    m |= m >> 14;
    return m & 0xFu;
}
__device__ __forceinline__ uint32_t nul_mask16(uint4 v) {
    return compress4(zero_bits(v.x)) | (compress4(zero_bits(v.y)) << 4) | (compress4(zero_bits(v.z)) << 8) |
           (compress4(zero_bits(v.w)) << 12);
}

__device__ __forceinline__ uint32_t runi(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)runi((uint32_t)(x >> 32)) << 32) | runi((uint32_t)x);
}
constexpr int32_t FAR = 0x3FFFFFFF;
/* group-relative offset of an absolute position, clamped to [-32, FAR] */
__device__ __forceinline__ int32_t relpos(uint64_t x, uint64_t base) {
    if (x < base) return (base - x) >= 32 ? -32 : -(int32_t)(base - x);
    return (x - base) >= (uint64_t)FAR ? FAR : (int32_t)(x - base);
}

/* ---- the bucketed LDS count table (as tokcount_lean.hip) ---- */
__device__ __forceinline__ uint32_t bkt_hash(uint32_t key) {
    return (uint32_t)__umul24((key ^ (key >> 15)) & 0xFFFFu, NB) >> 16;   /* [0, NB) */
}
__device__ __forceinline__ uint32_t bkt_next(uint32_t b) { return b + 1 == NB ? 0u : b + 1; }
__device__ __forceinline__ uint4 bkt_read(WShared& S, uint32_t b) { return reinterpret_cast<const uint4*>(S.TK)[b]; }
__device__ __forceinline__ uint32_t bkt_match(const uint4& kk, uint32_t key) {
    return kk.x == key ? 0u : kk.y == key ? 1u : kk.z == key ? 2u : kk.w == key ? 3u : 4u;
}
__device__ __forceinline__ uint32_t bkt_empty(const uint4& kk, uint32_t key) {
    const uint32_t em = (kk.x == 0u ? 1u : 0u) | (kk.y == 0u ? 2u : 0u) | (kk.z == 0u ? 4u : 0u) | (kk.w == 0u ? 8u : 0u);
    if (!em) return BW;
    const uint32_t r0 = key & (BW - 1u);
    const uint32_t rot = ((em | (em << BW)) >> r0) & ((1u << BW) - 1u);
    return ((uint32_t)__builtin_ctz(rot) + r0) & (BW - 1u);
}

__device__ __forceinline__ uint32_t claim_chunk(unsigned long long* ctr, uint32_t& sh, uint32_t n) {
#pragma unroll 1
    for (int t = 0; t < 8; ++t) {
        const uint32_t lo = (uint32_t)((uint64_t)n * sh / 8), hi = (uint32_t)((uint64_t)n * (sh + 1) / 8);
        if (hi > lo) {
            const uint64_t v = atomicAdd(&ctr[sh], 1ull);
            if (lo + v < hi) return lo + (uint32_t)v;
        }
        sh = (sh + 1) & 7u;
    }
    return n;
}

/* term slot of a token whose term is >= 16 bytes: re-read from HBM (rare for text) */
__device__ __noinline__ uint32_t win_long_slot(const LeanParams* P, uint64_t p0, uint64_t dend) {
    const uint8_t* __restrict__ bytes = P->c.bytes;
    uint64_t p = p0;
    while (p < dend && !is_ws(bytes[p])) ++p;
    uint64_t n = 0;
    while (p0 + n < p && bytes[p0 + n] != 0) ++n;
    uint64_t klo, khi;
    if (n < 16) {   /* a NUL inside the first 16 bytes: a short term after all */
        uint64_t lo = 0, hi = 0;
        for (uint32_t k = 0; k < n; ++k) {
            const uint64_t b = bytes[p0 + k];
            if (k < 8) lo |= b << (8 * k); else hi |= b << (8 * (k - 8));
        }
        make_short_key(lo, hi, (uint32_t)n, &klo, &khi);
        return vocab_insert_s(P->v.keys, P->v.rep, P->v.mask, klo, khi, 0, P->o.status);
    }
    make_long_key(bytes + p0, n, &klo, &khi);
    /* rep = (length << 40) | offset holds 24 length bits (TFIDF_E_CAPACITY beyond) */
    if (n >= 0xFFFFFFull) atomicOr(P->o.status, ST_TERM_LONG);
    const uint64_t rep = ((n < 0xFFFFFFull ? n : 0xFFFFFFull) << 40) | p0;
    return vocab_insert_s(P->v.keys, P->v.rep, P->v.mask, klo, khi, rep, P->o.status);
}
__device__ __noinline__ uint32_t win_insert(const LeanParams* P, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
    return vocab_insert_s(P->v.keys, P->v.rep, P->v.mask, ((uint64_t)k1 << 32) | k0, ((uint64_t)k3 << 32) | k2, 0,
                          P->o.status);
}

__device__ __forceinline__ void overflow_record(const LeanParams* P, uint32_t doc, uint32_t slot) {
    const uint64_t am = __ballot(1);   /* one device atomic per wave and call */
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
    unsigned long long b = 0;
    if (rank == 0u) b = atomicAdd(P->o.part_alloc, (unsigned long long)__popcll(am));
    const unsigned long long q = uni64(b) + rank;
    if (q < P->o.part_cap) { P->o.part_doc[q] = doc; P->o.part_slot[q] = slot; P->o.part_cnt[q] = 1u; }
    else atomicOr(P->o.status, ST_PART_FULL);
}

/* Counts `key` the slow way, from bucket b on (home bucket full, a lost claim, or overflow
 * mode).  Returns 1 when this call claimed a slot.  A key not in the table in overflow
 * mode, or after PMAX buckets, becomes a partial record of count 1. */
constexpr int PMAX = 16;
__device__ __noinline__ uint32_t bkt_slow(WShared& S, const LeanParams* P, uint32_t key, uint32_t b, bool over,
                                          uint32_t gd0, uint32_t sb) {
    for (int probe = 0, tries = 0; probe < PMAX && tries < 64; ++tries) {
        const uint4 kk = bkt_read(S, b);
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
    overflow_record(P, gd0 + rel, key & ((1u << sb) - 1u));
    return 0u;
}

__device__ __forceinline__ void wave_agg_add(uint32_t* ctr, uint32_t idx) {
    const uint32_t i0 = runi(idx);
    const uint64_t am = __ballot(1);
    if (__ballot(idx != i0) == 0ull) {
        if (__builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u)) == 0u)
            atomicAdd(&ctr[i0], (uint32_t)__popcll(am));
    } else {
        atomicAdd(&ctr[idx], 1u);
    }
}
__device__ __forceinline__ uint32_t wave_agg_add_rtn(uint32_t* ctr, uint32_t idx) {
    const uint32_t i0 = runi(idx);
    const uint64_t am = __ballot(1);
    uint32_t k;
    if (__ballot(idx != i0) == 0ull) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
        uint32_t b = 0;
        if (rank == 0u) b = atomicAdd(&ctr[i0], (uint32_t)__popcll(am));
        k = runi(b) + rank;
    } else {
        k = atomicAdd(&ctr[idx], 1u);
    }
    return k;
}

/* Emits every table entry of the group as a record and clears the table (any number of
 * documents): per-document counts, a block scan, then every entry straight to its slot. */
__device__ __forceinline__ void win_flush(WShared& S, const LeanParams* P, uint32_t gd0, uint32_t ng, uint64_t cs,
                                          uint64_t ce, uint32_t sb) {
    const int tid = threadIdx.x;
    if (tid < GCAP) { S.f.dcnt[tid] = 0; S.f.drun[tid] = 0; }
    lds_barrier();
    const uint32_t smask = (1u << sb) - 1u;
    for (int j = 0; j < EPT; ++j) {
        const uint32_t k = S.TK[j * NT + tid];
        if (k) wave_agg_add(&S.f.dcnt[0], (k & 0x7FFFFFFFu) >> sb);
    }
    lds_barrier();
    uint32_t packed = 0;
    if ((uint32_t)tid < ng) {
        uint8_t st = 0;
        const uint32_t cnt = S.f.dcnt[tid];
        const bool part = S.dpart[tid] != 0;
        if (cnt) {
            const bool complete = !part && S.gdoc[tid] >= cs && S.gdoc[tid + 1] <= ce && cnt <= (uint32_t)K5_MAX_PAIRS;
            st = complete ? 2 : 1;
            packed = complete ? cnt : (cnt << 16);
        }
        if (st == 1 || part) P->o.doc_flags[gd0 + tid] = DF_PARTIAL;
        S.f.dstate[tid] = st;
    }
    uint32_t tot;
    const uint32_t off = block_excl_scan<NT, true>(packed, S.wsum, &tot);
    if ((uint32_t)tid < ng) S.f.doff[tid] = off;
    const uint32_t nrec = tot & 0xFFFFu, npart = tot >> 16;
    if (tid == 0) {
        const unsigned long long rb = nrec ? atomicAdd(P->o.rec_alloc, (unsigned long long)nrec) : 0ull;
        if (rb + nrec > P->o.rec_cap) atomicOr(P->o.status, ST_REC_FULL);
        S.rec_base = rb;
    } else if (tid == 64) {
        const unsigned long long pb = npart ? atomicAdd(P->o.part_alloc, (unsigned long long)npart) : 0ull;
        if (pb + npart > P->o.part_cap) atomicOr(P->o.status, ST_PART_FULL);
        S.part_base = pb;
    }
    lds_barrier();
    const unsigned long long rb = S.rec_base, pb = S.part_base;
    const bool rec_ok = rb + nrec <= P->o.rec_cap, part_ok = pb + npart <= P->o.part_cap;
    if ((uint32_t)tid < ng && S.f.dstate[tid] == 2) {
        P->o.doc_recoff[gd0 + tid] = rb + (off & 0xFFFFu);
        P->o.doc_npairs[gd0 + tid] = S.f.dcnt[tid];
    }
    uint32_t* const rec_slot = P->o.rec_slot;
    uint32_t* const rec_cnt = P->o.rec_cnt;
    for (int j = 0; j < EPT; ++j) {
        const uint32_t key = S.TK[j * NT + tid];
        if (key) {
            const uint32_t c = S.TC[j * NT + tid];
            const uint32_t rel = (key & 0x7FFFFFFFu) >> sb;
            const uint32_t k = wave_agg_add_rtn(&S.f.drun[0], rel);
            const uint32_t dof = S.f.doff[rel];
            if (S.f.dstate[rel] == 2) {
                const uint64_t q = rb + (dof & 0xFFFFu) + k;
                if (rec_ok) { rec_slot[q] = key & smask; rec_cnt[q] = c; }
            } else {
                const uint64_t q = pb + (dof >> 16) + k;
                if (part_ok) { P->o.part_doc[q] = gd0 + rel; P->o.part_slot[q] = key & smask; P->o.part_cnt[q] = c; }
            }
            S.TK[j * NT + tid] = 0u;
            S.TC[j * NT + tid] = 0u;
        }
    }
}

/* The flush of a group of at most FEW documents (most c2 chunks hold one or two): 16-bit
 * per-document counters per thread, one block scan, no LDS atomics.  Same output. */
constexpr uint32_t FEW = 8;
__device__ __forceinline__ void win_flush_few(WShared& S, const LeanParams* P, uint32_t gd0, uint32_t ng, uint64_t cs,
                                              uint64_t ce, uint32_t sb) {
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    const uint32_t smask = (1u << sb) - 1u;
    uint32_t pk[FEW / 2] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const uint32_t k = S.TK[j * NT + tid];
        if (k) {
            const uint32_t rel = (k & 0x7FFFFFFFu) >> sb;
#pragma unroll
            for (uint32_t q = 0; q < FEW / 2; ++q)
                pk[q] += (rel >> 1) == q ? (1u << (16 * (rel & 1u))) : 0u;
        }
    }
    uint32_t inc[FEW / 2];
#pragma unroll
    for (uint32_t q = 0; q < FEW / 2; ++q) {
        inc[q] = wave_incl_scan(pk[q]);
        if (lane == 63) S.f.dcnt[w * (FEW / 2) + q] = inc[q];
    }
    lds_barrier();
    uint32_t rank[FEW / 2], tot[FEW / 2];
#pragma unroll
    for (uint32_t q = 0; q < FEW / 2; ++q) {
        uint32_t base = 0, t = 0;
#pragma unroll
        for (int k = 0; k < NWAVE; ++k) {
            const uint32_t x = S.f.dcnt[k * (FEW / 2) + q];
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
                const bool complete = !part && S.gdoc[d] >= cs && S.gdoc[d + 1] <= ce && cnt <= (uint32_t)K5_MAX_PAIRS;
                st = complete ? 2 : 1;
                packed = complete ? cnt : (cnt << 16);
            }
            if (st == 1 || part) P->o.doc_flags[gd0 + d] = DF_PARTIAL;
        }
        const uint32_t incl = wave_incl_scan(packed);
        const uint32_t all = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t off = incl - packed;
        const uint32_t nrec = all & 0xFFFFu, npart = all >> 16;
        unsigned long long a0 = 0, a1 = 0;
        if (lane == 0 && nrec) a0 = atomicAdd(P->o.rec_alloc, (unsigned long long)nrec);
        if (lane == 32 && npart) a1 = atomicAdd(P->o.part_alloc, (unsigned long long)npart);
        const unsigned long long rb = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(a0 >> 32), 0) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a0, 0);
        const unsigned long long pb = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(a1 >> 32), 32) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a1, 32);
        const bool rec_ok = rb + nrec <= P->o.rec_cap, part_ok = pb + npart <= P->o.part_cap;
        if (lane == 0 && !rec_ok) atomicOr(P->o.status, ST_REC_FULL);
        if (lane == 0 && !part_ok) atomicOr(P->o.status, ST_PART_FULL);
        if (d < ng) {
            uint64_t fb = ~0ull;
            if (st == 2) {
                fb = rec_ok ? rb + (off & 0xFFFFu) : ~0ull;
                P->o.doc_recoff[gd0 + d] = rb + (off & 0xFFFFu);
                P->o.doc_npairs[gd0 + d] = cnt;
            } else if (st == 1) {
                fb = part_ok ? pb + (off >> 16) : ~0ull;
            }
            S.fbase[d] = fb;
            S.f.dstate[d] = st;
        }
    }
    lds_barrier();
    uint32_t* const rec_slot = P->o.rec_slot;
    uint32_t* const rec_cnt = P->o.rec_cnt;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const uint32_t key = S.TK[j * NT + tid];
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
                if (S.f.dstate[rel] == 2) { rec_slot[qq] = key & smask; rec_cnt[qq] = S.TC[j * NT + tid]; }
                else { P->o.part_doc[qq] = gd0 + rel; P->o.part_slot[qq] = key & smask; P->o.part_cnt[qq] = S.TC[j * NT + tid]; }
            }
            S.TK[j * NT + tid] = 0u;
            S.TC[j * NT + tid] = 0u;
        }
    }
}

/* v_perm selector dword k of a term of length n */
__device__ __forceinline__ uint32_t perm_sel(uint32_t n, uint32_t k) {
    uint32_t s = 0;
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t p = 4 * k + j;
        const uint32_t b = p < n ? j : (p == n ? 4u : 12u);
        s |= b << (8 * j);
    }
    return s;
}

/* index of the group document containing window offset pos when two documents of the
 * window start at one position (empty documents): the last k < ng with gdoc[k] <= abs */
__device__ __noinline__ uint32_t doc_of_pos(const WShared& S, uint32_t ng, uint64_t abs) {
    uint32_t lo = 0, hi = ng;   /* gdoc[lo] <= abs (the token is owned), answer in [lo, hi) */
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (S.gdoc[mid] <= abs) lo = mid; else hi = mid;
    }
    return lo;
}

}  // namespace

__global__ __launch_bounds__(NT, WG_PER_CU) void k_tokcount_win(const LeanParams* __restrict__ Pg,
                                                              const uint8_t* __restrict__ bytes,
                                                              const uint4* __restrict__ vkeys, uint32_t vmask,
                                                              uint32_t sb, uint32_t gcap, uint32_t nchunk,
                                                              uint64_t c_lo, uint64_t c_hi, uint64_t last_blk) {
    __shared__ __attribute__((aligned(16))) WShared S;
    const LeanParams* P = Pg;
    asm volatile("" : "+s"(P));
    const int tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const int32_t seg0 = 32 * tid;           /* this thread's first byte, window-relative */

    for (int j = 0; j < EPT; ++j) { S.TK[j * NT + tid] = 0u; S.TC[j * NT + tid] = 0u; }
    S.dsb[tid] = 0u;
    if (tid == 0) { S.dsb[NT] = 0u; S.dup = 0u; S.fill = 0u; }
    if (tid < 64) {
        const uint32_t n = (uint32_t)tid >> 2, k = (uint32_t)tid & 3u;
        (&S.sel[n].x)[k] = perm_sel(n, k);
    }
    uint32_t tokens_wg = 0;

    /* the window loads: 32 bytes per thread, plus the head (thread 0) and the tail (thread
     * 255); addresses past the corpus read its last block (masked as outside the shard) */
    auto load_win = [&](uint64_t base, uint4& a, uint4& b, uint4& x) {
        const uint64_t pa = base + (uint64_t)seg0;
        a = ld16(bytes + (pa < last_blk ? pa : last_blk));
        b = ld16(bytes + (pa + 16 < last_blk ? pa + 16 : last_blk));
        x = make_uint4(0, 0, 0, 0);
        if (tid == 0) { const uint64_t h = base - 16; x = ld16(bytes + (h < last_blk ? h : last_blk)); }
        if (tid == NT - 1) { const uint64_t t = base + W; x = ld16(bytes + (t < last_blk ? t : last_blk)); }
    };

    uint32_t shard = blockIdx.x & 7u;
    if (tid == 0) {
        unsigned long long* ctr = P->o.chunk_shard;
        S.cur_chunk = claim_chunk(ctr, shard, nchunk);
        S.nxt_chunk = claim_chunk(ctr, shard, nchunk);
    }
    lds_barrier();
    uint4 pA = make_uint4(0, 0, 0, 0), pB = pA, pX = pA;   /* the next window, in flight */
    uint64_t pfb = ~0ull;                 /* window base pA/pB/pX were loaded for */
    uint64_t dpre = 0;                    /* doc_off[dfirst + tid] of this chunk, fetched during the previous one */
    bool dpre_ok = false;
    unsigned long long pend_v = 0;
    uint32_t chunk = runi(S.cur_chunk), nxt = runi(S.nxt_chunk);
    uint64_t cs = 0, ce = 0;
    uint32_t dfirst = 0, dlast = 0;
    if (chunk < nchunk) {
        cs = uni64(P->chunk_start[chunk]);
        ce = uni64(P->chunk_start[chunk + 1]);
        dfirst = runi(P->chunk_doc[chunk]);
        dlast = runi(P->chunk_doc[chunk + 1]);
    }
    while (chunk < nchunk) {
        if (tid == 0) pend_v = atomicAdd(&P->o.chunk_shard[shard], 1ull);
        uint64_t ncs = 0, nce = 0;
        uint32_t ndf = 0, ndl = 0;
        if (nxt < nchunk) {
            ncs = uni64(P->chunk_start[nxt]);
            nce = uni64(P->chunk_start[nxt + 1]);
            ndf = runi(P->chunk_doc[nxt]);
            ndl = runi(P->chunk_doc[nxt + 1]);
        }
        if (cs < ce)
        for (uint32_t gd0 = dfirst; gd0 <= dlast; gd0 += gcap) {
            const uint32_t ng = (dlast + 1 - gd0) < gcap ? (dlast + 1 - gd0) : gcap;
            if (gd0 == dfirst && dpre_ok) {
                if ((uint32_t)tid <= ng) S.gdoc[tid] = dpre;
            } else {
                const uint64_t* doff = P->c.doc_off;
                if ((uint32_t)tid <= ng) S.gdoc[tid] = doff[gd0 + tid];
            }
            dpre_ok = false;
            if (tid < GCAP) { S.dsz[tid] = 0; S.dpart[tid] = 0; }
            if (tid == 0) S.fill = 0;
            lds_barrier();
            const bool last_group = gd0 + gcap > dlast;
            const bool ahead = last_group && nxt < nchunk && ncs < nce;   /* prefetch for the next chunk */
            const uint64_t g0 = uni64(S.gdoc[0]), gn = uni64(S.gdoc[ng]);
            const uint64_t gs = g0 > cs ? g0 : cs;
            const uint64_t ge = gn < ce ? gn : ce;
            if (gs < ge) {
                const uint64_t b0 = gs & ~(uint64_t)15;          /* group base: window k owns [b0 + W k, +W) */
                const uint32_t nw = (uint32_t)((ge - b0 + W - 1) / W);
                const int32_t own_lo = (int32_t)(gs - b0), own_hi = (int32_t)(ge - b0);
                const int32_t rlo = relpos(c_lo, b0), rhi = relpos(c_hi, b0);
                int32_t wr = g0 >= b0 ? -1 : 0;                  /* document containing the window's first byte */
                const uint64_t gtok = tid <= (int)ng ? S.gdoc[tid] : 0ull;   /* this thread's document start */
                for (uint32_t w = 0; w < nw; ++w) {
                    const uint64_t ws = b0 + (uint64_t)w * W;
                    const int32_t wsr = (int32_t)(w * W);
                    uint4 A, B, X;
                    if (ws == pfb) { A = pA; B = pB; X = pX; }
                    else load_win(ws, A, B, X);
                    S.wb[1 + 2 * tid] = A;
                    S.wb[2 + 2 * tid] = B;
                    if (tid == 0) S.wb[0] = X;
                    if (tid == NT - 1) S.wb[1 + W / 16] = X;
                    /* document starts in [ws, ws + W + 16): bits (the group end ends terms too) */
                    if ((uint32_t)tid <= ng && gtok >= ws && gtok < ws + W + 16) {
                        const uint32_t p = (uint32_t)(gtok - ws);
                        const uint32_t bit = 1u << (p & 31u);
                        if (atomicOr(&S.dsb[p >> 5], bit) & bit) S.dup = 1u;
                    }
                    /* the next window: in this group, or the next chunk's first */
                    {
                        uint64_t na = ~0ull;
                        if (w + 1 < nw) na = ws + W;
                        else if (ahead) na = ncs & ~(uint64_t)15;
                        if (na != ~0ull) load_win(na, pA, pB, pX);
                        pfb = na;
                    }
                    lds_barrier();                                   /* B1: window bytes, start bits */
                    const bool dupw = S.dup != 0u;
                    /* ---- classify this thread's 32 bytes ---- */
                    const int32_t rlo_w = rlo - wsr, rhi_w = rhi - wsr;
                    const int32_t olo_w = own_lo - wsr, ohi_w = own_hi - wsr;
                    uint32_t wsm = ws_mask16_swar(A) | (ws_mask16_swar(B) << 16);
                    const bool in_shard = rlo_w <= -16 && rhi_w >= (int32_t)W + 16;   /* block-uniform */
                    if (!in_shard) wsm |= ~in_mask32(seg0, rlo_w, rhi_w);
                    uint32_t nul = 0;
                    if (__ballot((zero_bits(A.x) | zero_bits(A.y) | zero_bits(A.z) | zero_bits(A.w) | zero_bits(B.x) |
                                  zero_bits(B.y) | zero_bits(B.z) | zero_bits(B.w)) != 0u) != 0ull)
                        nul = nul_mask16(A) | (nul_mask16(B) << 16);
                    const uint32_t ds = S.dsb[tid];
                    S.dsb[tid] = 0u;
                    const uint32_t pbyte = reinterpret_cast<const uint8_t*>(S.wb)[16 + seg0 - 1];
                    const bool pws = is_ws(pbyte) || seg0 - 1 < rlo_w || seg0 - 1 >= rhi_w;
                    uint32_t own = 0xFFFFFFFFu;
                    if (!(olo_w <= 0 && ohi_w >= (int32_t)W)) own = in_mask32(seg0, olo_w, ohi_w);
                    const uint32_t starts = ~wsm & ((wsm << 1) | (pws ? 1u : 0u) | ds) & own;
                    const uint32_t stop = wsm | ds | nul;            /* a term ends here */
                    const uint32_t v = (uint32_t)__popc(starts) | ((uint32_t)__popc(ds) << 16);
                    const uint32_t inc = wave_incl_scan(v);
                    if (lane == 63) S.wsum[wid] = inc;
                    if (lane == 0) S.xs[wid] = stop;
                    if (tid == NT - 1) {   /* the tail's 16 bytes end terms only */
                        uint32_t t = ws_mask16_swar(X) | nul_mask16(X) | (S.dsb[NT] & 0xFFFFu) | 0xFFFF0000u;
                        if (!in_shard) t |= ~in_mask32((int32_t)W, rlo_w, rhi_w);
                        S.xs[NWAVE] = t;
                        S.dsb[NT] = 0u;
                    }
                    lds_barrier();                                   /* B2: scan sums, edge masks */
                    if (tid == 0) S.dup = 0u;
                    uint32_t base = 0, tot = 0;
#pragma unroll
                    for (int k = 0; k < NWAVE; ++k) {
                        const uint32_t s = S.wsum[k];
                        base += k < (int)wid ? s : 0u;
                        tot += s;
                    }
                    const uint32_t excl = base + inc - v;
                    const uint32_t tokbase = excl & 0xFFFFu, dsbase = excl >> 16;
                    const uint32_t ntok_w = tot & 0xFFFFu, nds_w = tot >> 16;
                    const uint32_t xnext = S.xs[wid + 1];
                    /* the DPP shift under the full exec mask: in a `lane == 63 ? ... :` branch lane 62
                     * would read a disabled lane 63 and keep its own value */
                    const uint32_t shl = lane_next(stop);
                    const uint32_t nstop = lane == 63 ? xnext : shl;
                    const uint64_t stop64 = ((uint64_t)nstop << 32) | stop;
                    const bool tok_dsz = nds_w != 0u || dupw;          /* docSize per token */
                    if (!tok_dsz && tid == 0 && ntok_w) S.dsz[wr] += ntok_w;
                    if (tid == 0) tokens_wg += ntok_w;
                    for (uint32_t pass0 = 0; pass0 < ntok_w; pass0 += LCAP) {
                        /* ---- token entries of this pass ---- */
                        uint32_t sm = starts, idx = tokbase;
                        while (sm) {
                            const uint32_t i = (uint32_t)__builtin_ctz(sm);
                            sm &= sm - 1u;
                            if (idx - pass0 < LCAP) {
                                const uint32_t e = ((uint32_t)(stop64 >> i) & 0xFFFEu) | ((nul >> i) & 1u);
                                const uint32_t len = (uint32_t)__builtin_ctz(e | 0x10000u);   /* 16: long */
                                uint32_t rel;
                                if (!dupw) rel = (uint32_t)(wr + (int32_t)dsbase + __popc(ds & ((2u << i) - 1u)));
                                else rel = doc_of_pos(S, ng, ws + (uint64_t)(seg0 + (int32_t)i));
                                if (tok_dsz) atomicAdd(&S.dsz[rel], 1u);
                                S.list[idx - pass0] = (uint32_t)(seg0 + (int32_t)i) | (len << 13) | (rel << 18);
                            }
                            ++idx;
                        }
                        lds_barrier();                               /* B3: the list */
                        const uint32_t n = (ntok_w - pass0) < LCAP ? (ntok_w - pass0) : LCAP;
                        /* ---- resolve + count, BATCH tokens per thread at a time ---- */
                        for (uint32_t j0 = 0; j0 < n; j0 += NT * BATCH) {
                            uint32_t ent[BATCH], hv[BATCH], k0[BATCH], k1[BATCH], k2[BATCH], k3[BATCH];
                            uint4 s4[BATCH], t4[BATCH];
                            /* in phases, so that every LDS read of a phase is in flight together (the
                             * compiler does not move LDS reads across the dependent ones of another
                             * token): entries; term bytes + selectors; keys, hashes and slot loads */
#pragma unroll
                            for (int b = 0; b < BATCH; ++b) {
                                const uint32_t j = j0 + (uint32_t)(b * NT + tid);
                                const uint32_t e = S.list[j < LCAP ? j : LCAP - 1];
                                ent[b] = j < n ? e : ENT_NONE;
                            }
                            u32x4u raw[BATCH];
                            uint4 sl[BATCH];
#pragma unroll
                            for (int b = 0; b < BATCH; ++b) {
                                const uint32_t p = ent[b] & 8191u;           /* ENT_NONE: a harmless read */
                                raw[b] = *reinterpret_cast<const u32x4u*>(reinterpret_cast<const uint8_t*>(S.wb) + 16 + p);
                                sl[b] = S.sel[(ent[b] >> 13) & 15u];         /* a long term builds a junk key */
                            }
#pragma unroll
                            for (int b = 0; b < BATCH; ++b) {
                                k0[b] = __builtin_amdgcn_perm(0x09090909u, raw[b].x, sl[b].x);
                                k1[b] = __builtin_amdgcn_perm(0x09090909u, raw[b].y, sl[b].y);
                                k2[b] = __builtin_amdgcn_perm(0x09090909u, raw[b].z, sl[b].z);
                                k3[b] = __builtin_amdgcn_perm(0x09090909u, raw[b].w, sl[b].w);
                                hv[b] = (uint32_t)key_hash(((uint64_t)k1[b] << 32) | k0[b], ((uint64_t)k3[b] << 32) | k2[b]) & vmask;
                                s4[b] = gload(vkeys + hv[b]);
                                t4[b] = gload(vkeys + ((hv[b] + 1) & vmask));
                            }
                            /* slots: the home or the next one; the rare paths (a miss: insert; a term
                             * of >= 16 bytes) behind one wave-uniform branch per batch */
                            uint32_t key[BATCH], slot[BATCH], rare = 0;
#pragma unroll
                            for (int b = 0; b < BATCH; ++b) {
                                const uint32_t len = (ent[b] >> 13) & 31u;
                                /* the or-chains stay one VGPR each (else they become four compares
                                 * and scalar mask arithmetic per slot) */
                                uint32_t d0 = (s4[b].x ^ k0[b]) | (s4[b].y ^ k1[b]) | (s4[b].z ^ k2[b]) | (s4[b].w ^ k3[b]);
                                uint32_t d1 = (t4[b].x ^ k0[b]) | (t4[b].y ^ k1[b]) | (t4[b].z ^ k2[b]) | (t4[b].w ^ k3[b]);
                                asm volatile("" : "+v"(d0), "+v"(d1));
                                slot[b] = d0 == 0u ? hv[b] : ((hv[b] + 1) & vmask);
                                const uint32_t miss = (d0 != 0u && d1 != 0u) || len == LEN_LONG ? 1u : 0u;
                                rare |= (ent[b] != ENT_NONE ? miss : 0u) << b;
                            }
                            if (__ballot(rare != 0u) != 0ull) {
                                if (rare) {
                                    const LeanParams* Q = P;
                                    asm volatile("" : "+s"(Q));
#pragma unroll
                                    for (int b = 0; b < BATCH; ++b)
                                        if ((rare >> b) & 1u)
                                            slot[b] = ((ent[b] >> 13) & 31u) == LEN_LONG
                                                ? win_long_slot(Q, ws + (ent[b] & 8191u), S.gdoc[(ent[b] >> 18) + 1])
                                                : win_insert(Q, k0[b], k1[b], k2[b], k3[b]);
                                }
                            }
#pragma unroll
                            for (int b = 0; b < BATCH; ++b)
                                key[b] = (ent[b] != ENT_NONE && slot[b] != INVALID_SLOT)
                                    ? (0x80000000u | ((ent[b] >> 18) << sb) | slot[b]) : 0u;
                            /* ---- count: every bucket read first ---- */
                            const bool over = S.fill >= FILL_LIMIT;
                            uint4 kk[BATCH];
#pragma unroll
                            for (int b = 0; b < BATCH; ++b) kk[b] = bkt_read(S, bkt_hash(key[b]));
                            uint32_t claims = 0, slowm = 0;
#pragma unroll
                            for (int b = 0; b < BATCH; ++b) {
                                const uint32_t bk = bkt_hash(key[b]);
                                if (key[b]) {
                                    const uint32_t j = bkt_match(kk[b], key[b]);
                                    if (j < BW) {
                                        atomicAdd(&S.TC[BW * bk + j], 1u);
                                    } else {
                                        const uint32_t e = bkt_empty(kk[b], key[b]);
                                        if (e < BW && !over) {
                                            const uint32_t old = atomicCAS(&S.TK[BW * bk + e], 0u, key[b]);
                                            if (old == 0u || old == key[b]) {
                                                atomicAdd(&S.TC[BW * bk + e], 1u);
                                                claims += old == 0u ? 1u : 0u;
                                            } else {
                                                slowm |= 1u << b;
                                            }
                                        } else {
                                            slowm |= 1u << b;
                                        }
                                    }
                                }
                            }
                            if (__ballot(slowm != 0u) != 0ull) {   /* full home bucket, lost claim, overflow */
                                if (slowm) {
                                    const LeanParams* Q = P;
                                    asm volatile("" : "+s"(Q));
#pragma unroll
                                    for (int b = 0; b < BATCH; ++b)
                                        if ((slowm >> b) & 1u) claims += bkt_slow(S, Q, key[b], bkt_hash(key[b]), over, gd0, sb);
                                }
                            }
                            const uint32_t wc = wave_sum(claims);
                            if (wc && lane == 0) (void)atomicAdd(&S.fill, wc);
                        }
                        lds_barrier();                               /* B4: list, window bytes free */
                    }
                    if (ntok_w == 0u) lds_barrier();
                    if (!dupw) wr += (int32_t)nds_w;
                    else wr = (int32_t)doc_of_pos(S, ng, ws + W - 1) - (g0 >= ws + W ? 1 : 0);
                }
            }
            if (ahead) {   /* the next chunk's document offsets, in flight during this flush */
                const uint32_t nng = (ndl + 1 - ndf) < gcap ? (ndl + 1 - ndf) : gcap;
                dpre = (uint32_t)tid <= nng ? P->c.doc_off[ndf + tid] : 0ull;
                dpre_ok = true;
            }
            lds_barrier();   /* the window state aliases the flush's */
            if (ng <= FEW) win_flush_few(S, P, gd0, ng, cs, ce, sb);
            else win_flush(S, P, gd0, ng, cs, ce, sb);
            if ((uint32_t)tid < ng) {
                const uint32_t n = S.dsz[tid];
                if (n) {
                    const uint32_t d = gd0 + tid;
                    if (S.gdoc[tid] >= cs && S.gdoc[tid + 1] <= ce) P->o.doc_size[d] = n;
                    else atomicAdd(&P->o.doc_size[d], n);
                }
            }
            lds_barrier();
            if (gd0 + gcap < gd0) break; /* overflow guard */
        }
        if (tid == 0) {
            const uint32_t lo = (uint32_t)((uint64_t)nchunk * shard / 8), hi = (uint32_t)((uint64_t)nchunk * (shard + 1) / 8);
            const uint32_t claim = lo + pend_v < hi ? lo + (uint32_t)pend_v : claim_chunk(P->o.chunk_shard, shard, nchunk);
            S.cur_chunk = nxt;
            S.nxt_chunk = claim;
        }
        lds_barrier();
        chunk = nxt;
        nxt = runi(S.nxt_chunk);
        cs = ncs;
        ce = nce;
        dfirst = ndf;
        dlast = ndl;
    }
    if (tid == 0 && tokens_wg) atomicAdd(P->o.ntokens, (unsigned long long)tokens_wg);
}

int launch_tokcount_win(const LeanParams* dparams, const LeanParams& h, hipStream_t s) {
    if (h.c1 <= h.c0) return 0;
    if (h.c0 != 0 || h.c1 > 0xFFFFFFFFull) return -3;   /* chunk indices are 32-bit here */
    if (h.v.mask >= (1ull << 24)) return -3;             /* slot + 7 document bits fit the LDS entry */
    static_assert(sizeof(WShared) * WG_PER_CU <= 163840, "LDS of WG_PER_CU workgroups per CU");
    static_assert(TB % NT == 0 && TB % BW == 0, "table rows");
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const uint64_t n = h.c1 - h.c0;
    const uint64_t wgs = (uint64_t)ncu * WG_PER_CU;
    const uint64_t grid = n < wgs ? n : wgs;
    const uint32_t sb = (uint32_t)__builtin_popcountll(h.v.mask);
    const uint32_t gcap = (1u << (31u - sb)) >= (uint32_t)GCAP ? (uint32_t)GCAP : (1u << (31u - sb));
    const uint64_t last_blk = h.c.nbytes ? ((h.c.nbytes - 1) & ~(uint64_t)15) : 0;
    k_tokcount_win<<<(unsigned)grid, NT, 0, s>>>(dparams, h.c.bytes, h.v.keys, (uint32_t)h.v.mask, sb, gcap,
                                                 (uint32_t)n, h.c.lo, h.c.hi, last_blk);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
