/*
 * tokcount_lean.hip — K1: fused tokenize + per-document term counting, written for a
 * small register footprint.  Replaces the reference's per-rank hot loop TFIDF.c:130-196:
 * fscanf("%s") tokenising (:141-147), the O(P) strcmp search/append of (word, doc)
 * records (:151-167) and the per-rank word table (:169-188).
 *
 * Algorithm (the one of tokcount_st.hip, restructured):
 *   chunks    a persistent grid takes K0's chunks (~16 KiB of whole documents, or a piece
 *             of a document longer than BIG_DOC) from 8 sharded counters; a chunk's
 *             documents are processed in groups of <= gcap; inside a group the four waves
 *             run without block barriers, wave w taking the 992-byte steps w, w+4, ...
 *   walk      per step each lane loads 16 bytes (lane 0: the 16 before the step, lane 63:
 *             the 16 after), stores them in the wave's LDS stage, classifies them (SWAR
 *             C-locale isspace, TFIDF.c:142,147; NUL ends a term, strcmp :152,172) and
 *             writes one 32-bit entry per token start (stage offset | term length |
 *             document in group).  docSize (TFIDF.c:141-143) is the number of token starts:
 *             one LDS add per step (per token only in a step that holds a document start).
 *   rounds    64 tokens per wave round: one unaligned ds_read_b128 of the term, four
 *             v_perm_b32 build the exact 128-bit identity key (dev_common.h), a 32-bit hash,
 *             the home vocabulary slot and the next one loaded at once; the next round's
 *             loads are issued before this round is counted in the bucketed LDS table
 *             (one ds_read_b128 of the home bucket, add or claim-by-CAS).
 *   flush     once per group: every (document, slot) entry becomes a record (complete
 *             documents) or a partial record (documents split across groups / chunks or
 *             overflowing the table), merged later by finalize.hip.
 *
 * What is different from tokcount_st.hip, and why: the scalar register file.  That kernel
 * held every kernel argument (about 66 SGPRs of pointers and sizes), 64-bit positions and
 * the chunk state live across its loops; 106 SGPRs with 131 spilled to VGPR lanes, and the
 * reloads (v_readlane, a VALU instruction each, plus the s_nop they need) were a large
 * share of its ~1000 VALU instructions per 992-byte step.  Here
 *   - pointers used only by the flush and the rare paths (record arrays, counters, the
 *     vocabulary's long-term table, the status word) are read from a parameter block in
 *     device memory (LeanParams) where they are used: scalar loads, nothing held;
 *   - positions inside a group are 32-bit offsets from the group's 16-byte aligned base;
 *   - rare paths (vocabulary insert, terms of >= 16 bytes, bucket chains, documents
 *     starting inside a step) run behind wave-uniform branches.
 *
 * LDS: 28 KiB table + ~11 KiB walk/document state -> four workgroups (16 waves) per CU.
 * Requires a 16-byte aligned corpus base.
 */
#include "dev_common.h"
#include "dev_vocab.h"
#include "kernels.h"

namespace {

constexpr int NT = 256;                   /* threads per workgroup */
constexpr int WG_PER_CU = 4;              /* 16 waves per CU */
constexpr int NWAVE = NT / 64;
constexpr uint32_t WSTEP = 992;           /* bytes a wave step owns (lanes 1..62) */
constexpr int TB = 3072;                  /* LDS table entries (u32 key + u32 count): 12 per thread */
constexpr uint32_t DD = 2;                /* documents of a group with dense hot-term counters */
constexpr uint32_t HW = HOT_MAX / 2;      /* words per document: two u16 counters each */
constexpr int EPT = TB / NT;
constexpr uint32_t FILL_LIMIT = TB - NT * 2 - 64; /* claims after which overflow mode starts */
constexpr int GCAP = 128;                 /* documents per group at most */
constexpr uint32_t BQ = 128;              /* per-wave queue of keys for the bucket table */
constexpr int TLW = 192;                  /* token entries per wave and pass */
constexpr uint32_t LEN_LONG = 31u;        /* entry length field: term of >= 16 bytes / past the window */
constexpr uint32_t BW = 4;                /* LDS table bucket width */
constexpr uint32_t NB = TB / BW;
constexpr int32_t FAR = 0x3FFFFFFF;       /* "no document start" in group-relative offsets */

struct LShared {
    uint32_t TK[TB];                      /* key32 = 1 << 31 | doc-in-group << sb | slot (0: empty) */
    uint32_t TC[TB];                      /* its count */
    uint32_t dense[DD * HW];              /* hot terms of the group's first DD documents: u16 counts */
    uint32_t bq[NWAVE][BQ];               /* keys waiting for a full round of the bucket table */
    uint64_t gdoc[GCAP + 1];              /* doc_off of the group's documents */
    uint32_t dsz[GCAP];                   /* docSize accumulators */
    union {
        struct {                          /* walk */
            uint4 stage[NWAVE][64];       /* the step's 64 groups: [sb - 16, sb + 1008) */
            uint32_t tl[NWAVE][TLW];
        } w;
        struct {                          /* flush */
            uint32_t dcnt[GCAP];
            uint32_t doff[GCAP];
            uint32_t drun[GCAP];
            uint8_t dstate[GCAP];
        } f;
    };
    uint4 sel[16];                        /* v_perm selectors of a term of length n */
    uint64_t fbase[8];
    uint8_t dpart[GCAP];                  /* document has overflow records */
    uint32_t fill;
    uint32_t hot_closed;                  /* this workgroup saw the hot ids run out */
    uint32_t cur_chunk, nxt_chunk;
    uint32_t wsum[NWAVE];
    unsigned long long rec_base, part_base;
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));   /* unaligned LDS read */

__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
    const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(r.x, r.y, r.z, r.w);
}

/* bits of bytes [gp, gp + 16) outside [rlo, rhi) (group-relative) */
__device__ __forceinline__ uint32_t bounds_ws32(int32_t gp, int32_t rlo, int32_t rhi) {
    const int32_t a = min(max(rlo - gp, 0), 16);
    const int32_t b = min(max(rhi - gp, 0), 16);
    const uint32_t in = b > a ? (((1u << b) - 1u) & ~((1u << a) - 1u)) : 0u;
    return ~in & 0xFFFFu;
}

__device__ __forceinline__ uint32_t zero_bits(uint32_t x) { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u; }
__device__ __forceinline__ uint32_t compress4(uint32_t m) {   /* bits 7, 15, 23, 31 -> bits 0-3 */
    m >>= 7;
    m |= m >> 7;
    m |= m >> 14;
    return m & 0xFu;
}

__device__ __forceinline__ uint32_t runi(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)runi((uint32_t)(x >> 32)) << 32) | runi((uint32_t)x);
}
/* group-relative offset of an absolute position, clamped to [-32, FAR] */
__device__ __forceinline__ int32_t relpos(uint64_t x, uint64_t base) {
    if (x < base) return (base - x) >= 32 ? -32 : -(int32_t)(base - x);
    return (x - base) >= (uint64_t)FAR ? FAR : (int32_t)(x - base);
}

/* ---- the bucketed LDS count table (as tokcount_st.hip) ---- */
/* bucket of an LDS key (rel << sb | slot, bit 31 set): the slot bits are already a hash;
 * the document bits are folded into the low 16, which a 24-bit multiply (full rate, unlike
 * v_mul_lo_u32 / v_mul_hi_u32) scales to [0, NB) */
__device__ __forceinline__ uint32_t bkt_hash(uint32_t key) {
    return (uint32_t)__umul24((key ^ (key >> 15)) & 0xFFFFu, NB) >> 16;   /* [0, NB) */
}
__device__ __forceinline__ uint32_t bkt_next(uint32_t b) { return b + 1 == NB ? 0u : b + 1; }
__device__ __forceinline__ uint4 bkt_read(LShared& S, uint32_t b) { return reinterpret_cast<const uint4*>(S.TK)[b]; }
__device__ __forceinline__ uint32_t bkt_match(const uint4& kk, uint32_t key) {
    return kk.x == key ? 0u : kk.y == key ? 1u : kk.z == key ? 2u : kk.w == key ? 3u : 4u;
}
/* the first empty slot of bucket kk, scanning from slot key % 4, 4 if full */
__device__ __forceinline__ uint32_t bkt_empty(const uint4& kk, uint32_t key) {
    const uint32_t em = (kk.x == 0u ? 1u : 0u) | (kk.y == 0u ? 2u : 0u) | (kk.z == 0u ? 4u : 0u) | (kk.w == 0u ? 8u : 0u);
    if (!em) return BW;
    const uint32_t r0 = key & (BW - 1u);
    const uint32_t rot = ((em | (em << BW)) >> r0) & ((1u << BW) - 1u);
    return ((uint32_t)__builtin_ctz(rot) + r0) & (BW - 1u);
}

/* The next chunk for a workgroup whose current counter shard is `sh` (see tokcount_st.hip:
 * one device-scope counter saturates at ~88 claims/us, so the chunks are cut into 8
 * contiguous shards with a counter each).  Returns n when nothing is left. */
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

/* term slot of a token whose term is >= 16 bytes (or runs past the 32-byte window): the
 * token is re-read from HBM (rare for text) */
__device__ __forceinline__ uint32_t lean_slow_slot_in(const LeanParams* P, uint64_t p0, uint64_t dend,
                                                     uint32_t* hot_closed, uint32_t* hid) {
    const uint8_t* __restrict__ bytes = P->c.bytes;
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
        return vocab_insert_hot(P->v.keys, P->v.rep, P->v.mask, klo, khi, 0, P->o.status, P->o.hot_slot, P->o.hot_ctr,
                                hot_closed, hid);
    }
    make_long_key(bytes + p0, n, &klo, &khi);
    /* rep = (length << 40) | offset holds 24 length bits (TFIDF_E_CAPACITY beyond) */
    if (n >= 0xFFFFFFull) atomicOr(P->o.status, ST_TERM_LONG);
    const uint64_t rep = ((n < 0xFFFFFFull ? n : 0xFFFFFFull) << 40) | p0;
    return vocab_insert_hot(P->v.keys, P->v.rep, P->v.mask, klo, khi, rep, P->o.status, P->o.hot_slot, P->o.hot_ctr,
                            hot_closed, hid);
}

__device__ __forceinline__ void overflow_record(const LeanParams* P, uint32_t doc, uint32_t slot) {
    /* one device atomic per wave and call */
    const uint64_t am = __ballot(1);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
    unsigned long long b = 0;
    if (rank == 0u) b = atomicAdd(P->o.part_alloc, (unsigned long long)__popcll(am));
    const unsigned long long q = uni64(b) + rank;
    if (q < P->o.part_cap) { P->o.part_doc[q] = doc; P->o.part_slot[q] = slot; P->o.part_cnt[q] = 1u; }
    else atomicOr(P->o.status, ST_PART_FULL);
}

/* The miss paths, out of line (their registers are not the rounds' problem); the hot id
 * comes back packed with the slot (slot | id << 32), not through memory: a pointer to a
 * round variable would put it in scratch, and every scratch access waits on vmcnt. */
__device__ __noinline__ uint64_t lean_slow_slot(const LeanParams* P, uint64_t p0, uint64_t dend, uint32_t* hot_closed) {
    uint32_t hid = HOT_NONE;
    const uint32_t sl = lean_slow_slot_in(P, p0, dend, hot_closed, &hid);
    return ((uint64_t)hid << 32) | sl;
}
__device__ __noinline__ uint64_t lean_insert(const LeanParams* P, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3,
                                             uint32_t* hot_closed) {
    uint32_t hid = HOT_NONE;
    const uint32_t sl = vocab_insert_hot(P->v.keys, P->v.rep, P->v.mask, ((uint64_t)k1 << 32) | k0,
                                         ((uint64_t)k3 << 32) | k2, 0, P->o.status, P->o.hot_slot, P->o.hot_ctr,
                                         hot_closed, &hid);
    return ((uint64_t)hid << 32) | sl;
}

/* Counts `key` the slow way, from bucket b on (home bucket full, a lost claim, or overflow
 * mode).  Returns 1 when this call claimed a slot.  A key not in the table in overflow
 * mode, or after PMAX buckets, becomes a partial record of count 1. */
constexpr int PMAX = 16;
__device__ __noinline__ uint32_t bkt_slow(LShared& S, const LeanParams* P, uint32_t key, uint32_t b, bool over, uint32_t gd0,
                             uint32_t sb) {
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

/* The hot-term counters a thread owns in the flush: words w = tid + NT * k (k < DPT) of
 * S.dense, i.e. document k / 2, term ids 2 (tid + NT (k & 1)) and that + 1. */
constexpr int DPT = (int)(DD * HW) / NT;
static_assert(HW == 2 * NT && (DD * HW) % NT == 0 && DD <= 4, "dense words per thread");
__device__ __forceinline__ uint32_t nz16(uint32_t w) { return ((w & 0xFFFFu) != 0u ? 1u : 0u) + ((w >> 16) != 0u ? 1u : 0u); }

/* Emits every table entry and every non-zero hot counter of the group as records and
 * clears both (any number of documents): per-document counts, a block scan, then every
 * entry straight to its slot.  A hot term's record carries slot cap + id (its rank comes
 * from rank_of_slot[cap + id], see launch_hot_ranks). */
__device__ __forceinline__ void lean_flush(LShared& S, const LeanParams* P, uint32_t gd0, uint32_t ng, uint64_t cs,
                                           uint64_t ce, uint32_t sb, uint32_t cap) {
    const int tid = threadIdx.x;
    if (tid < GCAP) { S.f.dcnt[tid] = 0; S.f.drun[tid] = 0; }
    lds_barrier();
    const uint32_t smask = (1u << sb) - 1u;
    /* two passes over the table in LDS (no per-thread copy of the entries: registers) */
    for (int j = 0; j < EPT; ++j) {
        const uint32_t k = S.TK[j * NT + tid];
        if (k) wave_agg_add(&S.f.dcnt[0], (k & 0x7FFFFFFFu) >> sb);
    }
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const uint32_t n = nz16(S.dense[tid + NT * k]);
        if (n) atomicAdd(&S.f.dcnt[k >> 1], n);
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
    auto emit = [&](uint32_t rel, uint32_t k, uint32_t slot, uint32_t c) {
        const uint32_t dof = S.f.doff[rel];
        if (S.f.dstate[rel] == 2) {
            const uint64_t q = rb + (dof & 0xFFFFu) + k;
            if (rec_ok) { rec_slot[q] = slot; rec_cnt[q] = c; }
        } else {
            const uint64_t q = pb + (dof >> 16) + k;
            if (part_ok) { P->o.part_doc[q] = gd0 + rel; P->o.part_slot[q] = slot; P->o.part_cnt[q] = c; }
        }
    };
    for (int j = 0; j < EPT; ++j) {
        const uint32_t key = S.TK[j * NT + tid];
        if (key) {
            const uint32_t c = S.TC[j * NT + tid];
            const uint32_t rel = (key & 0x7FFFFFFFu) >> sb;
            emit(rel, wave_agg_add_rtn(&S.f.drun[0], rel), key & smask, c);
            S.TK[j * NT + tid] = 0u;
            S.TC[j * NT + tid] = 0u;
        }
    }
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const uint32_t w = S.dense[tid + NT * k];
        if (w) {
            const uint32_t rel = (uint32_t)k >> 1, id = 2u * ((uint32_t)tid + NT * ((uint32_t)k & 1u));
            uint32_t r = atomicAdd(&S.f.drun[rel], nz16(w));
            if (w & 0xFFFFu) emit(rel, r++, cap + id, w & 0xFFFFu);
            if (w >> 16) emit(rel, r, cap + id + 1u, w >> 16);
            S.dense[tid + NT * k] = 0u;
        }
    }
}

/* The flush of a group of at most FEW documents (most c2 chunks hold one or two): 16-bit
 * per-document counters per thread, one block scan, no LDS atomics.  Same output. */
constexpr uint32_t FEW = 8;
__device__ __forceinline__ void lean_flush_few(LShared& S, const LeanParams* P, uint32_t gd0, uint32_t ng, uint64_t cs,
                                               uint64_t ce, uint32_t sb, uint32_t cap) {
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
    /* dense words: document k / 2 of each pair k -> field (k / 2) & 1 of pk[k / 4] */
#pragma unroll
    for (int k = 0; k < DPT; ++k) pk[k >> 2] += nz16(S.dense[tid + NT * k]) << (16 * ((k >> 1) & 1));
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
    auto emit = [&](uint32_t rel, uint32_t slot, uint32_t c) {
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
            if (S.f.dstate[rel] == 2) { rec_slot[qq] = slot; rec_cnt[qq] = c; }
            else { P->o.part_doc[qq] = gd0 + rel; P->o.part_slot[qq] = slot; P->o.part_cnt[qq] = c; }
        }
    };
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const uint32_t key = S.TK[j * NT + tid];
        if (key) {
            emit((key & 0x7FFFFFFFu) >> sb, key & smask, S.TC[j * NT + tid]);
            S.TK[j * NT + tid] = 0u;
            S.TC[j * NT + tid] = 0u;
        }
    }
    /* dense words after the table entries: the ranks per document continue (the scan
     * counted them in the same order) */
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const uint32_t wd = S.dense[tid + NT * k];
        if (wd) {
            const uint32_t rel = (uint32_t)k >> 1, id = 2u * ((uint32_t)tid + NT * ((uint32_t)k & 1u));
            if (wd & 0xFFFFu) emit(rel, cap + id, wd & 0xFFFFu);
            if (wd >> 16) emit(rel, cap + id + 1u, wd >> 16);
            S.dense[tid + NT * k] = 0u;
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

/* the document-start masks of a step whose window [sbo - 16, sbo + 1008) holds a document
 * start (wave-uniform loop over the group's documents from wr on) */
__device__ __noinline__ uint4 doc_starts(LShared& S, uint32_t wr, uint32_t ng, uint64_t b0, int32_t sbo, int32_t gp) {
    uint32_t ds = 0, dsn = 0, base = wr, wemp = 0;
    int32_t sprev = -0x40000000;
    for (uint32_t k = wr; k <= ng; ++k) {
        const int32_t sk = relpos(uni64(S.gdoc[k]), b0);
        if (sk >= sbo + (int32_t)WSTEP + 16) break;
        wemp |= (k > wr && sk == sprev) ? 1u : 0u;
        sprev = sk;
        base += (k > wr && sk < gp) ? 1u : 0u;
        if (sk >= gp && sk < gp + 16) {
            ds |= 1u << (uint32_t)(sk - gp);
            dsn |= k > wr ? 1u << (uint32_t)(sk - gp) : 0u;
        }
    }
    return make_uint4(ds, dsn, base, wemp);   /* by value: no scratch for out-parameters */
}

}  // namespace

__global__ __launch_bounds__(NT, WG_PER_CU) void k_tokcount_lean(const LeanParams* __restrict__ Pg,
                                                               const uint8_t* __restrict__ bytes,
                                                               const uint4* __restrict__ vkeys, uint32_t vmask,
                                                               uint32_t sb, uint32_t gcap, uint32_t nchunk,
                                                               uint64_t c_lo, uint64_t c_hi, uint64_t last_blk) {
    __shared__ __attribute__((aligned(16))) LShared S;
    /* Pg without __restrict__ from here on: its fields are read where used, never hoisted */
    const LeanParams* P = Pg;
    asm volatile("" : "+s"(P));
    const int tid = threadIdx.x, lane = tid & 63;
    /* the wave index as a scalar: the step loop, the document walk and every position
     * derived from them are then wave-uniform SGPR arithmetic and scalar branches, not
     * exec-masked VALU (threadIdx-derived values are divergent to the compiler) */
    const uint32_t wid = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);

    for (int j = 0; j < EPT; ++j) { S.TK[j * NT + tid] = 0u; S.TC[j * NT + tid] = 0u; }
    for (uint32_t j = (uint32_t)tid; j < DD * HW; j += NT) S.dense[j] = 0u;
    if (tid == 0) S.hot_closed = 0u;
    if (tid < 64) {
        const uint32_t n = (uint32_t)tid >> 2, k = (uint32_t)tid & 3u;
        (&S.sel[n].x)[k] = perm_sel(n, k);
    }
    uint32_t tokens_wg = 0;

    struct Round {
        uint32_t k0, k1, k2, k3;   /* identity key (short terms) */
        uint32_t hv, e;            /* home slot, token entry (0: no token) */
        uint4 s4, t4;              /* the two vocabulary slots loaded for it */
    };
    Round pend{};
    bool pending = false;
    /* the round being filled: lanes [0, carry) hold keys built from earlier steps of this
     * group, so every issued round is full (a step holds ~132 tokens: 64 + 64 + 4 would
     * leave one nearly empty round per step) */
    Round fillr{};
    uint32_t carry = 0;
    uint32_t gd0_cur = 0;
    uint64_t wbase_cur = 0;        /* absolute position of window byte 0 of step 0 of the group */

    /* vocabulary slot of a round (miss path: lock-free insert / long term) -> LDS key */
    /* vocabulary slot of a round (miss path: lock-free insert / long term); a hot term of
     * one of the group's first DD documents is counted right here in its dense counter (one
     * non-returning LDS add), everything else returns its LDS table key (0: nothing left) */
    auto resolve = [&](const Round& r) -> uint32_t {
        const uint32_t len = (r.e >> 10) & 31u;
        const uint32_t rel = (r.e >> 16) & 0xFFu;
        const bool valid = r.e != 0u;
        /* bitwise compares (xor / or3): no short-circuit branches on the exec mask; a slot's
         * hot mark (bytes 14-15) is not part of the term */
        const bool hit0 = ((r.s4.x ^ r.k0) | (r.s4.y ^ r.k1) | (r.s4.z ^ r.k2) | (unhot_w(r.s4.w) ^ r.k3)) == 0u;
        const bool hit1 = ((r.t4.x ^ r.k0) | (r.t4.y ^ r.k1) | (r.t4.z ^ r.k2) | (unhot_w(r.t4.w) ^ r.k3)) == 0u;
        uint32_t slot = hit0 ? r.hv : ((r.hv + 1) & vmask);
        uint32_t hid = hot_id_w(hit0 ? r.s4.w : r.t4.w);
        const bool rare = valid && (len == LEN_LONG || (!hit0 && !hit1));
        if (__ballot(rare) != 0ull) {
            if (rare) {
                const LeanParams* Q = P;
                asm volatile("" : "+s"(Q));
                const uint64_t sh = len == LEN_LONG
                    ? lean_slow_slot(Q, wbase_cur + (uint64_t)(r.e >> 24) * WSTEP + (r.e & 1023u), S.gdoc[rel + 1],
                                     &S.hot_closed)
                    : lean_insert(Q, r.k0, r.k1, r.k2, r.k3, &S.hot_closed);
                slot = (uint32_t)sh;
                hid = (uint32_t)(sh >> 32);
            }
        }
        const bool ok = valid && slot != INVALID_SLOT;
        const bool dense = ok && hid != HOT_NONE && rel < DD;
        if (dense) atomicAdd(&S.dense[rel * HW + (hid >> 1)], 1u << (16u * (hid & 1u)));
        return (ok && !dense) ? (0x80000000u | (rel << sb) | slot) : 0u;
    };
    /* the LDS count of a round: one ds_read_b128 of the home bucket; a match adds, a new key
     * claims a free slot with one CAS; the rest (full bucket, lost race, overflow) bkt_slow */
    auto count = [&](uint32_t key) {
        const bool over = S.fill >= FILL_LIMIT;
        const uint32_t b = bkt_hash(key);
        uint32_t claims = 0u;
        bool slow = false;
        if (key) {
            const uint4 kk = bkt_read(S, b);
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
            if (slow) {
                const LeanParams* Q = P;
                asm volatile("" : "+s"(Q));
                claims = bkt_slow(S, Q, key, b, over, gd0_cur, sb);
            }
        }
        const uint32_t wc = (uint32_t)__popcll(__ballot(claims != 0u));
        if (wc && lane == 0) (void)atomicAdd(&S.fill, wc);
    };
    /* Keys for the bucket table wait in the wave's queue until 64 of them make a full round:
     * the hot-term lanes of a round are done after one LDS add, and counting the rest in
     * rounds of whatever lanes remain would run the whole bucket path for a third of a wave. */
    uint32_t* const bq = S.bq[wid];
    uint32_t bq_n = 0;                    /* wave-uniform */
    auto enqueue = [&](uint32_t key) {
        const uint64_t m = __ballot(key != 0u);
        const uint32_t n = (uint32_t)__popcll(m);
        if (!n) return;
        const uint32_t pos = bq_n + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (key) bq[pos] = key;
        bq_n += n;
        if (bq_n >= 64u) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t k = bq[lane];
            const uint32_t rest = bq_n - 64u;
            const uint32_t kr = (uint32_t)lane < rest ? bq[64 + lane] : 0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if ((uint32_t)lane < rest) bq[lane] = kr;
            bq_n = rest;
            count(k);
        }
    };
    auto drain_queue = [&]() {
        if (bq_n) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            count((uint32_t)lane < bq_n ? bq[lane] : 0u);
            bq_n = 0;
        }
    };

    /* chunk schedule: thread 0 claims from 8 sharded counters, two chunks ahead */
    uint32_t shard = blockIdx.x & 7u;
    if (tid == 0) {
        unsigned long long* ctr = P->o.chunk_shard;
        S.cur_chunk = claim_chunk(ctr, shard, nchunk);
        S.nxt_chunk = claim_chunk(ctr, shard, nchunk);
    }
    lds_barrier();
    uint8_t* const stage = reinterpret_cast<uint8_t*>(&S.w.stage[wid][0]);
    uint32_t* const tl = S.w.tl[wid];
    const uint32_t lane16 = 16u * (uint32_t)lane;
    uint4 pf0 = make_uint4(0, 0, 0, 0);   /* the wave's next step of corpus bytes */
    uint64_t pfb = ~0ull;                 /* absolute base pf0 was loaded for (step `wid` of a group) */
    uint64_t dpre = 0;                    /* doc_off[dfirst + tid] of this chunk, fetched during the previous one */
    bool dpre_ok = false;
    unsigned long long pend_v = 0;
    uint32_t chunk = runi(S.cur_chunk), nxt = runi(S.nxt_chunk);
    uint64_t cs = 0, ce = 0;
    uint32_t dfirst = 0, dlast = 0;
    /* (loads through P are vector loads — the block is not provably read-only — so every
     * value read from it is made wave-uniform explicitly: scalar registers and branches) */
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
            gd0_cur = gd0;
            const uint32_t ng = (dlast + 1 - gd0) < gcap ? (dlast + 1 - gd0) : gcap;
            if (gd0 == dfirst && dpre_ok) {
                static_assert(GCAP < NT, "one thread per group document offset");
                if ((uint32_t)tid <= ng) S.gdoc[tid] = dpre;
            } else {
                const uint64_t* doff = P->c.doc_off;
                for (uint32_t k = tid; k <= ng; k += NT) S.gdoc[k] = doff[gd0 + k];
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
                const uint64_t b0 = gs & ~(uint64_t)15;          /* group base: step s owns [b0 + 992 s, +992) */
                const uint32_t nsteps = (uint32_t)((ge - b0 + WSTEP - 1) / WSTEP);
                const int32_t own_lo = (int32_t)(gs - b0), own_hi = (int32_t)(ge - b0);
                const int32_t rlo = relpos(c_lo, b0), rhi = relpos(c_hi, b0);
                const uint64_t wbase = b0 - 16;                  /* absolute position of window byte 0, step 0 */
                wbase_cur = wbase;
                /* the wave's first step: prefetched during the previous chunk when it aimed here */
                if (b0 != pfb) {
                    const uint64_t a = wbase + (uint64_t)wid * WSTEP + lane16;
                    pf0 = ld16(bytes + (a < last_blk ? a : last_blk));
                }
                pfb = ~0ull;
                uint32_t wr = 0;                                 /* document containing the step start */
                int32_t wcur = relpos(g0, b0);
                int32_t wnext = ng > 1 ? relpos(uni64(S.gdoc[1]), b0) : FAR;
                for (uint32_t s = wid; s < nsteps; s += NWAVE) {
                    const int32_t sbo = (int32_t)(s * WSTEP);    /* first owned byte, group-relative */
                    const int32_t gp = sbo - 16 + (int32_t)lane16; /* this lane's first byte */
                    const uint4 cur = pf0;
                    /* The wave's next step (or after its last one the next chunk's first) is
                     * loaded after this step's first round of vocabulary gathers, not now:
                     * vmcnt completes in issue order, so a corpus load issued here would hold up
                     * the wait for those gathers with the HBM latency.  Issued behind them it
                     * has a round's time before the next wait that covers it. */
                    uint64_t pfa;
                    {
                        const bool redirect = ahead && s + NWAVE >= nsteps;
                        if (redirect) {
                            const uint64_t nb0 = ncs & ~(uint64_t)15;
                            pfa = nb0 - 16 + (uint64_t)wid * WSTEP;
                            pfb = nb0;
                        } else {
                            pfa = wbase + (uint64_t)(s + NWAVE) * WSTEP;
                        }
                    }
                    bool pf_due = true;
                    auto prefetch = [&]() {
                        const uint64_t a = pfa + lane16;
                        pf0 = ld16(bytes + (a < last_blk ? a : last_blk));
                        pf_due = false;
                    };
                    reinterpret_cast<uint4*>(stage)[lane] = cur;
                    /* ---- classify (bytes outside the shard read as whitespace) ---- */
                    uint32_t ws = ws_mask16_swar(cur);
                    if (!(sbo - 16 >= rlo && sbo + (int32_t)WSTEP + 16 <= rhi)) ws |= bounds_ws32(gp, rlo, rhi);
                    while (wnext <= sbo) {   /* documents starting at or before the step start */
                        ++wr;
                        wcur = wnext;
                        wnext = wr + 1 < ng ? relpos(uni64(S.gdoc[wr + 1]), b0) : FAR;
                    }
                    uint32_t ds = 0, dsn = 0, base = wr, wemp = 0;
                    const bool hasdoc = wnext < sbo + (int32_t)WSTEP + 16 || wcur + 16 >= sbo;
                    if (hasdoc) {
                        const uint4 d4 = doc_starts(S, wr, ng, b0, sbo, gp);
                        ds = d4.x;
                        dsn = d4.y;
                        base = d4.z;
                        wemp = d4.w;
                    }
                    const uint32_t prev = (lane_prev(ws) >> 15) & 1u;
                    uint32_t own = (lane >= 1 && lane <= 62) ? 0xFFFFu : 0u;
                    if (!(sbo >= own_lo && sbo + (int32_t)WSTEP <= own_hi) && own) {
                        const int32_t a = min(max(own_lo - gp, 0), 16), b = min(max(own_hi - gp, 0), 16);
                        own = b > a ? (((1u << b) - 1u) & ~((1u << a) - 1u)) : 0u;
                    }
                    const uint32_t starts = ~ws & ((ws << 1) | prev | ds) & own & 0xFFFFu;
                    /* NUL bytes end a term (strcmp), not a token: exact masks only when the
                     * wave holds one */
                    uint32_t nul = 0;
                    if (__ballot((zero_bits(cur.x) | zero_bits(cur.y) | zero_bits(cur.z) | zero_bits(cur.w)) != 0u) != 0ull)
                        nul = compress4(zero_bits(cur.x)) | (compress4(zero_bits(cur.y)) << 4) |
                              (compress4(zero_bits(cur.z)) << 8) | (compress4(zero_bits(cur.w)) << 12);
                    const uint32_t stop = ws | ds;
                    const uint32_t stop32 = stop | (lane_next(stop) << 16), nul32 = nul | (lane_next(nul) << 16);
                    const uint32_t nmine = (uint32_t)__popc(starts);
                    const uint32_t incl = wave_incl_scan(nmine);
                    const uint32_t ntok = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                    if (ntok == 0) { prefetch(); continue; }
                    tokens_wg += ntok;
                    if (!hasdoc && lane == 0) atomicAdd(&S.dsz[wr], ntok);
                    for (uint32_t tb = 0; tb < ntok; tb += TLW) {
                        uint32_t sm = starts, idx = incl - nmine;
                        while (sm) {
                            const uint32_t i = __builtin_ctz(sm);
                            sm &= sm - 1;
                            if (idx - tb < (uint32_t)TLW) {
                                const uint32_t e = ((stop32 >> i) & ~1u) | (nul32 >> i);
                                const uint32_t len = e ? (uint32_t)__builtin_ctz(e) : LEN_LONG;
                                uint32_t rel = base;
                                if (hasdoc) {
                                    if (!wemp) {
                                        rel += (uint32_t)__popc(dsn & ((2u << i) - 1u));
                                    } else if (ds & ((2u << i) - 1u)) {   /* empty documents share a start */
                                        while (rel + 1 < ng && relpos(S.gdoc[rel + 1], b0) <= gp + (int32_t)i) ++rel;
                                    }
                                    atomicAdd(&S.dsz[rel], 1u);
                                }
                                tl[idx - tb] = ((uint32_t)lane << 4 | i) | ((len < 16u ? len : LEN_LONG) << 10) | (rel << 16);
                            }
                            ++idx;
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        const uint32_t cnt = (ntok - tb) < (uint32_t)TLW ? (ntok - tb) : (uint32_t)TLW;
                        /* ---- rounds of 64 tokens; round r+1's vocabulary loads are issued
                         * before round r is counted ---- */
                        for (uint32_t t0 = 0; t0 < cnt;) {
                            /* lanes [carry, carry + take) take entries t0.. of this step */
                            const uint32_t take = (64u - carry) < (cnt - t0) ? (64u - carry) : (cnt - t0);
                            if ((uint32_t)lane >= carry && (uint32_t)lane < carry + take) {
                                const uint32_t e = tl[t0 + (uint32_t)lane - carry];
                                const uint32_t pos = e & 1023u, len = (e >> 10) & 15u;
                                const u32x4u raw = *reinterpret_cast<const u32x4u*>(stage + pos);
                                const uint4 sl = S.sel[len];
                                fillr.e = e | (s << 24);
                                fillr.k0 = __builtin_amdgcn_perm(0x09090909u, raw.x, sl.x);
                                fillr.k1 = __builtin_amdgcn_perm(0x09090909u, raw.y, sl.y);
                                fillr.k2 = __builtin_amdgcn_perm(0x09090909u, raw.z, sl.z);
                                fillr.k3 = __builtin_amdgcn_perm(0x09090909u, raw.w, sl.w);
                            }
                            carry += take;
                            t0 += take;
                            if (carry == 64u) {
                                /* a full round.  Order matters: the pending round is resolved
                                 * first (its slots were loaded one round ago), then this round's
                                 * loads go straight into the pending round's registers, now dead,
                                 * and fly while the pending round is counted in LDS.  Issuing them
                                 * before the resolve would keep two sets of loaded registers live
                                 * and the copy between them waits for the loads (vmcnt). */
                                const uint32_t key = pending ? resolve(pend) : 0u;
                                pend = fillr;
                                pend.hv = (uint32_t)key_hash(((uint64_t)pend.k1 << 32) | pend.k0,
                                                             ((uint64_t)pend.k3 << 32) | pend.k2) & vmask;
                                pend.s4 = gload(vkeys + pend.hv);
                                pend.t4 = gload(vkeys + ((pend.hv + 1) & vmask));
                                if (pf_due) prefetch();
                                if (pending) enqueue(key);
                                pending = true;
                                carry = 0;
                            }
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
                    if (pf_due) prefetch();   /* no full round in this step */
                }
            }
            if (carry) {   /* the group's last, partial round (lanes >= carry hold no token) */
                const uint32_t key = pending ? resolve(pend) : 0u;
                pend = fillr;
                if ((uint32_t)lane >= carry) pend.e = 0u;
                pend.hv = (uint32_t)key_hash(((uint64_t)pend.k1 << 32) | pend.k0, ((uint64_t)pend.k3 << 32) | pend.k2) & vmask;
                pend.s4 = gload(vkeys + pend.hv);
                pend.t4 = gload(vkeys + ((pend.hv + 1) & vmask));
                if (pending) enqueue(key);
                pending = true;
                carry = 0;
            }
            if (pending) { enqueue(resolve(pend)); pending = false; }
            drain_queue();
            if (ahead) {   /* the next chunk's document offsets, in flight during this flush */
                const uint32_t nng = (ndl + 1 - ndf) < gcap ? (ndl + 1 - ndf) : gcap;
                dpre = (uint32_t)tid <= nng ? P->c.doc_off[ndf + tid] : 0ull;
                dpre_ok = true;
            }
            lds_barrier();   /* every wave's walk is done (the walk state aliases the flush's) */
            if (ng <= FEW) lean_flush_few(S, P, gd0, ng, cs, ce, sb, vmask + 1u);
            else lean_flush(S, P, gd0, ng, cs, ce, sb, vmask + 1u);
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
    if (lane == 0 && tokens_wg) atomicAdd(P->o.ntokens, (unsigned long long)tokens_wg);
}

int launch_tokcount_lean(const LeanParams* dparams, const LeanParams& h, hipStream_t s) {
    if (h.c1 <= h.c0) return 0;
    if (h.c0 != 0 || h.c1 > 0xFFFFFFFFull) return -3;   /* chunk indices are 32-bit here */
    if (h.v.mask >= (1ull << 28)) return -3;             /* slot must fit the LDS entry */
    static_assert(sizeof(LShared) * WG_PER_CU <= 163840, "LDS of WG_PER_CU workgroups per CU");
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
    k_tokcount_lean<<<(unsigned)grid, NT, 0, s>>>(dparams, h.c.bytes, h.v.keys, (uint32_t)h.v.mask, sb, gcap,
                                                  (uint32_t)n, h.c.lo, h.c.hi, last_blk);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* ---- hot terms after K1 (dev_vocab.h) ---- */
__global__ void k_hot_unmark(uint4* __restrict__ keys, const uint32_t* __restrict__ hot_slot,
                             const uint32_t* __restrict__ hot_ctr) {
    const uint32_t n = min(*hot_ctr, HOT_MAX);
    for (uint32_t id = threadIdx.x; id < n; id += blockDim.x) {
        const uint32_t sl = hot_slot[id];
        keys[sl].w = unhot_w(keys[sl].w);
    }
}
int launch_hot_unmark(uint4* keys, const uint32_t* hot_slot, const uint32_t* hot_ctr, hipStream_t s) {
    k_hot_unmark<<<1, 1024, 0, s>>>(keys, hot_slot, hot_ctr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ void k_hot_ranks(uint32_t* __restrict__ rank_of_slot, uint16_t* __restrict__ rank16, uint64_t cap,
                            const uint32_t* __restrict__ hot_slot, const uint32_t* __restrict__ hot_ctr) {
    const uint32_t n = min(*hot_ctr, HOT_MAX);
    for (uint32_t id = threadIdx.x; id < HOT_MAX; id += blockDim.x) {
        const uint32_t r = id < n ? rank_of_slot[hot_slot[id]] : 0u;
        rank_of_slot[cap + id] = r;
        if (rank16) rank16[cap + id] = (uint16_t)(id < n ? rank16[hot_slot[id]] : 0u);
    }
}
int launch_hot_ranks(uint32_t* rank_of_slot, uint16_t* rank16, uint64_t cap, const uint32_t* hot_slot,
                     const uint32_t* hot_ctr, hipStream_t s) {
    static_assert(HOT_SLOTS == HOT_MAX, "rank maps sized for every hot id");
    k_hot_ranks<<<1, 1024, 0, s>>>(rank_of_slot, rank16, cap, hot_slot, hot_ctr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
