/*
 * tokcount_vs.hip — K1: fused tokenize + per-document term counting, keyed by
 * vocabulary slot.  Replaces the reference's per-rank hot loop TFIDF.c:130-196:
 * fscanf("%s") tokenising (:141-147), the O(P) strcmp search/append of (word, doc)
 * records (:151-167) and the per-rank word table (:169-188).
 *
 * One 256-thread workgroup owns one chunk (K0, ~16 KiB of whole documents, or a
 * 16 KiB piece of a document longer than BIG_DOC) and walks it in 4 KiB steps:
 *
 *   classify  each lane holds one 16-byte group in registers (global_load_dwordx4,
 *             the next step prefetched) and forms 16-bit masks: whitespace (C-locale
 *             isspace, TFIDF.c:142,147), document starts (a document start always
 *             starts a token and ends the previous one) and owned bytes;
 *   count     token starts per step are block-reduced so that the flush decision is
 *             made once per step, identically in every thread, before any insert;
 *   resolve   each lane walks its own token starts: the 128-bit term key (dev_common.h;
 *             strcmp/NUL semantics) is cut from its 16 bytes plus its neighbour's
 *             (DPP lane shift), hashed, and looked up in the HBM vocabulary (one 16-byte
 *             load, L2-resident for Zipfian text; lock-free insert on a miss);
 *   insert    (document, slot) is counted in an LDS open-addressing table of u64
 *             entries  key(36 bits: doc-in-group 8 | slot 28) << 24 | count(24),
 *             claimed by one 64-bit LDS CAS, hit by one 64-bit LDS add;
 *   flush     when the next step could push the table over SOFT entries, and at the
 *             end of each document group: entries of documents that have ended are
 *             written as (slot, count) records grouped by document; the document still
 *             open is re-inserted (or, if it alone is too large, flushed to the
 *             partial stream); documents crossing a chunk edge always go to the
 *             partial stream (merged by finalize.hip's radix sort + reduce-by-key).
 *
 * LDS: 32 KiB table + ~6 KiB document state -> four workgroups (16 waves) per CU.
 * Requires a 16-byte aligned corpus base (clamped 16-byte group loads); engine.cpp
 * falls back to tokcount.hip's general kernel otherwise.
 */
#include "dev_common.h"
#include "dev_vocab.h"
#include "kernels.h"

namespace {

constexpr int NT = 256;
constexpr int STEP = NT * 16;             /* bytes per step: one 16-byte group per lane */
constexpr int TB = 4096;                  /* LDS table entries (u64) */
constexpr int EPT = TB / NT;              /* table entries scanned per thread in a flush */
constexpr uint32_t SOFT = 3072;           /* table entries after a step never exceed this */
constexpr int GCAP = 256;                 /* documents per group (doc-in-group: 8 bits) */
constexpr uint32_t SLOT_BITS = 28;
constexpr uint32_t CNT_BITS = 24;
constexpr uint64_t CNT_MASK = (1ull << CNT_BITS) - 1ull;
constexpr int KB = 2;                     /* tokens per lane whose vocabulary loads fly together */

/* Diagnostic build only (-DK1_STAMPS, lib/libtfidf_hip_stamps.so): thread 0 sums
 * s_memtime cycles per phase and lane-level event counters; never in the measured
 * library.  Phases: 0 group setup, 1 classify, 2 count+decide, 3 mid flush, 4 resolve+
 * insert, 5 group flush, 6 docSize write.  Counters: tokens, first-probe misses,
 * LDS probe iterations, wave token-loop iterations x 64. */
#ifdef K1_STAMPS
struct Stamps {
    uint64_t prev;
    uint64_t acc[K1_NSTAMP];
};
#define STAMP(st, k)                                                          \
    do {                                                                      \
        if (threadIdx.x == 0) {                                               \
            __builtin_amdgcn_sched_barrier(0);                                \
            uint64_t t_ = __builtin_amdgcn_s_memtime();                       \
            __builtin_amdgcn_s_waitcnt(0xC07F);                               \
            if ((st).prev) (st).acc[k] += t_ - (st).prev;                     \
            (st).prev = t_;                                                   \
            __builtin_amdgcn_sched_barrier(0);                                \
        }                                                                     \
    } while (0)
#define CNT(k, n) (cnt_[k] += (n))
#else
struct Stamps {};
#define STAMP(st, k) do { (void)(st); } while (0)
#define CNT(k, n) ((void)0)
#endif

struct VsShared {
    unsigned long long T[TB];             /* (doc, slot) -> count */
    uint64_t gdoc[GCAP + 1];              /* doc_off of the group's documents */
    uint32_t dsz[GCAP];                   /* docSize accumulators */
    uint32_t dcnt[GCAP];                  /* flush: entries per document */
    uint32_t doff[GCAP];                  /* flush: record offset (complete | partial << 16) */
    uint32_t drun[GCAP];                  /* flush: running record index per document */
    uint8_t dstate[GCAP];                 /* flush: 0 none, 1 partial, 2 complete, 3 keep */
    uint8_t dpart[GCAP];                  /* document already (or forced) in the partial stream */
    uint32_t wtok[2][NT / 64];            /* per-wave token counts of a step (double-buffered) */
    uint32_t wcl[2][NT / 64];             /* per-wave table claims of a step (double-buffered) */
    uint32_t wsum[NT / 64];
    uint32_t nkeep;
    unsigned long long rec_base, part_base;
};

/* Streaming corpus load: clamped to the last 16-byte block holding corpus bytes, and
 * non-temporal so the read-once corpus does not evict the vocabulary from L2. */
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16c(const uint8_t* __restrict__ bytes, uint64_t last_blk, uint64_t pos) {
    const uint64_t p = pos < last_blk ? pos : last_blk;
    const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(bytes + p));
    return make_uint4(r.x, r.y, r.z, r.w);
}

/* bytes of [pos, pos+16) outside the shard's [lo, hi) read as whitespace */
__device__ __forceinline__ uint32_t bounds_ws(uint64_t pos, uint64_t lo, uint64_t hi) {
    uint32_t m = 0;
    if (pos < lo || pos + 16 > hi) {
        const uint32_t a = pos < lo ? (uint32_t)min(lo - pos, (uint64_t)16) : 0u;
        const uint32_t b = hi > pos ? (uint32_t)min(hi - pos, (uint64_t)16) : 0u;
        const uint32_t in = b > a ? (((b >= 32u ? 0u : (1u << b)) - 1u) & ~((1u << a) - 1u)) : 0u;
        m = ~in & 0xFFFFu;
    }
    return m;
}

/* bit k set when a document of the group starts at gp + k (r: a document index whose
 * start is <= gp, or 0) */
__device__ __forceinline__ uint32_t doc_start_bits(const VsShared& S, uint32_t ng, uint32_t r, uint64_t gp) {
    uint32_t m = 0;
    for (uint32_t k = r; k <= ng; ++k) {
        const uint64_t s = S.gdoc[k];
        if (s >= gp + 16) break;
        if (s >= gp) m |= 1u << (uint32_t)(s - gp);
    }
    return m;
}

/* last document index r in [0, ng) with gdoc[r] <= x (0 if none) */
__device__ __forceinline__ uint32_t doc_of(const VsShared& S, uint32_t ng, uint64_t x) {
    uint32_t lo = 0, hi = ng;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (S.gdoc[mid] <= x) lo = mid; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint32_t tbl_hash(uint64_t key) {
    const uint32_t k = (uint32_t)key ^ (uint32_t)(key >> 28) * 0x9E3779B1u;
    return (k * 0x85EBCA6Bu) >> (32 - 12);
}

/* counts (key, +n) into the table probing from slot h (entry claimed with count n or
 * added to); returns true when it claimed a new entry */
__device__ __forceinline__ bool tbl_add_from(VsShared& S, uint64_t key, uint32_t h, uint32_t n, uint32_t* status) {
    const unsigned long long ent = (key << CNT_BITS) | n;
    for (int guard = 0; guard < TB; ++guard) {
        const unsigned long long old = atomicCAS(&S.T[h], 0ull, ent);
        if (old == 0ull) return true;
        if ((old >> CNT_BITS) == key) { atomicAdd(&S.T[h], (unsigned long long)n); return false; }
        h = (h + 1) & (TB - 1);
    }
    atomicOr(status, ST_BOUNDS);
    return false;
}
__device__ __forceinline__ bool tbl_add(VsShared& S, uint64_t key, uint32_t n, uint32_t* status) {
    return tbl_add_from(S, key, tbl_hash(key) & (TB - 1), n, status);
}

/* Term slot of a token whose term is >= 16 bytes or whose end lies past the 32 bytes a
 * lane holds: the token is re-read from HBM (rare for text). */
__device__ __forceinline__ uint32_t slow_slot(const uint8_t* __restrict__ bytes, uint4* keys, uint64_t* reps,
                                           uint64_t mask, uint64_t p0, uint64_t dend, uint32_t* status) {
    const VocabDev v{keys, reps, mask};
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
    const uint64_t rep = ((n < 0xFFFFFFull ? n : 0xFFFFFFull) << 40) | p0;
    return vocab_insert(v, klo, khi, rep, status);
}


/* Writes table entries as records and clears the table.  Documents that ended at or
 * before `pos` (all of them when `final`) are emitted; the document open at `pos` is
 * kept (re-inserted) unless its entries plus `ntok_next` would exceed SOFT, in which
 * case it is emitted to the partial stream.  Returns the entries kept. */
__device__ uint32_t vs_flush(VsShared& S, const K1Out& o, uint32_t gd0, uint32_t ng, uint64_t cs, uint64_t ce,
                             uint64_t pos, bool final, uint32_t ntok_next) {
    const int tid = threadIdx.x;
    if (tid < GCAP) { S.dcnt[tid] = 0; S.drun[tid] = 0; }
    if (tid == 0) S.nkeep = 0;
    __syncthreads();
    /* pass 1: entries into registers (lane-consecutive, conflict-free), per-document counts */
    unsigned long long e[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        e[j] = S.T[j * NT + tid];
        if (e[j]) atomicAdd(&S.dcnt[(uint32_t)(e[j] >> (CNT_BITS + SLOT_BITS))], 1u);
    }
    __syncthreads();
    /* per-document decision, one thread per document */
    uint32_t packed = 0;
    if (tid < GCAP) {
        uint8_t st = 0;
        const uint32_t cnt = (uint32_t)tid < ng ? S.dcnt[tid] : 0u;
        if (cnt) {
            bool closable = final || S.gdoc[tid + 1] <= pos;
            if (!closable && cnt + ntok_next > SOFT) { closable = true; S.dpart[tid] = 1; }
            if (closable) {
                const bool complete = !S.dpart[tid] && S.gdoc[tid] >= cs && S.gdoc[tid + 1] <= ce &&
                                      cnt <= (uint32_t)K5_MAX_PAIRS;
                if (!complete) S.dpart[tid] = 1;
                st = complete ? 2 : 1;
                packed = complete ? cnt : (cnt << 16);
            } else {
                st = 3;
                S.nkeep = cnt;
            }
        }
        S.dstate[tid] = st;
    }
    uint32_t tot;
    const uint32_t off = block_excl_scan<NT>(packed, S.wsum, &tot);
    if (tid < GCAP) S.doff[tid] = off;
    if (tid == 0) {
        const uint32_t nrec = tot & 0xFFFFu, npart = tot >> 16;
        unsigned long long rb = 0, pb = 0;
        if (o.ablate & 8u) { /* timing experiment: no allocation atomics */
            rb = ((unsigned long long)blockIdx.x * 4096ull) % (o.rec_cap > 8192 ? o.rec_cap - 8192 : 1);
            pb = ((unsigned long long)blockIdx.x * 4096ull) % (o.part_cap > 8192 ? o.part_cap - 8192 : 1);
        } else {
            rb = nrec ? atomicAdd(o.rec_alloc, (unsigned long long)nrec) : 0ull;
            pb = npart ? atomicAdd(o.part_alloc, (unsigned long long)npart) : 0ull;
        }
        if (rb + nrec > o.rec_cap) atomicOr(o.status, ST_REC_FULL);
        if (pb + npart > o.part_cap) atomicOr(o.status, ST_PART_FULL);
        S.rec_base = rb;
        S.part_base = pb;
    }
    __syncthreads();
    const unsigned long long rb = S.rec_base, pb = S.part_base;
    const bool rec_ok = rb + (tot & 0xFFFFu) <= o.rec_cap, part_ok = pb + (tot >> 16) <= o.part_cap;
    if (tid < GCAP && (uint32_t)tid < ng) {
        const uint8_t st = S.dstate[tid];
        if (st == 2) {
            o.doc_recoff[gd0 + tid] = rb + (off & 0xFFFFu);
            o.doc_npairs[gd0 + tid] = S.dcnt[tid];
        } else if (st == 1) {
            o.doc_flags[gd0 + tid] = DF_PARTIAL;
        }
    }
    /* pass 2: stage emitted entries in the (already read) table in output order —
     * complete records [0, nrec), partial records [nrec, nrec + npart) — so that the
     * HBM writes below are coalesced; remember kept ones */
    const uint32_t nrec = tot & 0xFFFFu, ntot = nrec + (tot >> 16);
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        if (!e[j]) continue;
        const uint32_t rel = (uint32_t)(e[j] >> (CNT_BITS + SLOT_BITS));
        const uint32_t slot = (uint32_t)(e[j] >> CNT_BITS) & ((1u << SLOT_BITS) - 1u);
        const uint64_t cnt = e[j] & CNT_MASK;
        const uint8_t st = S.dstate[rel];
        if (st == 3) { keep |= 1u << j; continue; }
        const uint32_t k = atomicAdd(&S.drun[rel], 1u);
        const uint32_t dof = S.doff[rel];
        if (st == 2) S.T[(dof & 0xFFFFu) + k] = slot | (cnt << 32);
        else S.T[nrec + (dof >> 16) + k] = slot | ((uint64_t)rel << SLOT_BITS) | (cnt << 36);
    }
    __syncthreads();
    /* coalesced write-out; each thread then clears exactly the entries it read */
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const uint32_t i = j * NT + tid;
        if (i < nrec) {
            const unsigned long long w = S.T[i];
            if (rec_ok) { o.rec_slot[rb + i] = (uint32_t)w; o.rec_cnt[rb + i] = (uint32_t)(w >> 32); }
        } else if (i < ntot) {
            const unsigned long long w = S.T[i];
            const uint64_t q = pb + (i - nrec);
            if (part_ok) {
                o.part_doc[q] = gd0 + ((uint32_t)(w >> SLOT_BITS) & 0xFFu);
                o.part_slot[q] = (uint32_t)w & ((1u << SLOT_BITS) - 1u);
                o.part_cnt[q] = (uint32_t)(w >> 36);
            }
        }
        S.T[i] = 0ull;
    }
    __syncthreads();
    if (keep) {
#pragma unroll
        for (int j = 0; j < EPT; ++j)
            if (keep & (1u << j)) tbl_add(S, e[j] >> CNT_BITS, (uint32_t)(e[j] & CNT_MASK), o.status);
    }
    const uint32_t nk = S.nkeep;
    __syncthreads();
    return nk;
}

}  // namespace

/* wave-uniform copy of a value the compiler keeps in VGPRs (LDS-loaded) */
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}
__device__ __forceinline__ uint32_t uni32(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

/* Persistent: a grid of (CUs x 4) workgroups walks the chunks [c0, c1) round-robin, so
 * the per-workgroup setup (LDS table clear, kernel-argument state) is paid once. */
__global__ __launch_bounds__(NT, 4) void k_tokcount_vs(CorpusDev c, const uint64_t* __restrict__ chunk_start,
                                                       const uint32_t* __restrict__ chunk_doc, uint64_t c0,
                                                       uint64_t c1, VocabDev v, K1Out o) {
    __shared__ __attribute__((aligned(16))) VsShared S;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t last_blk = c.nbytes ? ((c.nbytes - 1) & ~(uint64_t)15) : 0;

#pragma unroll
    for (int j = 0; j < EPT; ++j) S.T[j * NT + tid] = 0ull;
    unsigned long long tokens_chunk = 0;
    uint32_t step = 0;  /* global step counter: buffer parity */
    Stamps st;
#ifdef K1_STAMPS
    st.prev = 0;
    for (int k = 0; k < K1_NSTAMP; ++k) st.acc[k] = 0;
    uint32_t cnt_[K1_NCOUNT] = {0, 0, 0, 0};
#endif
    STAMP(st, 0);
    if (tid < NT / 64) { S.wcl[0][tid] = 0; S.wcl[1][tid] = 0; }

    for (uint64_t chunk = c0 + blockIdx.x; chunk < c1; chunk += gridDim.x) {
    const uint64_t cs = chunk_start[chunk], ce = chunk_start[chunk + 1];
    if (cs >= ce) continue;
    const uint32_t dfirst = chunk_doc[chunk], dlast = chunk_doc[chunk + 1];
    for (uint32_t gd0 = dfirst; gd0 <= dlast; gd0 += GCAP) {
        const uint32_t ng = (dlast + 1 - gd0) < (uint32_t)GCAP ? (dlast + 1 - gd0) : (uint32_t)GCAP;
        for (uint32_t k = tid; k <= ng; k += NT) S.gdoc[k] = c.doc_off[gd0 + k];
        if (tid < GCAP) { S.dsz[tid] = 0; S.dpart[tid] = 0; }
        __syncthreads();
        const uint64_t g0 = uni64(S.gdoc[0]), gn = uni64(S.gdoc[ng]);
        const uint64_t gs = g0 > cs ? g0 : cs;
        const uint64_t ge = gn < ce ? gn : ce;
        STAMP(st, 0);
        uint32_t fill = 0; /* table entries, identical in every thread */
        if (gs < ge) {
            const uint64_t wbase0 = gs & ~(uint64_t)15;
            /* lanes 0 and 63 also prefetch the group before / after their own (the byte
             * before a wave's first group; the bytes a token runs into past its last) */
            const bool edge_lane = lane == 0 || lane == 63;
            const uint64_t eoff = lane == 0 ? (uint64_t)0 - 16ull : 16ull;
            uint4 pf = ld16c(c.bytes, last_blk, wbase0 + 16ull * tid);
            uint4 pe = make_uint4(0, 0, 0, 0);
            if (edge_lane) pe = ld16c(c.bytes, last_blk, wbase0 + 16ull * tid + eoff);
            for (uint64_t sbase = wbase0; sbase < ge; sbase += STEP, ++step) {
                const uint32_t par = step & 1u;
                const uint64_t gpos = sbase + 16ull * tid;
                const uint4 cur = pf, edge = pe;
                if (o.ablate & 16u) pf = make_uint4(0x20616161u ^ (uint32_t)gpos, 0x61612061u, 0x61206161u, 0x20616161u);
                else pf = ld16c(c.bytes, last_blk, gpos + STEP); /* next step, harmless past ge */
                if (edge_lane) pe = ld16c(c.bytes, last_blk, gpos + STEP + eoff);
                /* ---- classify ---- */
                const uint32_t ws = ws_mask16(cur) | bounds_ws(gpos, c.lo, c.hi);
                const uint32_t r0 = doc_of(S, ng, gpos);
                const uint32_t ds = doc_start_bits(S, ng, r0, gpos);
                const uint32_t stop = ws | ds;
                uint32_t own = 0;
                if (gpos + 16 > gs && gpos < ge) {
                    const uint32_t a = gpos < gs ? (uint32_t)(gs - gpos) : 0u;
                    const uint32_t b = gpos + 16 > ge ? (uint32_t)(ge - gpos) : 16u;
                    own = ((1u << b) - 1u) & ~((1u << a) - 1u);
                }
                uint32_t prev = (lane_prev(ws) >> 15) & 1u;
                if (lane == 0) prev = (gpos > c.lo && gpos - 1 < c.hi) ? (is_ws(edge.w >> 24) ? 1u : 0u) : 1u;
                const uint32_t starts = ~ws & (((ws << 1) | prev) | ds) & own & 0xFFFFu;
                /* the neighbour's 16 bytes and stop mask (tokens running into it) */
                uint4 nxt;
                nxt.x = lane_next(cur.x);
                nxt.y = lane_next(cur.y);
                nxt.z = lane_next(cur.z);
                nxt.w = lane_next(cur.w);
                uint32_t nstop = lane_next(stop);
                if (lane == 63 && starts) {
                    nxt = edge;
                    nstop = ws_mask16(nxt) | bounds_ws(gpos + 16, c.lo, c.hi) | doc_start_bits(S, ng, r0, gpos + 16);
                }
                STAMP(st, 1);
                /* ---- step token count -> flush decision (identical in every thread) ---- */
                const uint32_t wt = wave_sum((uint32_t)__popc(starts));
                if (lane == 0) S.wtok[par][wid] = wt;
                __syncthreads();
                uint32_t ntok = 0, ncl = 0;
#pragma unroll
                for (int q = 0; q < NT / 64; ++q) { ntok += S.wtok[par][q]; ncl += S.wcl[par ^ 1u][q]; }
                fill += ncl;
                tokens_chunk += ntok;
                STAMP(st, 2);
                if (fill + ntok > SOFT) fill = vs_flush(S, o, gd0, ng, cs, ce, sbase, false, ntok);
                STAMP(st, 3);
                /* ---- resolve + insert this lane's tokens ---- */
                uint32_t claims = 0;
                if (starts && !(o.ablate & 4u)) {
                    const uint64_t q0 = ((uint64_t)cur.y << 32) | cur.x, q1 = ((uint64_t)cur.w << 32) | cur.z;
                    const uint64_t q2 = ((uint64_t)nxt.y << 32) | nxt.x, q3 = ((uint64_t)nxt.w << 32) | nxt.z;
                    const uint32_t s32 = stop | (nstop << 16);
                    uint32_t rel = r0;
                    uint64_t nstart = S.gdoc[rel + 1];
                    uint32_t run_rel = rel, run_n = 0;
                    uint32_t sm = starts;
                    CNT(0, __popc(starts));
                    while (sm) {
                        CNT(3, 1);
                        /* batch of KB tokens: keys, then every first vocabulary probe in
                         * flight together, then the LDS counting */
                        uint64_t klo[KB], khi[KB];
                        uint32_t hv[KB], relk[KB], ipos[KB], kind[KB];
                        uint4 s4[KB];
#pragma unroll
                        for (int k = 0; k < KB; ++k) {
                            kind[k] = 0;
                            ipos[k] = 0;
                            klo[k] = khi[k] = 0;
                            if (sm) {
                                const uint32_t i = __builtin_ctz(sm);
                                sm &= sm - 1;
                                const uint64_t ap = gpos + i;
                                while (nstart <= ap) { ++rel; nstart = S.gdoc[rel + 1]; }
                                const uint32_t m = s32 >> (i + 1);
                                const uint32_t len = m ? (uint32_t)__builtin_ctz(m) + 1u : 32u;
                                const uint32_t sh = (i & 7u) * 8u;
                                const uint64_t a = i < 8 ? q0 : q1, b = i < 8 ? q1 : q2, cc = i < 8 ? q2 : q3;
                                const uint64_t lo = sh ? (a >> sh) | (b << (64 - sh)) : a;
                                const uint64_t hi = sh ? (b >> sh) | (cc << (64 - sh)) : b;
                                kind[k] = make_short_key(lo, hi, len, &klo[k], &khi[k]) < 16u ? 1u : 2u;
                                ipos[k] = i;
                            }
                            relk[k] = rel;
                            hv[k] = kind[k] == 1u ? (uint32_t)(key_hash(klo[k], khi[k]) & v.mask) : 0u;
                            if (o.ablate & 1u) { s4[k] = make_uint4((uint32_t)klo[k], (uint32_t)(klo[k] >> 32), (uint32_t)khi[k], (uint32_t)(khi[k] >> 32)); if (kind[k] == 2u) kind[k] = 1u; }
                            else s4[k] = v.keys[hv[k]];
                        }
                        uint64_t key[KB];
                        uint32_t hl[KB];
#pragma unroll
                        for (int k = 0; k < KB; ++k) {
                            uint32_t slot = INVALID_SLOT;
                            if (kind[k] == 1u) {
                                const bool hit = s4[k].x == (uint32_t)klo[k] && s4[k].y == (uint32_t)(klo[k] >> 32) &&
                                                 s4[k].z == (uint32_t)khi[k] && s4[k].w == (uint32_t)(khi[k] >> 32);
                                CNT(1, hit ? 0 : 1);
                                slot = hit ? hv[k] : vocab_insert(v, klo[k], khi[k], 0, o.status);
                            } else if (kind[k] == 2u) {
                                slot = slow_slot(c.bytes, v.keys, v.rep, v.mask, gpos + ipos[k], S.gdoc[relk[k] + 1], o.status);
                            }
                            if (kind[k]) {
                                if (relk[k] != run_rel) {
                                    if (run_n) atomicAdd(&S.dsz[run_rel], run_n);
                                    run_rel = relk[k];
                                    run_n = 0;
                                }
                                ++run_n;
                            }
                            /* invalid slot: status flagged, the run is retried */
                            key[k] = slot == INVALID_SLOT ? ~0ull : (((uint64_t)relk[k] << SLOT_BITS) | slot);
                            hl[k] = tbl_hash(key[k]) & (TB - 1);
                        }
                        /* first LDS probes of the batch issued together (one lane's LDS
                         * operations execute in order, so a repeated key sees its claim) */
                        unsigned long long old[KB];
                        if (o.ablate & 2u) continue;
#pragma unroll
                        for (int k = 0; k < KB; ++k)
                            old[k] = key[k] != ~0ull ? atomicCAS(&S.T[hl[k]], 0ull, (key[k] << CNT_BITS) | 1ull) : 1ull;
#pragma unroll
                        for (int k = 0; k < KB; ++k) {
                            if (key[k] == ~0ull) continue;
                            if (old[k] == 0ull) { ++claims; continue; }
                            if ((old[k] >> CNT_BITS) == key[k]) { atomicAdd(&S.T[hl[k]], 1ull); continue; }
                            if (tbl_add_from(S, key[k], (hl[k] + 1) & (TB - 1), 1u, o.status)) ++claims;
                        }
                    }
                    if (run_n) atomicAdd(&S.dsz[run_rel], run_n);
                }
                const uint32_t wc = wave_sum(claims);
                if (lane == 0) S.wcl[par][wid] = wc;
                STAMP(st, 4);
            }
        }
        /* group end is a document boundary (or the chunk end): emit everything */
        if (!(o.ablate & 32u)) vs_flush(S, o, gd0, ng, cs, ce, ge, true, 0);
        STAMP(st, 5);
        if ((uint32_t)tid < ng) {
            const uint32_t n = S.dsz[tid];
            if (n) {
                const uint32_t d = gd0 + tid;
                if (S.gdoc[tid] >= cs && S.gdoc[tid + 1] <= ce) o.doc_size[d] = n;
                else atomicAdd(&o.doc_size[d], n);
            }
        }
        if (tid < NT / 64) { S.wcl[0][tid] = 0; S.wcl[1][tid] = 0; }
        __syncthreads();
        STAMP(st, 6);
        if (gd0 + GCAP < gd0) break; /* overflow guard */
    }
    }  /* chunk loop */
    if (tid == 0 && !(o.ablate & 8u)) atomicAdd(o.ntokens, tokens_chunk);
#ifdef K1_STAMPS
    if (tid == 0 && o.stamps) {
        for (int k = 0; k < K1_NSTAMP; ++k) atomicAdd(&o.stamps[k], (unsigned long long)st.acc[k]);
        atomicAdd(&o.stamps[K1_NSTAMP], 1ull);
    }
    if (o.stamps)
        for (int k = 0; k < K1_NCOUNT; ++k)
            if (cnt_[k]) atomicAdd(&o.stamps[K1_NSTAMP + 1 + k], (unsigned long long)cnt_[k]);
#endif
}

int launch_tokcount_vs(const CorpusDev& c, const uint64_t* chunk_start, const uint32_t* chunk_doc, uint64_t c0,
                       uint64_t c1, const VocabDev& v, const K1Out& o, hipStream_t s) {
    if (c1 <= c0) return 0;
    if (v.mask >= (1ull << SLOT_BITS)) return -3; /* slot must fit the LDS entry */
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const uint64_t grid = (c1 - c0) < (uint64_t)ncu * 4 ? (c1 - c0) : (uint64_t)ncu * 4;
    k_tokcount_vs<<<(unsigned)grid, NT, 0, s>>>(c, chunk_start, chunk_doc, c0, c1, v, o);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
