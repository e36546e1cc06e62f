/*
 * tokcount_vs.hip — K1: fused tokenize + per-document term counting, keyed by
 * vocabulary slot.  Replaces the reference's per-rank hot loop TFIDF.c:130-196:
 * fscanf("%s") tokenising (:141-147), the O(P) strcmp search/append of (word, doc)
 * records (:151-167) and the per-rank word table (:169-188).
 *
 * A persistent grid (CUs x 4 workgroups of 256 threads) walks the K0 chunks (~16 KiB of
 * whole documents, or a 16 KiB piece of a document longer than BIG_DOC).  Inside a
 * chunk the four waves work WITHOUT block barriers: wave w takes the 1 KiB steps
 * w, w+4, ... of the chunk, each lane one 16-byte group, two steps of loads in flight.
 *
 *   classify  SWAR whitespace mask (C-locale isspace, TFIDF.c:142,147) per 16-byte group;
 *             document starts of the step (a wave-uniform loop over the group's doc_off
 *             in LDS) start tokens and end the previous ones; the neighbouring lane's
 *             bytes and masks come over DPP lane shifts, the wave's edge lanes prefetch
 *             the group before / after their own;
 *   resolve   each lane walks its own token starts, two at a time: the 128-bit term key
 *             (dev_common.h; strcmp/NUL semantics) is cut from 32 bytes of registers,
 *             hashed with 32-bit multiplies and looked up in the HBM vocabulary (one
 *             16-byte load, both loads of a pair in flight; lock-free insert on a miss);
 *   count     (document, slot) is counted in an LDS open-addressing table of u64 entries
 *             key(36 bits: doc-in-group 8 | slot 28) << 24 | count(24): one 64-bit LDS
 *             CAS claims, one 64-bit LDS add counts.  Claims beyond FILL_LIMIT switch the
 *             workgroup to overflow mode: a (document, term) pair not yet in the table is
 *             written straight to the partial stream with count 1 and its document is
 *             merged later, so the table never fills and never needs a mid-chunk flush;
 *   flush     once per chunk (and document group): entries are grouped per document in
 *             LDS and written as coalesced (slot, count) records — complete documents to
 *             the record stream, documents crossing a chunk edge (or over K5's in-LDS sort
 *             size, or overflowed) to the partial stream merged by finalize.hip.
 *
 * LDS: 32 KiB table + ~6 KiB document state -> four workgroups (16 waves) per CU.
 * Requires a 16-byte aligned corpus base (clamped 16-byte group loads); engine.cpp
 * falls back to tokcount.hip's general kernel otherwise.
 */
#include "dev_common.h"
#include "dev_vocab.h"
#include "kernels.h"

namespace {

#ifndef K1_NT
#define K1_NT 256
#endif
constexpr int NT = K1_NT;               /* threads per workgroup (timing experiments override) */
constexpr int NWAVE = NT / 64;
constexpr int WSTEP = 1024;               /* bytes per wave step: one 16-byte group per lane */
#ifndef K1_TB
#define K1_TB 4096
#endif
constexpr int TB = K1_TB;                 /* LDS table entries (u64), a power of two */
constexpr int EPT = TB / NT;              /* table entries per thread in a flush */
constexpr uint32_t FILL_LIMIT = TB - NT * 2 - 64; /* claims after which overflow mode starts */
constexpr int GCAP = 256;                 /* documents per group (doc-in-group: 8 bits) */
constexpr uint32_t SLOT_BITS = 28;
constexpr uint64_t VS_HOME = ~1ull;     /* even pairs (quads, one 64-byte line per key, measured slower:
                                           c4 K1 4.92 -> 5.36 ms at 32M slots, 6.73 at 16M) */
constexpr uint32_t CNT_BITS = 24;
constexpr uint64_t CNT_MASK = (1ull << CNT_BITS) - 1ull;

constexpr int TLW = 2 * GCAP * 4 / 2 / NWAVE; /* token-list entries per wave (shares dcnt/doff) */

/* Diagnostic build only (-DK1_STAMPS, lib/libtfidf_hip_stamps.so): thread 0 sums
 * s_memtime cycles per phase; never in the measured library.  Phases: 0 group setup,
 * 1 walk (wave 0), 2 flush, 3 docSize write.  Counters: tokens, first-probe misses. */
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
    union {
        struct {
            uint32_t dcnt[GCAP];          /* flush: entries per document */
            uint32_t doff[GCAP];          /* flush: record offset (complete | partial << 16) */
        };
        uint16_t tlist[NWAVE][TLW];       /* walk: each wave's compacted token starts */
    };
    uint32_t drun[GCAP];                  /* flush: running record index per document */
    uint8_t dstate[GCAP];                 /* flush: 0 none, 1 partial, 2 complete */
    uint8_t dpart[GCAP];                  /* document has overflow records */
    uint32_t fill;                        /* table claims of the group */
    uint32_t over;                        /* overflow mode */
    uint32_t wsum[NWAVE];
    unsigned long long rec_base, part_base;
    uint64_t next_chunk;                  /* dynamic chunk schedule */
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
    const uint32_t a = pos < lo ? (uint32_t)min(lo - pos, (uint64_t)16) : 0u;
    const uint32_t b = hi > pos ? (uint32_t)min(hi - pos, (uint64_t)16) : 0u;
    const uint32_t in = b > a ? (((1u << b) - 1u) & ~((1u << a) - 1u)) : 0u;
    return ~in & 0xFFFFu;
}

__device__ __forceinline__ uint32_t tbl_hash(uint64_t key) {
    const uint32_t k = (uint32_t)key ^ (uint32_t)(key >> 28) * 0x9E3779B1u;
    return (k * 0x85EBCA6Bu) >> (32 - 13);   /* & (TB - 1) by the callers */
}

/* wave-uniform copy of a value the compiler keeps in VGPRs (LDS-loaded) */
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

/* Term slot of a token whose term is >= 16 bytes or whose end lies past the 32 bytes a
 * lane holds: the token is re-read from HBM (rare for text). */
__device__ __forceinline__ uint32_t slow_slot(const uint8_t* __restrict__ bytes, const VocabDev& v, uint64_t p0,
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
        return vocab_insert<VS_HOME>(v, klo, khi, 0, status);
    }
    make_long_key(bytes + p0, n, &klo, &khi);
    /* rep = (length << 40) | offset holds 24 length bits: a term of 16 MiB or more would be
     * emitted truncated, so the run fails with TFIDF_E_CAPACITY instead */
    if (n >= 0xFFFFFFull) atomicOr(status, ST_TERM_LONG);
    const uint64_t rep = ((n < 0xFFFFFFull ? n : 0xFFFFFFull) << 40) | p0;
    return vocab_insert<VS_HOME>(v, klo, khi, rep, status, bytes);
}

/* A (document, term) pair met after the table reached FILL_LIMIT and not in it: one
 * partial record of count 1 (finalize.hip sums partial records per (doc, term)). */
__device__ __noinline__ void overflow_record(unsigned long long* part_alloc, uint64_t part_cap, uint32_t* part_doc,
                                             uint32_t* part_slot, uint32_t* part_cnt, uint32_t* status, uint32_t doc,
                                             uint32_t slot) {
    /* one device atomic per wave and call, not per lane: in overflow mode (config 4: every
     * token a new pair) millions of lanes would otherwise queue on this one counter */
    const uint64_t am = __ballot(1);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
    unsigned long long b = 0;
    if (rank == 0u) b = atomicAdd(part_alloc, (unsigned long long)__popcll(am));
    const unsigned long long q = (((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
                                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b)) + rank;
    if (q < part_cap) { part_doc[q] = doc; part_slot[q] = slot; part_cnt[q] = 1u; }
    else atomicOr(status, ST_PART_FULL);
}

__device__ __forceinline__ void overflow_pair(VsShared& S, const K1Out& o, uint64_t key, uint32_t gd0) {
    const uint32_t rel = (uint32_t)(key >> SLOT_BITS);
    S.dpart[rel] = 1;
    overflow_record(o.part_alloc, o.part_cap, o.part_doc, o.part_slot, o.part_cnt, o.status, gd0 + rel,
                    (uint32_t)key & ((1u << SLOT_BITS) - 1u));
}

/* Counts `key` into the table from slot h (the first probe already returned `old`: a
 * CAS, or a plain read in overflow mode; `nx` is a plain read of slot h+1 issued in the
 * same LDS batch, so the common collision costs no extra round trip before the second
 * probe decision).  Returns 1 when this call claimed an entry.
 * A probe sequence longer than PMAX also goes to the partial stream: a pair counted
 * partly in the table and partly as partial records is still summed exactly by the
 * merge, so the table can never fill up or loop. */
constexpr int PMAX = 64;
__device__ __forceinline__ uint32_t tbl_count(VsShared& S, const K1Out& o, uint64_t key, uint32_t h,
                                              unsigned long long old, unsigned long long nx, bool over,
                                              uint32_t gd0) {
    const unsigned long long ent = (key << CNT_BITS) | 1ull;
    if (old != 0ull && (old >> CNT_BITS) != key) {
        /* collision at h: the read-ahead of h+1 decides without a dependent probe */
        h = (h + 1) & (TB - 1);
        if ((nx >> CNT_BITS) == key && nx != 0ull) { atomicAdd(&S.T[h], 1ull); return 0u; }
        old = (nx == 0ull && !over) ? atomicCAS(&S.T[h], 0ull, ent) : nx;
    }
    for (int probe = 2;; ++probe) {
        if (old == 0ull) {
            if (!over) return 1u;
            break;
        }
        if ((old >> CNT_BITS) == key) { atomicAdd(&S.T[h], 1ull); return 0u; }
        if (probe >= PMAX) break;
        h = (h + 1) & (TB - 1);
        old = over ? S.T[h] : atomicCAS(&S.T[h], 0ull, ent);
    }
    overflow_pair(S, o, key, gd0);
    return 0u;
}

/* ctr[idx] += 1 for every active lane.  Most table entries of a flush belong to one
 * document, so a per-lane atomic would serialise up to 64 same-address LDS updates per
 * instruction: when the active lanes agree on idx one lane adds the popcount. */
__device__ __forceinline__ void wave_agg_add(uint32_t* ctr, uint32_t idx) {
    const uint32_t i0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)idx);
    const uint64_t am = __ballot(1);
    if (__ballot(idx != i0) == 0ull) {
        if (__builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u)) == 0u)
            atomicAdd(&ctr[i0], (uint32_t)__popcll(am));
    } else {
        atomicAdd(&ctr[idx], 1u);
    }
}
/* as wave_agg_add, returning this lane's old value (distinct per lane: a running rank) */
__device__ __forceinline__ uint32_t wave_agg_add_rtn(uint32_t* ctr, uint32_t idx) {
    const uint32_t i0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)idx);
    const uint64_t am = __ballot(1);
    uint32_t k;
    if (__ballot(idx != i0) == 0ull) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
        uint32_t b = 0;
        if (rank == 0u) b = atomicAdd(&ctr[i0], (uint32_t)__popcll(am));
        k = (uint32_t)__builtin_amdgcn_readfirstlane((int)b) + rank;
    } else {
        k = atomicAdd(&ctr[idx], 1u);
    }
    return k;
}

/* Emits every table entry of the group as records and clears the table. */
__device__ void vs_flush(VsShared& S, const K1Out& o, uint32_t gd0, uint32_t ng, uint64_t cs, uint64_t ce,
                         Stamps& st) {
    /* opaque copy of the thread index: keeps the per-entry indices (j * NT + tid) from being
     * hoisted out of the chunk loop and spilled — reloading them from scratch in the
     * write-out loop waited on every outstanding record store (vmcnt(0)) per iteration */
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    lds_barrier();   /* every wave's walk is done (the token lists alias dcnt/doff) */
    if (tid < GCAP) S.dcnt[tid] = 0;
    lds_barrier();
    STAMP(st, 12);
    /* pass 1: entries into registers (lane-consecutive, conflict-free), per-document counts */
    unsigned long long e[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        e[j] = S.T[j * NT + tid];
        if (e[j]) wave_agg_add(&S.dcnt[0], (uint32_t)(e[j] >> (CNT_BITS + SLOT_BITS)));
    }
    lds_barrier();
    STAMP(st, 13);
    /* per-document decision, one thread per document */
    uint32_t packed = 0;
    if ((uint32_t)tid < ng) {
        uint8_t st = 0;
        const uint32_t cnt = S.dcnt[tid];
        const bool part = S.dpart[tid] != 0;
        if (cnt) {
            const bool complete = !part && S.gdoc[tid] >= cs && S.gdoc[tid + 1] <= ce && cnt <= (uint32_t)K5_MAX_PAIRS;
            st = complete ? 2 : 1;
            packed = complete ? cnt : (cnt << 16);
        }
        if (st == 1 || part) o.doc_flags[gd0 + tid] = DF_PARTIAL;
        S.dstate[tid] = st;
    }
    uint32_t tot;
    const uint32_t off = block_excl_scan<NT, true>(packed, S.wsum, &tot);
    if ((uint32_t)tid < ng) S.doff[tid] = off;
    const uint32_t nrec = tot & 0xFFFFu, npart = tot >> 16, ntot = nrec + npart;
    /* the two allocations in different waves, so their L2 round trips overlap */
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
    STAMP(st, 14);
    const unsigned long long rb = S.rec_base, pb = S.part_base;
    const bool rec_ok = rb + nrec <= o.rec_cap, part_ok = pb + npart <= o.part_cap;
    if ((uint32_t)tid < ng && S.dstate[tid] == 2) {
        o.doc_recoff[gd0 + tid] = rb + (off & 0xFFFFu);
        o.doc_npairs[gd0 + tid] = S.dcnt[tid];
    }
    /* pass 2: stage entries in the (already read) table in output order — complete
     * records [0, nrec), partial records [nrec, ntot) — for coalesced HBM writes */
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        if (e[j]) {
            const uint32_t rel = (uint32_t)(e[j] >> (CNT_BITS + SLOT_BITS));
            const uint32_t slot = (uint32_t)(e[j] >> CNT_BITS) & ((1u << SLOT_BITS) - 1u);
            const uint64_t cnt = e[j] & CNT_MASK;
            const uint32_t k = wave_agg_add_rtn(&S.drun[0], rel);
            const uint32_t dof = S.doff[rel];
            if (S.dstate[rel] == 2) S.T[(dof & 0xFFFFu) + k] = slot | (cnt << 32);
            else S.T[nrec + (dof >> 16) + k] = slot | ((uint64_t)rel << SLOT_BITS) | (cnt << 36);
        }
    }
    lds_barrier();
    STAMP(st, 15);
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
    STAMP(st, 16);
}

}  // namespace

/* Persistent: a grid of (CUs x 4) workgroups walks the chunks [c0, c1) round-robin. */
#ifndef K1_WAVES_PER_SIMD
#define K1_WAVES_PER_SIMD 4
#endif
__global__ __launch_bounds__(NT, K1_WAVES_PER_SIMD) void k_tokcount_vs(CorpusDev c, const uint64_t* __restrict__ chunk_start,
                                                       const uint32_t* __restrict__ chunk_doc, uint64_t c0,
                                                       uint64_t c1, VocabDev v, K1Out o) {
    __shared__ __attribute__((aligned(16))) VsShared S;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t last_blk = c.nbytes ? ((c.nbytes - 1) & ~(uint64_t)15) : 0;
    const bool edge_lane = lane == 0 || lane == 63;
    const uint64_t eoff = lane == 0 ? (uint64_t)0 - 16ull : 16ull;

#pragma unroll
    for (int j = 0; j < EPT; ++j) S.T[j * NT + tid] = 0ull;
    unsigned long long tokens_wg = 0;
    Stamps st;
#ifdef K1_STAMPS
    st.prev = 0;
    for (int k = 0; k < K1_NSTAMP; ++k) st.acc[k] = 0;
    uint32_t cnt_[K1_NCOUNT] = {0, 0, 0, 0};
#endif
    STAMP(st, 0);

    /* one token round of the wave (one token per lane): its key, document, vocabulary
     * hash and the two vocabulary slots loaded for it */
    struct Round {
        uint64_t klo, khi, ap;
        uint32_t hv, rel, kind;
        uint4 s4, t4;
    };
    Round pend{};
    bool pending = false;
    uint32_t gd0_cur = 0;
    /* finish a round: vocabulary slot (miss path: lock-free insert / long term), docSize,
     * LDS (doc, slot) count, overflow accounting */
    auto claims_finish = [&](const Round& r) {
        uint32_t slot = INVALID_SLOT;
        if (r.kind == 1u) {
            const bool hit0 = r.s4.x == (uint32_t)r.klo && r.s4.y == (uint32_t)(r.klo >> 32) &&
                              r.s4.z == (uint32_t)r.khi && r.s4.w == (uint32_t)(r.khi >> 32);
            const bool hit1 = r.t4.x == (uint32_t)r.klo && r.t4.y == (uint32_t)(r.klo >> 32) &&
                              r.t4.z == (uint32_t)r.khi && r.t4.w == (uint32_t)(r.khi >> 32);
            CNT(1, (hit0 || hit1) ? 0 : 1);
            slot = hit0 ? r.hv : hit1 ? ((r.hv + 1) & (uint32_t)v.mask) : vocab_insert<VS_HOME>(v, r.klo, r.khi, 0, o.status);
        } else if (r.kind == 2u) {
            slot = slow_slot(c.bytes, v, r.ap, S.gdoc[r.rel + 1], o.status);
        }
        STAMP(st, 7);
        /* docSize: one LDS add per wave when the round's tokens share a document */
        {
            const uint64_t vm = __ballot(r.kind != 0u);
            if (vm) {
                const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.rel);
                if (__ballot(r.kind != 0u && r.rel != r0) == 0ull) {
                    if (lane == 0) atomicAdd(&S.dsz[r0], (uint32_t)__popcll(vm));
                } else if (r.kind) {
                    atomicAdd(&S.dsz[r.rel], 1u);
                }
            }
        }
        STAMP(st, 8);
        /* invalid slot: status flagged, the run is retried */
        const uint64_t key = slot == INVALID_SLOT ? ~0ull : (((uint64_t)r.rel << SLOT_BITS) | slot);
        const uint32_t hl = tbl_hash(key) & (TB - 1);
        /* first LDS probe: a CAS claim, or a plain read in overflow mode */
        const bool over = S.over != 0;
        const bool valid = key != ~0ull;
        unsigned long long old = 0ull, nx = 0ull;
        if (valid) {
            old = over ? S.T[hl] : atomicCAS(&S.T[hl], 0ull, (key << CNT_BITS) | 1ull);
            nx = S.T[(hl + 1) & (TB - 1)];
        }
        /* the common outcomes (claimed, or counted at the home slot) stay branch-light;
         * collisions and overflow mode take tbl_count, entered once per wave if any lane
         * needs it */
        const bool hit = valid && old != 0ull && (old >> CNT_BITS) == key;
        const bool claimed = valid && old == 0ull && !over;
        if (hit) atomicAdd(&S.T[hl], 1ull);
        uint32_t claims = claimed ? 1u : 0u;
        const bool rest = valid && !hit && !claimed;
        if (__ballot(rest) != 0ull) {
            if (rest) claims = tbl_count(S, o, key, hl, old, nx, over, gd0_cur);
        }
        STAMP(st, 9);
        /* claims -> overflow mode: one LDS add per wave and round */
        const uint32_t wc = (uint32_t)__popcll(__ballot(claims != 0u));
        if (wc && lane == 0) {
            const uint32_t f = atomicAdd(&S.fill, wc);
            if (f + wc >= FILL_LIMIT) S.over = 1;
        }
        STAMP(st, 10);
    };

    /* chunks are handed out by a global counter (chunk sizes vary up to BIG_DOC, so a
     * static round-robin share leaves a tail of the slowest workgroups); the next index
     * is claimed when a chunk starts, so the atomic's round trip is hidden */
    if (tid == 0) S.next_chunk = c0 + atomicAdd(o.chunk_ctr, 1ull);
    lds_barrier();
    uint64_t next_claim = 0;
    for (uint64_t chunk = uni64(S.next_chunk); chunk < c1; chunk = uni64(S.next_chunk)) {
        if (tid == 0) next_claim = c0 + atomicAdd(o.chunk_ctr, 1ull);
        const uint64_t cs = chunk_start[chunk], ce = chunk_start[chunk + 1];
        const uint32_t dfirst = chunk_doc[chunk], dlast = chunk_doc[chunk + 1];
        if (cs < ce)
        for (uint32_t gd0 = dfirst; gd0 <= dlast; gd0 += GCAP) {
            gd0_cur = gd0;
            const uint32_t ng = (dlast + 1 - gd0) < (uint32_t)GCAP ? (dlast + 1 - gd0) : (uint32_t)GCAP;
            for (uint32_t k = tid; k <= ng; k += NT) S.gdoc[k] = c.doc_off[gd0 + k];
            if (tid < GCAP) { S.dsz[tid] = 0; S.dpart[tid] = 0; S.drun[tid] = 0; }
            if (tid == 0) { S.fill = 0; S.over = 0; }
            lds_barrier();
            const uint64_t g0 = uni64(S.gdoc[0]), gn = uni64(S.gdoc[ng]);
            const uint64_t gs = g0 > cs ? g0 : cs;
            const uint64_t ge = gn < ce ? gn : ce;
            STAMP(st, 0);
            if (gs < ge) {
                /* ---- barrier-free walk: wave wid takes steps wid, wid + 4, ... ---- */
                const uint64_t b0 = gs & ~(uint64_t)15;
                const uint32_t nsteps = (uint32_t)((ge - b0 + WSTEP - 1) / WSTEP);
                const uint64_t lane_off = 16ull * lane;
                uint4 pf0 = make_uint4(0, 0, 0, 0), pe0 = pf0;
                {
                    const uint64_t a0 = b0 + (uint64_t)wid * WSTEP + lane_off;
                    pf0 = ld16c(c.bytes, last_blk, a0);
                    if (edge_lane) pe0 = ld16c(c.bytes, last_blk, a0 + eoff);
                }
                uint32_t wr = 0;             /* wave-uniform: document containing the step start */
                uint16_t* tl = S.tlist[wid];
                for (uint32_t s = wid; s < nsteps; s += NWAVE) {
                    const uint64_t sb = b0 + (uint64_t)s * WSTEP;
                    const uint64_t gpos = sb + lane_off;
                    /* one step of prefetch: the copy into `cur` waits for the load issued a
                     * step ago (a second buffer's copy forced a wait for the load just
                     * issued at every step end) */
                    const uint4 cur = pf0, edge = pe0;
                    {
                        const uint64_t a1 = gpos + 1ull * NWAVE * WSTEP; /* harmless past ge */
                        pf0 = ld16c(c.bytes, last_blk, a1);
                        if (edge_lane) pe0 = ld16c(c.bytes, last_blk, a1 + eoff);
                    }
                    STAMP(st, 11);
                    /* ---- classify (per lane, one 16-byte group) ---- */
                    const bool inner = sb >= c.lo + 16 && sb + WSTEP + 16 <= c.hi;
                    uint32_t ws = ws_mask16_swar(cur);
                    if (!inner) ws |= bounds_ws(gpos, c.lo, c.hi);
                    /* document starts in [sb, sb + WSTEP + 16): wave-uniform loop */
                    while (wr + 1 < ng && uni64(S.gdoc[wr + 1]) <= sb) ++wr;
                    uint32_t ds = 0, nds = 0, kend = wr + 1;
                    for (uint32_t k = wr; k <= ng; ++k) {
                        const uint64_t sk = uni64(S.gdoc[k]);
                        if (sk >= sb + WSTEP + 16) break;
                        kend = k + 1;
                        if (sk >= gpos && sk < gpos + 16) ds |= 1u << (uint32_t)(sk - gpos);
                        if (sk >= gpos + 16 && sk < gpos + 32) nds |= 1u << (uint32_t)(sk - gpos - 16);
                    }
                    if (kend > ng) kend = ng;
                    const uint32_t stop = ws | ds;
                    uint32_t prev = (lane_prev(ws) >> 15) & 1u;
                    if (lane == 0) prev = (gpos > c.lo && gpos - 1 < c.hi) ? (is_ws(edge.w >> 24) ? 1u : 0u) : 1u;
                    uint32_t own = 0xFFFFu;
                    if (!(sb >= gs && sb + WSTEP <= ge)) {
                        own = 0;
                        if (gpos + 16 > gs && gpos < ge) {
                            const uint32_t a = gpos < gs ? (uint32_t)(gs - gpos) : 0u;
                            const uint32_t b = gpos + 16 > ge ? (uint32_t)(ge - gpos) : 16u;
                            own = ((1u << b) - 1u) & ~((1u << a) - 1u);
                        }
                    }
                    const uint32_t starts = ~ws & ((ws << 1) | prev | ds) & own & 0xFFFFu;
                    uint4 nxt;
                    nxt.x = lane_next(cur.x);
                    nxt.y = lane_next(cur.y);
                    nxt.z = lane_next(cur.z);
                    nxt.w = lane_next(cur.w);
                    uint32_t nstop = lane_next(stop);
                    if (lane == 63) {
                        nxt = edge;
                        uint32_t nws = ws_mask16_swar(edge);
                        if (!inner) nws |= bounds_ws(gpos + 16, c.lo, c.hi);
                        nstop = nws | nds;
                    }
                    const uint32_t s32 = stop | (nstop << 16);
                    STAMP(st, 4);
                    /* ---- compact the step's token starts (wave prefix sum) ---- */
                    const uint32_t nmine = (uint32_t)__popc(starts);
                    const uint32_t incl = wave_incl_scan(nmine);
                    const uint32_t ntok = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                    if (ntok == 0) continue;
                    tokens_wg += ntok;
                    for (uint32_t base = 0; base < ntok; base += TLW) {
                        {
                            uint32_t sm = starts, idx = incl - nmine;
                            while (sm) {
                                const uint32_t i = __builtin_ctz(sm);
                                sm &= sm - 1;
                                if (idx - base < (uint32_t)TLW) tl[idx - base] = (uint16_t)((lane << 4) | i);
                                ++idx;
                            }
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        const uint32_t cnt = (ntok - base) < (uint32_t)TLW ? (ntok - base) : (uint32_t)TLW;
                        STAMP(st, 5);
                        /* ---- resolve + count, 64 tokens per round, all lanes busy; the
                         * vocabulary loads of round r+1 are issued before round r is
                         * counted (one round in flight, also across steps) ---- */
                        for (uint32_t t0 = 0; t0 < cnt; t0 += 64) {
                            Round q;
                            {
                                const uint32_t t = t0 + lane;
                                const bool val = t < cnt;
                                const uint32_t pos = val ? (uint32_t)tl[t] : 0u;
                                const uint32_t src = pos >> 4, i = pos & 15u;
                                const int ba = (int)(src << 2);
                                const uint32_t c0 = __builtin_amdgcn_ds_bpermute(ba, cur.x), c1 = __builtin_amdgcn_ds_bpermute(ba, cur.y);
                                const uint32_t c2 = __builtin_amdgcn_ds_bpermute(ba, cur.z), c3 = __builtin_amdgcn_ds_bpermute(ba, cur.w);
                                const uint32_t n0 = __builtin_amdgcn_ds_bpermute(ba, nxt.x), n1 = __builtin_amdgcn_ds_bpermute(ba, nxt.y);
                                const uint32_t n2 = __builtin_amdgcn_ds_bpermute(ba, nxt.z), n3 = __builtin_amdgcn_ds_bpermute(ba, nxt.w);
                                const uint32_t sv = __builtin_amdgcn_ds_bpermute(ba, s32);
                                const uint64_t q0 = ((uint64_t)c1 << 32) | c0, q1 = ((uint64_t)c3 << 32) | c2;
                                const uint64_t q2 = ((uint64_t)n1 << 32) | n0, q3 = ((uint64_t)n3 << 32) | n2;
                                const uint32_t m = sv >> (i + 1);
                                const uint32_t len = m ? (uint32_t)__builtin_ctz(m) + 1u : 32u;
                                const uint32_t sh = (i & 7u) * 8u;
                                const uint64_t a = i < 8 ? q0 : q1, b = i < 8 ? q1 : q2, cc = i < 8 ? q2 : q3;
                                const uint64_t lo = sh ? (a >> sh) | (b << (64 - sh)) : a;
                                const uint64_t hi = sh ? (b >> sh) | (cc << (64 - sh)) : b;
                                q.kind = val ? (make_short_key(lo, hi, len, &q.klo, &q.khi) < 16u ? 1u : 2u) : 0u;
                                q.ap = sb + pos;
                                /* document: wr plus the step's document starts at or before the token */
                                uint32_t rel = wr;
                                for (uint32_t k = wr + 1; k < kend; ++k) rel += uni64(S.gdoc[k]) <= q.ap ? 1u : 0u;
                                q.rel = rel;
                                q.hv = q.kind == 1u ? (uint32_t)(key_hash(q.klo, q.khi) & v.mask & VS_HOME) : 0u;   /* home (dev_vocab.h) */
                                /* the home slot and the next one: a key displaced by one slot
                                 * (linear probing) still resolves without a dependent load */
                                q.s4 = v.keys[q.hv];
                                q.t4 = v.keys[(q.hv + 1) & (uint32_t)v.mask];
                            }
                            STAMP(st, 6);
                            if (pending) claims_finish(pend);
                            pend = q;
                            pending = true;
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
                }
            }
            if (pending) { claims_finish(pend); pending = false; }
#ifdef K1_STAMPS
            STAMP(st, 10);
            lds_barrier();   /* diagnostic: separates the wait for the other waves */
#endif
            STAMP(st, 1);
            /* group end is a document boundary (or the chunk end): emit everything */
            vs_flush(S, o, gd0, ng, cs, ce, st);
            STAMP(st, 2);
            if ((uint32_t)tid < ng) {
                const uint32_t n = S.dsz[tid];
                if (n) {
                    const uint32_t d = gd0 + tid;
                    if (S.gdoc[tid] >= cs && S.gdoc[tid + 1] <= ce) o.doc_size[d] = n;
                    else atomicAdd(&o.doc_size[d], n);
                }
            }
            lds_barrier();
            STAMP(st, 3);
            if (gd0 + GCAP < gd0) break; /* overflow guard */
        }
        if (tid == 0) S.next_chunk = next_claim;
        lds_barrier();
    }
    /* tokens (wave-uniform count): one atomic per wave */
    if (lane == 0 && tokens_wg) atomicAdd(o.ntokens, tokens_wg);
#ifdef K1_STAMPS
    if (tid == 0 && o.stamps) {
        for (int k = 0; k < K1_NSTAMP; ++k) atomicAdd(&o.stamps[k], (unsigned long long)st.acc[k]);
        atomicAdd(&o.stamps[K1_NSTAMP], 1ull);
    }
    CNT(0, (uint32_t)tokens_wg);
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
#ifndef K1_WGS_PER_CU
#define K1_WGS_PER_CU 4
#endif
    const uint64_t wgs = (uint64_t)ncu * K1_WGS_PER_CU;
    const uint64_t grid = (c1 - c0) < wgs ? (c1 - c0) : wgs;
    k_tokcount_vs<<<(unsigned)grid, NT, 0, s>>>(c, chunk_start, chunk_doc, c0, c1, v, o);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
