/*
 * tokcount_st.hip — K1: fused tokenize + per-document term counting with an LDS-staged
 * walk.  Replaces the reference's per-rank hot loop TFIDF.c:130-196: fscanf("%s")
 * tokenising (:141-147), the O(P) strcmp search/append of (word, doc) records (:151-167)
 * and the per-rank word table (:169-188).
 *
 * Work split (as tokcount_vs.hip): a persistent grid takes K0's chunks (~24 KiB of whole
 * documents, or a piece of a document longer than BIG_DOC) from a global counter; inside
 * a chunk the four waves of a workgroup run without block barriers, wave w taking the
 * 1 KiB steps w, w+4, ...; (document, term) pairs are counted in one LDS table per
 * workgroup and flushed as coalesced records once per chunk.
 *
 * What makes a token cheap here — everything positional is settled ONCE per 16-byte group
 * in the walk, so the per-token round is a straight line:
 *   walk   each lane classifies its 16 bytes (SWAR C-locale isspace, TFIDF.c:142,147, and
 *          NUL: strcmp/strcpy stop there, :152,172), finds its document starts and the
 *          document index of its first byte, and stores its bytes in the wave's LDS stage
 *          (plus the 16 bytes after the step).  The lane that owns a token start then
 *          writes one 32-bit token entry: byte offset | term length (distance to the next
 *          whitespace, document start or NUL — read from its own and the next lane's
 *          masks) | document index.
 *   round  64 tokens, one per lane: the entry, ONE unaligned ds_read_b128 of the term's
 *          bytes from the stage, ONE ds_read_b128 of the v_perm selectors for its length
 *          (bytes < n kept, byte n = TAB, the rest zero: the 128-bit identity key of
 *          dev_common.h in four v_perm_b32), the vocabulary hash, two adjacent vocabulary
 *          slots loaded in one go, then the (document, slot) count in LDS.  The next
 *          round's vocabulary loads are issued before the current round is counted.
 * Terms of 16 bytes or more (and tokens running past the 32-byte window) take the HBM
 * slow path of tokcount_vs.hip.  The flush, the overflow mode (partial records merged by
 * finalize.hip) and the record layout are tokcount_vs.hip's.
 *
 * LDS: 28 KiB table + ~10 KiB walk/document state -> four workgroups (16 waves) per CU.
 * Requires a 16-byte aligned corpus base (engine.cpp falls back to tokcount.hip).
 */
#include "dev_common.h"
#include "dev_vocab.h"
#include "kernels.h"


/* Diagnostic build only (-DK1_STAMPS, make variant NAME=stamps DEFS=-DK1_STAMPS, run with
 * TFIDF_STAMPS=1): lane 0 of every wave sums s_memtime cycles per phase — 0 chunk set-up
 * (claim, metadata, group set-up up to its barrier), 1 walk (classify, token entries),
 * 2 token rounds, 3 drain, 4 wait at the flush barrier (the other waves' walks), 5 flush,
 * 6 document sizes + chunk end — then the chunk count (word 7) and the wave count (word
 * 8); never in the measured library. */
#define K1S_NPH 7
#ifdef K1_STAMPS
#define STP(k)                                                              \
    do {                                                                    \
        if (lane == 0) {                                                    \
            __builtin_amdgcn_sched_barrier(0);                              \
            const uint64_t t_ = __builtin_amdgcn_s_memtime();               \
            __builtin_amdgcn_s_waitcnt(0xC07F);                             \
            if (st_prev) st_acc[st_ph] += t_ - st_prev;                     \
            st_prev = t_;                                                   \
            st_ph = (k);                                                    \
            __builtin_amdgcn_sched_barrier(0);                              \
        }                                                                   \
    } while (0)
#else
#define STP(k) do { } while (0)
#endif

namespace {

constexpr int NT = 256;                /* threads per workgroup */
constexpr int WG_PER_CU = 4;                /* 16 waves per CU */
constexpr int NWAVE = NT / 64;
constexpr int WSTEP = 992;                /* bytes a wave step owns: lanes 1..62, one 16-byte group each;
                                             lane 0 holds the 16 bytes before (the byte before
                                             the step), lane 63 the 16 after (terms crossing the
                                             step end): no separate edge loads or edge lanes */
constexpr int TB = 3584;                /* LDS table entries (u32 key + u32 count): 14 per thread */
constexpr int EPT = TB / NT;
constexpr uint32_t FILL_LIMIT = TB - NT * 2 - 64; /* claims after which overflow mode starts */
constexpr int GCAP = 256;            /* documents per group at most (LDS arrays) */
static_assert(GCAP <= NT, "one thread per document of a group");
constexpr uint32_t SLOT_BITS = 28;        /* vocabulary slots < 2^28 */
constexpr int TLW = 192;                  /* token entries per wave and compaction pass */
constexpr uint32_t LEN_LONG = 31u;

struct StShared {
    uint32_t TK[TB];                      /* key32 = 1 << 31 | doc-in-group << sb | slot (0: empty) */
    uint32_t TC[TB];                      /* its count */
    uint64_t gdoc[GCAP + 1];              /* doc_off of the group's documents */
    uint32_t dsz[GCAP];                   /* docSize accumulators */
    union {
        struct {                          /* walk */
            uint4 stage[NWAVE][64];       /* the step's 64 groups: [sb - 16, sb + 1008) */
            uint32_t tl[NWAVE][TLW];
        } w;
        struct {                          /* flush */
            uint32_t dcnt[GCAP];          /* entries per document */
            uint32_t doff[GCAP];          /* record offset (complete | partial << 16) */
            uint32_t drun[GCAP];          /* running record index per document */
            uint8_t dstate[GCAP];         /* 0 none, 1 partial, 2 complete */
        } f;
    };
    uint4 sel[16];                        /* v_perm selectors of a term of length n */
    uint64_t fbase[8];                    /* st_flush_few: first record of each document */
    uint8_t dpart[GCAP];                  /* document has overflow records */
    uint32_t fill;                        /* table claims of the group */
    uint64_t cur_chunk, nxt_chunk;        /* dynamic chunk schedule: this chunk and the next */
    uint32_t wsum[NWAVE];
    unsigned long long rec_base, part_base;
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));   /* unaligned LDS read */

/* streaming corpus load: clamped to the last 16-byte block, non-temporal (read once) */
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

/* bit 7 of every zero byte (exact) */
__device__ __forceinline__ uint32_t zero_bits(uint32_t x) { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u; }
__device__ __forceinline__ uint32_t compress4(uint32_t m) {   /* bits 7, 15, 23, 31 -> bits 0-3 */
    m >>= 7;
    m |= m >> 7;
    m |= m >> 14;
    return m & 0xFu;
}

/* The LDS count table: buckets of BW slots (TK: 32-bit keys, 0 = empty; TC: counts).  A
 * key lives in its home bucket unless that bucket was full when it was inserted, then in
 * the next bucket with room (slots are only emptied by the flush, so a home bucket with an
 * empty slot proves a key is not further on).  With 4-slot buckets a c2 chunk's ~1000
 * keys in 896 buckets leave the home bucket full for ~2.6 % of new keys, which sends about
 * half of all rounds through bkt_slow (0.2 ms of K1, measured in round 2 with slow keys
 * dropped); 8-slot buckets (two ds_read_b128) make that rare but cost the same in compares
 * at 16 KiB chunks (c2 2.255 vs 2.222 ms, c5 2.441 vs 2.432 ms).  With 24 KiB chunks
 * (CHUNK_BYTES_ST: ~1.5x the keys per group) 8-slot buckets win: c2 K1 2.233 -> 2.161 ms,
 * c5 2.434 -> 2.315 ms, and no more overflow records than 16 KiB chunks with 4-slot ones
 * (4-slot buckets at 24 KiB: merge c2 0.10 -> 0.125 ms), profiles/r03_chunk_ab.txt. */
#ifndef K1S_BW
#define K1S_BW 8
#endif
constexpr uint32_t BW = K1S_BW;
static_assert(BW == 4 || BW == 8, "bucket width");
constexpr uint32_t NB = TB / BW;
struct BktK {
    uint4 a, b;                           /* slots 0-3, 4-7 (b unused for 4-slot buckets) */
};
__device__ __forceinline__ uint32_t bkt_hash(uint32_t key) {
    return (uint32_t)(((uint64_t)(key * 0x9E3779B1u) * (uint64_t)NB) >> 32);   /* [0, NB) */
}
__device__ __forceinline__ uint32_t bkt_next(uint32_t b) { return b + 1 == NB ? 0u : b + 1; }
__device__ __forceinline__ BktK bkt_read(StShared& S, uint32_t b) {
    const uint4* t = reinterpret_cast<const uint4*>(S.TK) + b * (BW / 4);
    BktK k;
    k.a = t[0];
    k.b = BW == 8 ? t[1] : make_uint4(0, 0, 0, 0);
    return k;
}
/* slot of `key` in bucket kk (BW if absent) */
__device__ __forceinline__ uint32_t bkt_match(const BktK& kk, uint32_t key) {
    uint32_t j = kk.a.x == key ? 0u : kk.a.y == key ? 1u : kk.a.z == key ? 2u : kk.a.w == key ? 3u : 4u;
    if (BW == 8 && j == 4u)
        j = kk.b.x == key ? 4u : kk.b.y == key ? 5u : kk.b.z == key ? 6u : kk.b.w == key ? 7u : 8u;
    return j;
}
/* the first empty slot of bucket kk, scanning from slot key % BW (different keys spread over
 * the free slots of a bucket they share), BW if full */
__device__ __forceinline__ uint32_t bkt_empty(const BktK& kk, uint32_t key) {
    uint32_t em = (kk.a.x == 0u ? 1u : 0u) | (kk.a.y == 0u ? 2u : 0u) | (kk.a.z == 0u ? 4u : 0u) | (kk.a.w == 0u ? 8u : 0u);
    if (BW == 8)
        em |= (kk.b.x == 0u ? 16u : 0u) | (kk.b.y == 0u ? 32u : 0u) | (kk.b.z == 0u ? 64u : 0u) | (kk.b.w == 0u ? 128u : 0u);
    if (!em) return BW;
    const uint32_t r0 = key & (BW - 1u);
    const uint32_t rot = ((em | (em << BW)) >> r0) & ((1u << BW) - 1u);
    return ((uint32_t)__builtin_ctz(rot) + r0) & (BW - 1u);
}
__device__ __forceinline__ void tbl_read(StShared& S, uint32_t i, uint32_t& key, uint32_t& cnt) { key = S.TK[i]; cnt = S.TC[i]; }
__device__ __forceinline__ void tbl_clear(StShared& S, uint32_t i) { S.TK[i] = 0u; S.TC[i] = 0u; }

/* The next chunk for a workgroup whose current counter shard is `sh`.  One device-scope
 * counter saturates at ~88 claims per microsecond (MI355X_MICROARCH.md, price list
 * "dequeue"): c2's 57 442 chunks alone would take 0.65 ms through it.  The chunks are cut
 * into 8 contiguous shards with a counter each; a workgroup claims from its home shard
 * (blockIdx.x & 7) and moves on to the next shard once that one is exhausted, so every
 * chunk is claimed exactly once and a finished shard costs each workgroup one extra
 * atomic.  Returns c0 + n when nothing is left. */
__device__ __forceinline__ uint64_t claim_chunk(unsigned long long* ctr, uint32_t& sh, uint64_t c0, uint64_t n) {
    for (int t = 0; t < 8; ++t) {
        const uint64_t lo = n * sh / 8, hi = n * (sh + 1) / 8;
        if (hi > lo) {
            const uint64_t v = atomicAdd(&ctr[sh], 1ull);
            if (lo + v < hi) return c0 + lo + v;
        }
        sh = (sh + 1) & 7u;
    }
    return c0 + n;
}

__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

/* term slot of a token whose term is >= 16 bytes (or runs past the 32-byte window): the
 * token is re-read from HBM (rare for text) */
/* (VocabDev by reference puts the kernel's copy in scratch, so the rounds reload the table
 * pointer / mask with scratch loads; passed by value it stays in SGPRs, but then 14 more
 * SGPRs spill and K1 measured 2.37-2.38 vs 2.23 ms on c2: kept by reference) */
__device__ __noinline__ uint32_t slow_slot(const uint8_t* __restrict__ bytes, const VocabDev& v, uint64_t p0,
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
    /* rep = (length << 40) | offset holds 24 length bits: a term of 16 MiB or more would be
     * emitted truncated, so the run fails with TFIDF_E_CAPACITY instead */
    if (n >= 0xFFFFFFull) atomicOr(status, ST_TERM_LONG);
    const uint64_t rep = ((n < 0xFFFFFFull ? n : 0xFFFFFFull) << 40) | p0;
    return vocab_insert(v, klo, khi, rep, status);
}

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

/* Counts `key` the slow way, from bucket b on, re-reading each bucket: the home bucket was
 * full without the key, another lane's claim took the free slot this lane wanted, or the
 * group is in overflow mode.  Returns 1 when this call claimed a slot.  A key not in the
 * table in overflow mode, or after PMAX buckets, becomes a partial record of count 1 (the
 * merge sums them), so the table never fills or loops. */
constexpr int PMAX = 16;
#ifndef BKT_SLOW_ATTR
#define BKT_SLOW_ATTR __forceinline__
#endif
__device__ BKT_SLOW_ATTR uint32_t bkt_slow(StShared& S, const K1Out& o, uint32_t key, uint32_t b, bool over,
                                          uint32_t gd0, uint32_t sb) {
    for (int probe = 0, tries = 0; probe < PMAX && tries < 64; ++tries) {
        const BktK kk = bkt_read(S, b);
        const uint32_t j = bkt_match(kk, key);
        if (j < BW) { atomicAdd(&S.TC[BW * b + j], 1u); return 0u; }
        const uint32_t e = bkt_empty(kk, key);
        if (e < BW) {
            if (over) break;               /* not in the table: a bucket with room ends the chain */
            const uint32_t old = atomicCAS(&S.TK[BW * b + e], 0u, key);
            if (old == 0u || old == key) {
                atomicAdd(&S.TC[BW * b + e], 1u);
                return old == 0u ? 1u : 0u;
            }
            continue;                      /* lost the slot to another key: re-read this bucket */
        }
        b = bkt_next(b);
        ++probe;
    }
    const uint32_t rel = (key & 0x7FFFFFFFu) >> sb;
    S.dpart[rel] = 1;
    overflow_record(o.part_alloc, o.part_cap, o.part_doc, o.part_slot, o.part_cnt, o.status, gd0 + rel,
                    key & ((1u << sb) - 1u));
    return 0u;
}

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

/* Emits every table entry of the group as records and clears the table: complete
 * documents to the record stream, documents crossing a chunk edge, over K5's in-LDS sort
 * size or overflowed to the partial stream.  Per-document counts (wave-aggregated LDS
 * adds), a block scan of them, then every entry is written straight to its record slot
 * (its rank inside its document from a wave-aggregated LDS counter): no LDS staging pass. */
__device__ void st_flush(StShared& S, const K1Out& o, uint32_t gd0, uint32_t ng, uint64_t cs, uint64_t ce,
                         uint32_t sb) {
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));   /* keep j * NT + tid out of the chunk loop (no spills) */
    lds_barrier();                  /* every wave's walk is done (the walk state aliases dcnt...) */
    if (tid < GCAP) { S.f.dcnt[tid] = 0; S.f.drun[tid] = 0; }
    lds_barrier();
    const uint32_t smask = (1u << sb) - 1u;
    uint32_t ek[EPT], ec[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        tbl_read(S, j * NT + tid, ek[j], ec[j]);
        if (ek[j]) wave_agg_add(&S.f.dcnt[0], (ek[j] & 0x7FFFFFFFu) >> sb);
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
        if (st == 1 || part) o.doc_flags[gd0 + tid] = DF_PARTIAL;
        S.f.dstate[tid] = st;
    }
    uint32_t tot;
    const uint32_t off = block_excl_scan<NT, true>(packed, S.wsum, &tot);
    if ((uint32_t)tid < ng) S.f.doff[tid] = off;
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
    if ((uint32_t)tid < ng && S.f.dstate[tid] == 2) {
        o.doc_recoff[gd0 + tid] = rb + (off & 0xFFFFu);
        o.doc_npairs[gd0 + tid] = S.f.dcnt[tid];
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const uint32_t key = ek[j];
        if (key) {
            const uint32_t rel = (key & 0x7FFFFFFFu) >> sb;
            const uint32_t k = wave_agg_add_rtn(&S.f.drun[0], rel);
            const uint32_t dof = S.f.doff[rel];
            if (S.f.dstate[rel] == 2) {
                const uint64_t q = rb + (dof & 0xFFFFu) + k;
                if (rec_ok) { o.rec_slot[q] = key & smask; o.rec_cnt[q] = ec[j]; }
            } else {
                const uint64_t q = pb + (dof >> 16) + k;
                if (part_ok) { o.part_doc[q] = gd0 + rel; o.part_slot[q] = key & smask; o.part_cnt[q] = ec[j]; }
            }
            tbl_clear(S, j * NT + tid);
        }
    }
}

/* The flush of a group of at most FEW documents (most c2 chunks hold one or two): every
 * thread counts its entries per document in 16-bit fields of FEW/2 words, one block scan
 * of those words gives each thread its first rank in every document and the documents'
 * totals, one thread allocates the records, and every entry is written at document base
 * + rank with no LDS atomic.  Same output as st_flush. */
constexpr uint32_t FEW = 8;
__device__ void st_flush_few(StShared& S, const K1Out& o, uint32_t gd0, uint32_t ng, uint64_t cs, uint64_t ce,
                             uint32_t sb) {
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, w = tid >> 6;
    lds_barrier();                  /* every wave's walk is done */
    const uint32_t smask = (1u << sb) - 1u;
    uint32_t ek[EPT], ec[EPT];
    uint32_t pk[FEW / 2] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        tbl_read(S, j * NT + tid, ek[j], ec[j]);
        if (ek[j]) {
            const uint32_t rel = (ek[j] & 0x7FFFFFFFu) >> sb;
#pragma unroll
            for (uint32_t q = 0; q < FEW / 2; ++q)
                pk[q] += (rel >> 1) == q ? (1u << (16 * (rel & 1u))) : 0u;
        }
    }
    /* block exclusive scan of the FEW/2 packed words (fields never carry: totals <= TB) */
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
    /* per document (lane d of wave 0): complete (record stream) or partial; one wave scan
     * of the documents' counts gives their offsets; lanes 0 and 32 allocate the records */
    if (w == 0) {
        const uint32_t d = (uint32_t)lane;
        uint32_t cnt = 0, packed = 0;
        uint8_t st = 0;
        bool part = false;
        if (d < ng) {
#pragma unroll
            for (uint32_t q = 0; q < FEW / 2; ++q)
                if ((d >> 1) == q) cnt = (tot[q] >> (16 * (d & 1u))) & 0xFFFFu;
            part = S.dpart[d] != 0;
            if (cnt) {
                const bool complete = !part && S.gdoc[d] >= cs && S.gdoc[d + 1] <= ce && cnt <= (uint32_t)K5_MAX_PAIRS;
                st = complete ? 2 : 1;
                packed = complete ? cnt : (cnt << 16);
            }
            if (st == 1 || part) o.doc_flags[gd0 + d] = DF_PARTIAL;
        }
        const uint32_t incl = wave_incl_scan(packed);
        const uint32_t all = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t off = incl - packed;
        const uint32_t nrec = all & 0xFFFFu, npart = all >> 16;
        unsigned long long a0 = 0, a1 = 0;
        if (lane == 0 && nrec) a0 = atomicAdd(o.rec_alloc, (unsigned long long)nrec);
        if (lane == 32 && npart) a1 = atomicAdd(o.part_alloc, (unsigned long long)npart);
        const unsigned long long rb = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(a0 >> 32), 0) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a0, 0);
        const unsigned long long pb = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(a1 >> 32), 32) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a1, 32);
        const bool rec_ok = rb + nrec <= o.rec_cap, part_ok = pb + npart <= o.part_cap;
        if (lane == 0 && !rec_ok) atomicOr(o.status, ST_REC_FULL);
        if (lane == 0 && !part_ok) atomicOr(o.status, ST_PART_FULL);
        if (d < ng) {
            uint64_t fb = ~0ull;   /* first record of document d, ~0 when its stream overflowed */
            if (st == 2) {
                fb = rec_ok ? rb + (off & 0xFFFFu) : ~0ull;
                o.doc_recoff[gd0 + d] = rb + (off & 0xFFFFu);
                o.doc_npairs[gd0 + d] = cnt;
            } else if (st == 1) {
                fb = part_ok ? pb + (off >> 16) : ~0ull;
            }
            S.fbase[d] = fb;
            S.f.dstate[d] = st;
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
                if (S.f.dstate[rel] == 2) { o.rec_slot[qq] = key & smask; o.rec_cnt[qq] = ec[j]; }
                else { o.part_doc[qq] = gd0 + rel; o.part_slot[qq] = key & smask; o.part_cnt[qq] = ec[j]; }
            }
            tbl_clear(S, j * NT + tid);
        }
    }
}

/* v_perm selector dword k of a term of length n: byte j of the key dword is data byte j
 * (4k + j < n), TAB (4k + j == n: byte 0 of the 0x09090909 source) or zero */
__device__ __forceinline__ uint32_t perm_sel(uint32_t n, uint32_t k) {
    uint32_t s = 0;
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t p = 4 * k + j;
        const uint32_t b = p < n ? j : (p == n ? 4u : 12u);
        s |= b << (8 * j);
    }
    return s;
}

}  // namespace

__global__ __launch_bounds__(NT, WG_PER_CU) void k_tokcount_st(CorpusDev c, const uint64_t* __restrict__ chunk_start,
                                                       const uint32_t* __restrict__ chunk_doc, uint64_t c0,
                                                       uint64_t c1, VocabDev v, K1Out o, uint32_t sb, uint32_t gcap) {
    __shared__ __attribute__((aligned(16))) StShared S;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t last_blk = c.nbytes ? ((c.nbytes - 1) & ~(uint64_t)15) : 0;

    for (int j = 0; j < EPT; ++j) tbl_clear(S, j * NT + tid);
    if (tid < 64) {
        const uint32_t n = (uint32_t)tid >> 2, k = (uint32_t)tid & 3u;
        (&S.sel[n].x)[k] = perm_sel(n, k);
    }
    unsigned long long tokens_wg = 0;
#ifdef K1_STAMPS
    uint64_t st_acc[K1S_NPH + 1] = {}, st_prev = 0;
    uint32_t st_ph = 0;
#endif

    /* one token round of the wave (one token per lane) */
    struct Round {
        uint64_t ap;
        uint32_t k0, k1, k2, k3;   /* identity key (short terms) */
        uint32_t hv, rel, kind;
        uint4 s4, t4;              /* the two vocabulary slots loaded for it */
    };
    Round pend{};
    bool pending = false;
    uint32_t gd0_cur = 0;
    /* resolve a round: vocabulary slot (miss path: lock-free insert / long term) and
     * docSize; returns the LDS table key (0: no token) */
    auto resolve = [&](const Round& r) -> uint32_t {
        uint32_t slot = INVALID_SLOT;
        if (r.kind == 1u) {
            const bool hit0 = r.s4.x == r.k0 && r.s4.y == r.k1 && r.s4.z == r.k2 && r.s4.w == r.k3;
            const bool hit1 = r.t4.x == r.k0 && r.t4.y == r.k1 && r.t4.z == r.k2 && r.t4.w == r.k3;
            slot = hit0 ? r.hv : hit1 ? ((r.hv + 1) & (uint32_t)v.mask)
                                      : vocab_insert(v, ((uint64_t)r.k1 << 32) | r.k0, ((uint64_t)r.k3 << 32) | r.k2, 0,
                                                     o.status);
        } else if (r.kind == 2u) {
            slot = slow_slot(c.bytes, v, r.ap, S.gdoc[r.rel + 1], o.status);
        }
        /* docSize: one LDS add per wave when the round's tokens share a document */
        const uint64_t vm = __ballot(r.kind != 0u);
        if (vm) {
            const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.rel);
            if (__ballot(r.kind != 0u && r.rel != r0) == 0ull) {
                if (lane == 0) atomicAdd(&S.dsz[r0], (uint32_t)__popcll(vm));
            } else if (r.kind) {
                atomicAdd(&S.dsz[r.rel], 1u);
            }
        }
        return slot == INVALID_SLOT ? 0u : (0x80000000u | (r.rel << sb) | slot);
    };
    /* The LDS count of a round: ONE ds_read_b128 of the key's home bucket; a match is
     * counted with a non-returning add, a new key claims a free slot of the bucket with one
     * CAS (then adds); the rare rest (full bucket, a lost race, overflow mode) takes
     * bkt_slow.  (A linear-probing table of u64 entries, CAS first, took the same time at
     * about twice the instructions.) */
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
            if (slow) claims = bkt_slow(S, o, key, b, over, gd0_cur, sb);
        }
        const uint32_t wc = (uint32_t)__popcll(__ballot(claims != 0u));
        if (wc && lane == 0) {
            /* no return value: later rounds read fill (claims of up to 4 waves x 64 lanes in
             * flight fit the table's margin above FILL_LIMIT) */
            (void)atomicAdd(&S.fill, wc);
        }
    };
    auto finish = [&](const Round& r) { count(resolve(r)); };
    auto drain = [&]() {
        if (pending) { finish(pend); pending = false; }
    };

    /* Chunks come from sharded counters (claim_chunk), claimed two ahead, so the next chunk is known to
     * every wave while this one runs.  What a chunk needs before its first token — its
     * bounds, its documents' offsets and the first step of corpus bytes — is fetched during
     * the previous chunk: the bounds at its start (scalar loads), the offsets before its
     * flush (one u64 per thread), and each wave's last step prefetch of the chunk is aimed at
     * the next chunk's first step instead of past the end.  A chunk then starts without a
     * dependent HBM round trip. */
    uint32_t shard = blockIdx.x & 7u;   /* thread 0's current counter shard */
    if (tid == 0) {
        S.cur_chunk = claim_chunk(o.chunk_shard, shard, c0, c1 - c0);
        S.nxt_chunk = claim_chunk(o.chunk_shard, shard, c0, c1 - c0);
    }
    lds_barrier();
    uint64_t claim = 0;
    uint8_t* const stage = reinterpret_cast<uint8_t*>(&S.w.stage[wid][0]);
    uint32_t* const tl = S.w.tl[wid];
    const uint64_t lane_off = 16ull * lane;
    uint4 pf0 = make_uint4(0, 0, 0, 0);             /* the wave's next step of corpus bytes */
    uint64_t pfb = ~0ull;                           /* step base pf0 holds step `wid` of, if any */
    uint64_t dpre = 0;                              /* doc_off[dfirst + tid] of this chunk ... */
    bool dpre_ok = false;                           /* ... when fetched during the previous one */
    unsigned long long pend_v = 0;                  /* thread 0: the claim issued at chunk start */
    uint64_t chunk = uni64(S.cur_chunk), nxt = uni64(S.nxt_chunk);
    uint64_t cs = 0, ce = 0;
    uint32_t dfirst = 0, dlast = 0;
    if (chunk < c1) {
        cs = chunk_start[chunk];
        ce = chunk_start[chunk + 1];
        dfirst = chunk_doc[chunk];
        dlast = chunk_doc[chunk + 1];
    }
    const uint64_t nchunk = c1 - c0;
    while (chunk < c1) {
        STP(0);
#ifdef K1_STAMPS
        if (lane == 0) st_acc[K1S_NPH] += 1;
#endif
        /* the claim is issued now and its value used at the chunk end (no wait here) */
        if (tid == 0) pend_v = atomicAdd(&o.chunk_shard[shard], 1ull);
        uint64_t ncs = 0, nce = 0;
        uint32_t ndf = 0, ndl = 0;
        if (nxt < c1) {
            ncs = chunk_start[nxt];
            nce = chunk_start[nxt + 1];
            ndf = chunk_doc[nxt];
            ndl = chunk_doc[nxt + 1];
        }
        if (cs < ce)
        for (uint32_t gd0 = dfirst; gd0 <= dlast; gd0 += gcap) {
            gd0_cur = gd0;
            const uint32_t ng = (dlast + 1 - gd0) < gcap ? (dlast + 1 - gd0) : gcap;
            if (gd0 == dfirst && dpre_ok) {
                if ((uint32_t)tid <= ng) S.gdoc[tid] = dpre;
                if (tid == 0 && ng >= (uint32_t)NT) S.gdoc[NT] = c.doc_off[gd0 + NT];
            } else {
                for (uint32_t k = tid; k <= ng; k += NT) S.gdoc[k] = c.doc_off[gd0 + k];
            }
            dpre_ok = false;
            if (tid < GCAP) { S.dsz[tid] = 0; S.dpart[tid] = 0; }
            if (tid == 0) S.fill = 0;
            lds_barrier();
            STP(1);
            const bool last_group = gd0 + gcap > dlast;
            const bool ahead = last_group && nxt < c1 && ncs < nce;   /* prefetch for the next chunk */
            const uint64_t nb0 = ncs & ~(uint64_t)15;
            const uint64_t g0 = uni64(S.gdoc[0]), gn = uni64(S.gdoc[ng]);
            const uint64_t gs = g0 > cs ? g0 : cs;
            const uint64_t ge = gn < ce ? gn : ce;
            if (gs < ge) {
                const uint64_t b0 = gs & ~(uint64_t)15;
                const uint32_t nsteps = (uint32_t)((ge - b0 + WSTEP - 1) / WSTEP);
                if (b0 != pfb) pf0 = ld16c(c.bytes, last_blk, b0 + (uint64_t)wid * WSTEP + lane_off - 16ull);
                pfb = ~0ull;
                uint32_t wr = 0;             /* wave-uniform: document containing the step start */
                uint64_t wcur = g0, wnext = ng > 1 ? uni64(S.gdoc[1]) : gn;   /* gdoc[wr], gdoc[wr + 1] */
                for (uint32_t s = wid; s < nsteps; s += NWAVE) {
                    const uint64_t sb = b0 + (uint64_t)s * WSTEP;     /* first owned byte */
                    const uint64_t gpos = sb + lane_off - 16ull;      /* this lane's group */
                    const uint4 cur = pf0;
                    {
                        /* the wave's next step, or after its last one the next chunk's first */
                        const bool redirect = ahead && s + NWAVE >= nsteps;
                        const uint64_t a1 = redirect ? nb0 + (uint64_t)wid * WSTEP + lane_off - 16ull
                                                     : gpos + 1ull * NWAVE * WSTEP; /* harmless past ge */
                        if (redirect) pfb = nb0;
                        pf0 = ld16c(c.bytes, last_blk, a1);
                    }
                    /* the step's 64 groups into the wave's stage; this wave's reads of the
                     * previous step were issued before (LDS in order) */
                    reinterpret_cast<uint4*>(stage)[lane] = cur;
                    /* ---- classify (bytes outside the shard read as whitespace) ---- */
                    const bool inner = sb >= c.lo + 16 && sb + WSTEP + 16 <= c.hi;
                    uint32_t ws = ws_mask16_swar(cur);
                    if (!inner) ws |= bounds_ws(gpos, c.lo, c.hi);
                    /* document starts in the window [sb - 16, sb + WSTEP + 16) and the
                     * document of each lane's first byte.  Most steps hold no document start
                     * (wnext past the window): no loop then */
                    while (wr + 1 < ng && wnext <= sb) {
                        ++wr;
                        wcur = wnext;
                        wnext = uni64(S.gdoc[wr + 1]);
                    }
                    uint32_t ds = 0, base = wr;
                    if (wnext < sb + WSTEP + 16 || wcur + 16 >= sb) {
                        for (uint32_t k = wr; k <= ng; ++k) {   /* k = wr: a start AT sb is a start too */
                            const uint64_t sk = uni64(S.gdoc[k]);
                            if (sk >= sb + WSTEP + 16) break;
                            base += (k > wr && sk < gpos) ? 1u : 0u;
                            if (sk >= gpos && sk < gpos + 16) ds |= 1u << (uint32_t)(sk - gpos);
                        }
                    }
                    const uint32_t prev = (lane_prev(ws) >> 15) & 1u;
                    uint32_t own = (lane >= 1 && lane <= 62) ? 0xFFFFu : 0u;
                    if (!(sb >= gs && sb + WSTEP <= ge) && own) {
                        own = 0;
                        if (gpos + 16 > gs && gpos < ge) {
                            const uint32_t a = gpos < gs ? (uint32_t)(gs - gpos) : 0u;
                            const uint32_t b = gpos + 16 > ge ? (uint32_t)(ge - gpos) : 16u;
                            own = ((1u << b) - 1u) & ~((1u << a) - 1u);
                        }
                    }
                    const uint32_t starts = ~ws & ((ws << 1) | prev | ds) & own & 0xFFFFu;
                    /* NUL bytes end a term (strcmp), not a token: rare, exact masks only
                     * when the wave holds one */
                    uint32_t nul = 0;
                    if (__ballot((zero_bits(cur.x) | zero_bits(cur.y) | zero_bits(cur.z) | zero_bits(cur.w)) != 0u) != 0ull)
                        nul = compress4(zero_bits(cur.x)) | (compress4(zero_bits(cur.y)) << 4) |
                              (compress4(zero_bits(cur.z)) << 8) | (compress4(zero_bits(cur.w)) << 12);
                    const uint32_t stop = ws | ds;
                    /* term end = the first stop after the start byte or the first NUL from
                     * the start byte on (a NUL start gives the empty term); the next lane's
                     * masks extend the window to 32 bytes */
                    const uint32_t stop32 = stop | (lane_next(stop) << 16), nul32 = nul | (lane_next(nul) << 16);
                    /* ---- token entries (wave prefix sum over the lanes' start counts) ---- */
                    const uint32_t nmine = (uint32_t)__popc(starts);
                    const uint32_t incl = wave_incl_scan(nmine);
                    const uint32_t ntok = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                    if (ntok == 0) continue;
                    tokens_wg += ntok;
                    for (uint32_t tb = 0; tb < ntok; tb += TLW) {
                        {
                            uint32_t sm = starts, idx = incl - nmine;
                            while (sm) {
                                const uint32_t i = __builtin_ctz(sm);
                                sm &= sm - 1;
                                if (idx - tb < (uint32_t)TLW) {
                                    const uint32_t e = ((stop32 >> i) & ~1u) | (nul32 >> i);
                                    const uint32_t len = e ? (uint32_t)__builtin_ctz(e) : LEN_LONG;
                                    /* the document of byte i: the lane's first-byte document,
                                     * advanced past every start <= i (empty documents share
                                     * a start, so walk doc_off instead of counting bits) */
                                    uint32_t rel = base;
                                    if (ds & ((2u << i) - 1u))
                                        while (rel + 1 < ng && S.gdoc[rel + 1] <= gpos + i) ++rel;
                                    tl[idx - tb] = ((uint32_t)lane << 4 | i) | ((len < 16u ? len : LEN_LONG) << 10) |
                                                   (rel << 16);   /* offset in the stage */
                                }
                                ++idx;
                            }
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        const uint32_t cnt = (ntok - tb) < (uint32_t)TLW ? (ntok - tb) : (uint32_t)TLW;
                        STP(2);
                        /* ---- rounds of 64 tokens; the vocabulary loads of round r+1 are
                         * issued before round r is counted ---- */
                        for (uint32_t t0 = 0; t0 < cnt; t0 += 64) {
                            Round q;
                            const uint32_t t = t0 + lane;
                            const bool val = t < cnt;
                            const uint32_t e = val ? tl[t] : 0u;
                            const uint32_t pos = e & 1023u, len = (e >> 10) & 31u;
                            q.rel = e >> 16;
                            q.ap = sb - 16ull + pos;
                            q.kind = val ? (len == LEN_LONG ? 2u : 1u) : 0u;
                            const u32x4u raw = *reinterpret_cast<const u32x4u*>(stage + pos);
                            const uint4 sl = S.sel[len & 15u];
                            q.k0 = __builtin_amdgcn_perm(0x09090909u, raw.x, sl.x);
                            q.k1 = __builtin_amdgcn_perm(0x09090909u, raw.y, sl.y);
                            q.k2 = __builtin_amdgcn_perm(0x09090909u, raw.z, sl.z);
                            q.k3 = __builtin_amdgcn_perm(0x09090909u, raw.w, sl.w);
                            q.hv = q.kind == 1u ? (uint32_t)(key_hash(((uint64_t)q.k1 << 32) | q.k0,
                                                                      ((uint64_t)q.k3 << 32) | q.k2) & v.mask & ~1ull)
                                                : 0u;   /* even home slot (dev_vocab.h) */
                            /* the home slot and the next one: a key displaced by one slot
                             * (linear probing) resolves without a dependent load */
                            q.s4 = gload(v.keys + q.hv);
                            q.t4 = gload(v.keys + ((q.hv + 1) & (uint32_t)v.mask));
                            if (pending) finish(pend);
                            pend = q;
                            pending = true;
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        STP(1);
                    }
                }
            }
            STP(3);
            drain();
            STP(4);
            if (ahead) {   /* the next chunk's document offsets, in flight during this flush */
                const uint32_t nng = (ndl + 1 - ndf) < gcap ? (ndl + 1 - ndf) : gcap;
                dpre = (uint32_t)tid <= nng ? c.doc_off[ndf + tid] : 0ull;
                dpre_ok = true;
            }
            /* group end is a document boundary (or the chunk end): emit everything */
#ifdef K1_STAMPS
            lds_barrier();
#endif
            STP(5);
            if (ng <= FEW) st_flush_few(S, o, gd0, ng, cs, ce, sb);
            else st_flush(S, o, gd0, ng, cs, ce, sb);
            STP(6);
            if ((uint32_t)tid < ng) {
                const uint32_t n = S.dsz[tid];
                if (n) {
                    const uint32_t d = gd0 + tid;
                    if (S.gdoc[tid] >= cs && S.gdoc[tid + 1] <= ce) o.doc_size[d] = n;
                    else atomicAdd(&o.doc_size[d], n);
                }
            }
            lds_barrier();
            if (gd0 + gcap < gd0) break; /* overflow guard */
        }
        if (tid == 0) {
            const uint64_t lo = nchunk * shard / 8, hi = nchunk * (shard + 1) / 8;
            claim = lo + pend_v < hi ? c0 + lo + pend_v : claim_chunk(o.chunk_shard, shard, c0, nchunk);
            S.cur_chunk = nxt;
            S.nxt_chunk = claim;
        }
        lds_barrier();
        chunk = nxt;
        nxt = uni64(S.nxt_chunk);
        cs = ncs;
        ce = nce;
        dfirst = ndf;
        dlast = ndl;
    }
    if (lane == 0 && tokens_wg) atomicAdd(o.ntokens, tokens_wg);
#ifdef K1_STAMPS
    STP(0);
    if (lane == 0 && o.stamps)
        for (int k = 0; k <= K1S_NPH; ++k) atomicAdd(&o.stamps[k], (unsigned long long)st_acc[k]);
    if (lane == 0 && o.stamps) atomicAdd(&o.stamps[K1S_NPH + 1], 1ull);
#endif
}

int launch_tokcount_st(const CorpusDev& c, const uint64_t* chunk_start, const uint32_t* chunk_doc, uint64_t c0,
                       uint64_t c1, const VocabDev& v, const K1Out& o, hipStream_t s) {
    if (c1 <= c0) return 0;
    if (v.mask >= (1ull << SLOT_BITS)) return -3; /* slot must fit the LDS entry */
    static_assert(sizeof(StShared) * WG_PER_CU <= 163840, "LDS of WG_PER_CU workgroups per CU");
    static_assert(TB % NT == 0 && TB % BW == 0, "table rows");
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const uint64_t wgs = (uint64_t)ncu * WG_PER_CU;
    const uint64_t grid = (c1 - c0) < wgs ? (c1 - c0) : wgs;
    /* key32 = 1 << 31 | doc-in-group << sb | slot: the group size follows the slot bits */
    const uint32_t sb = (uint32_t)__builtin_popcountll(v.mask);
    const uint32_t gcap = (1u << (31u - sb)) >= (uint32_t)GCAP ? (uint32_t)GCAP : (1u << (31u - sb));
    k_tokcount_st<<<(unsigned)grid, NT, 0, s>>>(c, chunk_start, chunk_doc, c0, c1, v, o, sb, gcap);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
