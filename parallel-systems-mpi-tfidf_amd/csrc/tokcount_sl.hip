/*
 * tokcount_sl.hip — K1: fused tokenize + per-document term counting, persistent
 * workgroups claiming chunks, straight-line token rounds.  Replaces the reference's per-rank hot loop
 * TFIDF.c:130-196: the two fscanf("%s") passes (:141-147), the O(P) strcmp search/append
 * of (word, doc) records (:151-167) and the per-rank word table (:169-188).
 *
 * The kernel is written for instruction issue, which is what bounds this stage on gfx950
 * (the LDS-staged kernel it replaces issued ~480 VALU + ~210 SALU
 * wave-instructions per 64 tokens, a third of them spill and exec-mask traffic):
 *   - four workgroups per CU stay resident and claim K0 chunks from a global counter, the
 *     next claim sent when a chunk starts (chunk sizes vary: one workgroup per chunk
 *     measured 2.90 ms on c2 for the per-workgroup set-up, a static share 2.46 for its tail,
 *     the claim loop 1.94-1.97; profiles/r04_k1_ab_c2.txt);
 *   - corpus and vocabulary reads are buffer loads with 32-bit offsets from a per-chunk
 *     (corpus) or per-launch (vocabulary) resource: out-of-range lanes read zero instead of
 *     being clamped, and a probe's two slots are one address with offsets 0 and 16;
 *   - every position is a signed 32-bit offset from the chunk base b0 = chunk_start & ~15;
 *   - the vocabulary pair: terms are inserted from an even home slot (dev_vocab.h), so the
 *     two slots a round loads never wrap;
 *   - a round is a straight line for the common case (both vocabulary slots compared, the
 *     LDS bucket read, one CAS and one add per lane whatever the outcome: branching on the
 *     outcome measured 0.16 ms slower on c2); a claim lost to another lane of the same
 *     round (1.4 per round on c2: 64 lanes over 448 buckets) retries inline at the next
 *     slots, and a full home bucket is probed once more inline at the next bucket (c2 K1
 *     1.96 -> 1.76 ms: the out-of-line call had run in 69 % of the rounds); the rest
 *     (vocabulary miss, a term of 16 bytes or more, overflow mode, 6 % of the rounds) runs
 *     in out-of-line functions behind one wave-uniform test each;
 *   - docSize is counted per step in the walk (one scalar LDS add when the step lies in one
 *     document), the LDS table's fill per wave in a scalar register.
 *
 * Work inside a chunk: the four waves run without block barriers, wave w taking the
 * 992-byte step w first and then the next unclaimed one from an LDS counter (a static
 * w, w+4, ... share left the other waves waiting at the flush for the slowest); each lane classifies 16 bytes (SWAR C-locale isspace,
 * TFIDF.c:142,147, and NUL: strcmp stops there, :152,172), the lane owning a token start
 * writes a 32-bit token entry (stage offset | term length | document in group), and the
 * wave resolves its entries in rounds of 64 (one token per lane): one unaligned
 * ds_read_b128 of the term bytes + four v_perm build the 128-bit identity key (dev_common.h),
 * a multiply hash picks the vocabulary pair, and the (document, slot) pair is counted in an
 * LDS table of 8-slot buckets.  The next round's vocabulary loads are in flight while a
 * round is counted.  At the group end the table is flushed as coalesced records (complete
 * documents) or partial records (documents split across chunks, merged by finalize.hip).
 *
 * LDS: 28 KiB table + ~10 KiB walk/document state -> four workgroups (16 waves) per CU.
 * Requires a 16-byte aligned corpus base and a vocabulary of <= 2^22 slots.
 */
#include "dev_common.h"
#include "dev_vocab.h"
#include "kernels.h"

/* timing ablations (diagnostic builds only, wrong output by design): every record write of
 * K1 is suppressed so the stages after it see an empty, consistent record set */
#if defined(SL_ABL_NOVOCAB) || defined(SL_ABL_NOCOUNT) || defined(SL_ABL_NOROUNDS) || defined(SL_ABL_NOWRITE) || \
    defined(SL_ABL_NOALLOC) || defined(SL_ABL_L2C)
#define SL_ABL 1
#else
#define SL_ABL 0
#endif
/* SL_ABL_NOALLOC: the records are stored, all at the start of the arrays (no allocation
 * atomics); the stage after K1 still sees an empty record set */
#ifdef SL_ABL_NOALLOC
#define SL_ABL_ST 0
#else
#define SL_ABL_ST SL_ABL
#endif

namespace {

#ifndef SL_NT
#define SL_NT 256
#endif
constexpr int NT = SL_NT;               /* threads per workgroup (SL_NT=320: five waves, A/B) */
constexpr int NWAVE = NT / 64;
#ifndef SL_WGCU
#define SL_WGCU 4
#endif
constexpr int WG_PER_CU = SL_WGCU;      /* 16 waves per CU */
constexpr int WSTEP = 992;              /* bytes a wave step owns: lanes 1..62 one 16-byte group each;
                                           lane 0 holds the 16 bytes before the step, lane 63 the 16
                                           after it (terms crossing the step end) */
#ifndef SL_TB
#define SL_TB 3584
#endif
constexpr int TB = SL_TB;               /* LDS count table entries (u32 key + u32 count) */
constexpr int EPT = TB / NT;
constexpr uint32_t BW = 8;              /* slots per bucket (two ds_read_b128) */
constexpr uint32_t NB = TB / BW;
constexpr uint32_t WAVE_CLAIMS = (TB - 2 * NT - 64) / NWAVE;   /* claims per wave before overflow mode */
constexpr int GCAP = 256;               /* documents per group at most */
constexpr int TLW = 192;                /* token entries per wave and pass */
constexpr uint32_t LEN_LONG = 31u;
constexpr uint32_t SLOT_BITS = 25;      /* vocabulary slots < 2^25 (K1_SL_MAX_CAP; the LDS key's document
                                           field shrinks as the slot field grows: gcap below) */
constexpr int PMAX = 16;
#ifdef SL_STAMPS
constexpr int SL_NPH = 12;              /* diagnostic phases (SL_STAMPS) */
#endif                /* LDS buckets probed before a key becomes a partial record */

struct SlShared {
    uint32_t TK[TB];                    /* key32 = 1 << 31 | doc-in-group << sb | slot (0: empty) */
    uint32_t TC[TB];                    /* its count */
    int32_t gdoc[GCAP + 1];             /* document starts of the group, relative to b0 (clamped) */
    uint32_t dsz[GCAP];                 /* docSize accumulators */
    union {
        struct {
            uint4 stage[NWAVE][64];     /* a wave's step: [sb - 16, sb + 1008) */
            uint32_t tl[NWAVE][TLW];    /* token entries */
        } w;
        struct {
            uint32_t dcnt[GCAP];
            uint32_t doff[GCAP];
            uint32_t drun[GCAP];
            uint8_t dstate[GCAP];
        } f;
        struct {
            uint32_t wtot[NWAVE * 4];   /* few-document flush: each wave's per-document entry counts */
            uint4 lrank[NT];            /* ... each thread's first staging index per document (16-bit) */
        } q;
    };
    uint4 sel[16];                      /* v_perm selectors of a term of length n */
    uint32_t lbase[8];                  /* few-document flush: a document's first staging index */
    uint32_t fl_nrec, fl_npart;         /* flush: records and partial records of the group */
    uint8_t dpart[GCAP];                /* document has overflow records */
    uint8_t dfull[GCAP];                /* document lies wholly inside the chunk */
    uint32_t wsum[NWAVE];
    unsigned long long rec_base, part_base;
    unsigned long long next_chunk;      /* persistent form: the workgroup's next chunk (claimed ahead) */
    uint32_t step_next;                 /* the group's next unclaimed step */
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));

#define RSRC_WORD3 0x00020000   /* gfx9 raw buffer: 32-bit data format, no swizzle */

template <int AUX> __device__ __forceinline__ uint4 bload16(__amdgpu_buffer_rsrc_t r, int32_t off) {
    const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
    return make_uint4(v.x, v.y, v.z, v.w);
}

/* bit 7 of every zero byte (exact) */
__device__ __forceinline__ uint32_t zero_bits(uint32_t x) { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u; }
__device__ __forceinline__ uint32_t compress4(uint32_t m) {
    m >>= 7;
    m |= m >> 7;
    m |= m >> 14;
    return m & 0xFu;
}

/* C-locale isspace() of 16 bytes (TFIDF.c:142,147: the bytes fscanf("%s") stops at,
 * {0x20, 0x09..0x0D}) as a 16-bit mask, bit i = byte i, and whether any byte is below 0x09
 * (NUL or 0x01..0x08: the caller then looks for NUL bytes, which end a term).  Per dword
 * seven SWAR ops leave a flag in bit 7 of each whitespace byte (every per-byte sum stays
 * inside its byte, so the tests are exact); the four dwords' flags are gathered into the
 * mask by v_dot4_u32_u8 with the weights of each byte position (one instruction per dword
 * instead of a shift/or cascade). */
__device__ __forceinline__ uint32_t ws_flags4(uint32_t x, uint32_t& lt9) {
    const uint32_t y = x & 0x7F7F7F7Fu;
    const uint32_t a = y + 0x77777777u;                         /* bit 7: low7 >= 0x09 */
    const uint32_t b = y + 0x72727272u;                         /* bit 7: low7 >= 0x0E */
    const uint32_t c = (y ^ 0x20202020u) + 0x7F7F7F7Fu;         /* bit 7: low7 != 0x20 */
    lt9 |= ~(a | x) & 0x80808080u;                              /* bytes < 0x09 */
    return ((a & ~b) | ~c) & ~x & 0x80808080u;
}
__device__ __forceinline__ uint32_t ws_mask16_dot(uint4 v, uint32_t& lt9) {
    const uint32_t f0 = ws_flags4(v.x, lt9), f1 = ws_flags4(v.y, lt9);
    const uint32_t f2 = ws_flags4(v.z, lt9), f3 = ws_flags4(v.w, lt9);
    /* flag bytes are 0x80 or 0: sum of 0x80 * weight, weights 1,2,4,8 | 16,32,64,128 */
    const uint32_t lo = __builtin_amdgcn_udot4(f0, 0x08040201u, __builtin_amdgcn_udot4(f1, 0x80402010u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(f2, 0x08040201u, __builtin_amdgcn_udot4(f3, 0x80402010u, 0u, false), false);
    return (lo + (hi << 8)) >> 7;
}

/* bytes of [pos, pos+16) outside [lo, hi) (chunk-relative) */
__device__ __forceinline__ uint32_t outside16(int32_t pos, int32_t lo, int32_t hi) {
    const int32_t a = lo - pos, b = hi - pos;
    const uint32_t am = a <= 0 ? 0u : (a >= 16 ? 0xFFFFu : ((1u << a) - 1u));
    const uint32_t bm = b <= 0 ? 0u : (b >= 16 ? 0xFFFFu : ((1u << b) - 1u));
    return ~(bm & ~am) & 0xFFFFu;
}

__device__ __forceinline__ uint32_t bkt_hash(uint32_t key) {
    return __umulhi(key * 0x9E3779B1u, NB);   /* [0, NB) */
}
struct BktK {
    uint4 a, b;
};
__device__ __forceinline__ uint32_t bkt_slot(uint32_t b, uint32_t j) { return BW * b + j; }
__device__ __forceinline__ BktK bkt_read(const uint32_t* TK, uint32_t b) {
    const uint4* t = reinterpret_cast<const uint4*>(TK) + 2 * b;
    BktK k;
    k.a = t[0];
    k.b = t[1];
    return k;
}
__device__ __forceinline__ uint32_t bkt_match(const BktK& kk, uint32_t key) {
    uint32_t j = kk.a.x == key ? 0u : kk.a.y == key ? 1u : kk.a.z == key ? 2u : kk.a.w == key ? 3u : 8u;
    if (j == 8u) j = kk.b.x == key ? 4u : kk.b.y == key ? 5u : kk.b.z == key ? 6u : kk.b.w == key ? 7u : 8u;
    return j;
}
/* A claim starts at a slot derived from the key and takes the first empty slot from there
 * on, cyclically in the bucket, so different keys of one round rarely aim at the same slot
 * (round 4's claims all took the bucket's first empty slot: 1.52 lost claims per round, 70 %
 * of rounds retried; this form: c2 K1 1.72 -> 1.65 ms, profiles/r05_k1_ab_c2.txt).  Every claimer
 * of a key walks the same cyclic order from the same start and slots are never emptied
 * during a group, so a key is never claimed twice: a walker meets the key's slot (its CAS
 * returns the key) before any slot that was empty when the key was placed.  Occupancy from
 * the keys' top bits (every key has bit 31 set): the top bytes of four slots gathered by two
 * v_perm, their bit 7 moved to one bit each. */
__device__ __forceinline__ uint32_t bkt_occ(const BktK& kk) {   /* bit i: slot i holds a key */
    const uint32_t ta = __builtin_amdgcn_perm(kk.a.y, kk.a.x, 0x0C0C0703u) | __builtin_amdgcn_perm(kk.a.w, kk.a.z, 0x07030C0Cu);
    const uint32_t tb = __builtin_amdgcn_perm(kk.b.y, kk.b.x, 0x0C0C0703u) | __builtin_amdgcn_perm(kk.b.w, kk.b.z, 0x07030C0Cu);
    /* bit 7 of each byte, weighted 1..128 by two v_dot4_u32_u8 */
    return __builtin_amdgcn_udot4(ta & 0x80808080u, 0x08040201u,
                                  __builtin_amdgcn_udot4(tb & 0x80808080u, 0x80402010u, 0u, false), false) >> 7;
}
__device__ __forceinline__ uint32_t bkt_pref(uint32_t key) { return (key * 0x85EBCA77u) >> 29; }
/* the first slot at or after p (cyclically) that `occ` marks empty; BW when none */
__device__ __forceinline__ uint32_t bkt_pick(uint32_t occ, uint32_t p) {
    const uint32_t e = ~occ & 0xFFu;
    const uint32_t r = ((e | (e << 8)) >> p) & 0xFFu;
    return r ? ((p + (uint32_t)__builtin_ctz(r)) & (BW - 1u)) : BW;
}

/* one partial record of count 1 (overflow mode / no room): one device atomic per wave */
__device__ __noinline__ void overflow_record(const K1Out* o, uint32_t doc, uint32_t slot) {
    const uint64_t am = __ballot(1);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
    unsigned long long b = 0;
    if (rank == 0u) b = gatomic_add(o->part_alloc, (unsigned long long)__popcll(am));
    const unsigned long long q = (((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
                                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b)) + rank;
    if (SL_ABL) return;
    if (q < o->part_cap) { gmem(o->part_doc)[q] = doc; gmem(o->part_slot)[q] = slot; gmem(o->part_cnt)[q] = 1u; }
    else atomicOr(o->status, ST_PART_FULL);
}

/* The rare LDS count cases: home bucket full without the key, a lost claim, or overflow
 * mode.  Counts `key` from bucket b on (re-reading each bucket); a key that is not in the
 * table in overflow mode, or after PMAX buckets, becomes a partial record of count 1.
 * Returns 1 when this call claimed a slot. */
__device__ __noinline__ uint32_t bkt_slow(uint32_t* TK, uint32_t* TC, uint8_t* dpart, const K1Out* o, uint32_t key,
                                          uint32_t b, bool over, uint32_t gd0, uint32_t sb) {
    for (int probe = 0, tries = 0; probe < PMAX && tries < 64; ++tries) {
        const BktK kk = bkt_read(TK, b);
        const uint32_t j = bkt_match(kk, key);
        if (j < BW) { atomicAdd(&TC[bkt_slot(b, j)], 1u); return 0u; }
        const uint32_t e = bkt_pick(bkt_occ(kk), bkt_pref(key));   /* the key's first empty slot */
        if (e < BW) {
            if (over) break;
            const uint32_t old = atomicCAS(&TK[bkt_slot(b, e)], 0u, key);
            if (old == 0u || old == key) {
                atomicAdd(&TC[bkt_slot(b, e)], 1u);
                return old == 0u ? 1u : 0u;
            }
            continue;
        }
        b = b + 1 == NB ? 0u : b + 1;
        ++probe;
    }
    const uint32_t rel = (key & 0x7FFFFFFFu) >> sb;
    dpart[rel] = 1;
    overflow_record(o, gd0 + rel, key & ((1u << sb) - 1u));
    return 0u;
}

/* The rare vocabulary cases of a round: a short term in neither slot of its home pair
 * (first occurrences, displaced keys: the lock-free insert of dev_vocab.h) or a term of 16
 * bytes or more / running past the 32-byte window (kind 2: re-read from HBM). */
__device__ __noinline__ uint32_t resolve_slow(const uint8_t* __restrict__ bytes, uint4* keys, uint64_t* reps,
                                              uint64_t mask, uint32_t* status, uint32_t kind, uint32_t k0,
                                              uint32_t k1, uint32_t k2, uint32_t k3, uint64_t p0, uint64_t dend) {
    if (kind == 1u)
        return vocab_insert_s(keys, reps, mask, ((uint64_t)k1 << 32) | k0, ((uint64_t)k3 << 32) | k2, 0, status);
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
        return vocab_insert_s(keys, reps, mask, klo, khi, 0, status);
    }
    make_long_key(bytes + p0, n, &klo, &khi);
    /* rep = (length << 40) | offset holds 24 length bits (TFIDF_E_CAPACITY beyond) */
    if (n >= 0xFFFFFFull) atomicOr(status, ST_TERM_LONG);
    const uint64_t rep = ((n < 0xFFFFFFull ? n : 0xFFFFFFull) << 40) | p0;
    return vocab_insert_s(keys, reps, mask, klo, khi, rep, status, bytes);
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

/* The flush's second half: every entry has been placed in the staging area (the table's own
 * TK/TC words: records [0, nrec), partial records [nrec, nrec + npart), key and count), so the
 * group's records leave as ONE contiguous run from rb and its partial records as one from pb
 * — consecutive lanes store consecutive words (round 4 stored each entry at its document's
 * base + rank from the lane that held it: scattered partial lines, 0.33 ms of c2's K1 for
 * 0.5 GB, profiles/r05_k1_ablations_c2.txt).  Then the whole table is cleared. */
__device__ __forceinline__ void sl_write_staged(SlShared& S, const K1Out* o, uint32_t gd0, uint32_t sb, uint32_t nrec,
                                                uint32_t npart, unsigned long long rb, unsigned long long pb,
                                                bool rec_ok, bool part_ok) {
    const int tid = threadIdx.x;
    uint32_t* const rec_slot = o->rec_slot;   /* read once (see sl_flush_few) */
    uint32_t* const rec_cnt = o->rec_cnt;
    uint32_t* const part_doc = o->part_doc;
    uint32_t* const part_slot = o->part_slot;
    uint32_t* const part_cnt = o->part_cnt;
    const uint32_t smask = (1u << sb) - 1u;
    lds_barrier();
    if (rec_ok && !SL_ABL_ST)
        for (uint32_t i = (uint32_t)tid; i < nrec; i += NT) {
            gmem(rec_slot)[rb + i] = S.TK[i] & smask;
            gmem(rec_cnt)[rb + i] = S.TC[i];
        }
    if (part_ok && !SL_ABL_ST)
        for (uint32_t i = (uint32_t)tid; i < npart; i += NT) {
            const uint32_t k = S.TK[nrec + i];
            gmem(part_doc)[pb + i] = gd0 + ((k & 0x7FFFFFFFu) >> sb);
            gmem(part_slot)[pb + i] = k & smask;
            gmem(part_cnt)[pb + i] = S.TC[nrec + i];
        }
    lds_barrier();
    uint4* t = reinterpret_cast<uint4*>(S.TK);
#pragma unroll
    for (int j = tid; j < 2 * TB / 4; j += NT) t[j] = make_uint4(0, 0, 0, 0);   /* TK and TC are adjacent */
}

/* Emits the group's table entries as records (complete documents: the record stream;
 * documents crossing the chunk, over K5's in-LDS sort size or with overflow records: the
 * partial stream) — any number of documents: per-document counts by wave-aggregated LDS
 * adds, a block scan, every entry written at its document's base + its rank. */
__device__ __forceinline__ void sl_flush(SlShared& S, const K1Out* o, uint32_t gd0, uint32_t ng, uint32_t sb) {
    const int tid = threadIdx.x;
    lds_barrier();
    if (tid < GCAP) { S.f.dcnt[tid] = 0; S.f.drun[tid] = 0; }
    lds_barrier();
    uint32_t ek[EPT], ec[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        ek[j] = S.TK[j * NT + tid];
        ec[j] = S.TC[j * NT + tid];
        if (ek[j]) wave_agg_add(&S.f.dcnt[0], (ek[j] & 0x7FFFFFFFu) >> sb);
    }
    lds_barrier();
    uint32_t packed = 0;
    if ((uint32_t)tid < ng) {
        uint8_t st = 0;
        const uint32_t cnt = S.f.dcnt[tid];
        const bool part = S.dpart[tid] != 0;
        if (cnt) {
            const bool complete = !part && S.dfull[tid] && cnt <= (uint32_t)K5_MAX_PAIRS;
            st = complete ? 2 : 1;
            packed = complete ? cnt : (cnt << 16);
        }
        if ((st == 1 || part) && !SL_ABL) gmem(o->doc_flags)[gd0 + tid] = DF_PARTIAL;
        S.f.dstate[tid] = st;
    }
    uint32_t tot;
    const uint32_t off = block_excl_scan<NT, true>(packed, S.wsum, &tot);
    if ((uint32_t)tid < ng) S.f.doff[tid] = off;
    const uint32_t nrec = tot & 0xFFFFu, npart = tot >> 16;
    if (tid == 0) {
        const unsigned long long rb = (nrec && !SL_ABL) ? gatomic_add(o->rec_alloc, (unsigned long long)nrec) : 0ull;
        if (rb + nrec > o->rec_cap) atomicOr(o->status, ST_REC_FULL);
        S.rec_base = rb;
    } else if (tid == 64) {
        const unsigned long long pb = (npart && !SL_ABL) ? gatomic_add(o->part_alloc, (unsigned long long)npart) : 0ull;
        if (pb + npart > o->part_cap) atomicOr(o->status, ST_PART_FULL);
        S.part_base = pb;
    }
    lds_barrier();
    const unsigned long long rb = S.rec_base, pb = S.part_base;
    const bool rec_ok = rb + nrec <= o->rec_cap, part_ok = pb + npart <= o->part_cap;
    if ((uint32_t)tid < ng && S.f.dstate[tid] == 2) {
        gmem(o->doc_recoff)[gd0 + tid] = rb + (off & 0xFFFFu);
        gmem(o->doc_npairs)[gd0 + tid] = SL_ABL ? 0u : S.f.dcnt[tid];
    }
    /* every entry to its staging index: its document's base in the record or partial run
     * + its rank among the document's entries (all entries are in registers: the table's
     * words are free) */
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const uint32_t key = ek[j];
        if (key) {
            const uint32_t rel = (key & 0x7FFFFFFFu) >> sb;
            const uint32_t k = wave_agg_add_rtn(&S.f.drun[0], rel);
            const uint32_t dof = S.f.doff[rel];
            const uint32_t loc = (S.f.dstate[rel] == 2 ? (dof & 0xFFFFu) : nrec + (dof >> 16)) + k;
            S.TK[loc] = key;
            S.TC[loc] = ec[j];
        }
    }
    sl_write_staged(S, o, gd0, sb, nrec, npart, rb, pb, rec_ok, part_ok);
}

/* The flush of a group of at most FEW documents (most chunks hold one or two): per-thread
 * 16-bit document counters and one block scan, no LDS atomics.  Same output as sl_flush. */
constexpr uint32_t FEW = 8;
#ifdef SL_STAMPS
#define SLF_STAMP(k)                                                        \
    do {                                                                    \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();         \
        st_acc[k] += t_ - st_t;                                             \
        st_t = t_;                                                          \
    } while (0)
#define SLF_ARGS , unsigned long long* st_acc, unsigned long long& st_t
#else
#define SLF_STAMP(k) do {} while (0)
#define SLF_ARGS
#endif
__device__ __forceinline__ void sl_flush_few(SlShared& S, const K1Out* o, uint32_t gd0, uint32_t ng, uint32_t sb SLF_ARGS) {
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    lds_barrier();
    uint32_t ek[EPT], ec[EPT];
    /* per document, this thread's entry count in a 4-bit field (EPT < 16): one shift-add per
     * entry (an empty entry, key 0, adds 0 to document 0's field) */
    uint32_t c4 = 0;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        ek[j] = S.TK[j * NT + tid];
        ec[j] = S.TC[j * NT + tid];
        c4 += (ek[j] >> 31) << (4u * ((ek[j] & 0x7FFFFFFFu) >> sb));
    }
    static_assert(EPT < 16 && FEW == 8, "4-bit per-document entry counts of eight documents");
    uint32_t pk[FEW / 2], inc[FEW / 2];
#pragma unroll
    for (uint32_t q = 0; q < FEW / 2; ++q) {
        pk[q] = ((c4 >> (8u * q)) & 15u) | (((c4 >> (8u * q + 4u)) & 15u) << 16);
        inc[q] = wave_incl_scan(pk[q]);
        if (lane == 63) S.q.wtot[w * (FEW / 2) + q] = inc[q];
    }
    SLF_STAMP(9);
    lds_barrier();
    uint32_t rank[FEW / 2], tot[FEW / 2];
#pragma unroll
    for (uint32_t q = 0; q < FEW / 2; ++q) {
        uint32_t base = 0, t = 0;
#pragma unroll
        for (int k = 0; k < NWAVE; ++k) {
            const uint32_t x = S.q.wtot[k * (FEW / 2) + q];
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
                const bool complete = !part && S.dfull[d] && cnt <= (uint32_t)K5_MAX_PAIRS;
                st = complete ? 2 : 1;
                packed = complete ? cnt : (cnt << 16);
            }
            if ((st == 1 || part) && !SL_ABL) gmem(o->doc_flags)[gd0 + d] = DF_PARTIAL;
        }
        const uint32_t incl = wave_incl_scan(packed);
        const uint32_t all = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t off = incl - packed;
        const uint32_t nrec = all & 0xFFFFu, npart = all >> 16;
        unsigned long long a0 = 0, a1 = 0;
        if (lane == 0 && nrec && !SL_ABL) a0 = gatomic_add(o->rec_alloc, (unsigned long long)nrec);
        if (lane == 32 && npart && !SL_ABL) a1 = gatomic_add(o->part_alloc, (unsigned long long)npart);
        const unsigned long long rb = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(a0 >> 32), 0) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a0, 0);
        const unsigned long long pb = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(a1 >> 32), 32) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a1, 32);
        const bool rec_ok = rb + nrec <= o->rec_cap, part_ok = pb + npart <= o->part_cap;
        if (lane == 0 && !rec_ok) atomicOr(o->status, ST_REC_FULL);
        if (lane == 0 && !part_ok) atomicOr(o->status, ST_PART_FULL);
        if (d < ng && st == 2) {
            gmem(o->doc_recoff)[gd0 + d] = rb + (off & 0xFFFFu);
            gmem(o->doc_npairs)[gd0 + d] = SL_ABL ? 0u : cnt;
        }
        if (d < FEW) S.lbase[d] = d >= ng ? 0u : (st == 2 ? (off & 0xFFFFu) : nrec + (off >> 16));   /* staging index */
        if (lane == 0) {
            S.fl_nrec = nrec;
            S.fl_npart = npart;
            S.rec_base = rec_ok ? rb : ~0ull;
            S.part_base = part_ok ? pb : ~0ull;
        }
    }
    lds_barrier();
    SLF_STAMP(10);
    /* every entry to its staging index (sl_write_staged): its document's base + the entries
     * of that document before it (earlier threads, then this thread's earlier entries).  The
     * thread's first index per document goes to LDS as eight 16-bit values (staging indices
     * < TB), so an entry reads its base instead of selecting it from registers */
    {
        const uint4 lb0 = *reinterpret_cast<const uint4*>(&S.lbase[0]);
        const uint4 lb1 = *reinterpret_cast<const uint4*>(&S.lbase[4]);
        S.q.lrank[tid] = make_uint4(rank[0] + (lb0.x | (lb0.y << 16)), rank[1] + (lb0.z | (lb0.w << 16)),
                                    rank[2] + (lb1.x | (lb1.y << 16)), rank[3] + (lb1.z | (lb1.w << 16)));
    }
    const uint16_t* const lr16 = reinterpret_cast<const uint16_t*>(&S.q.lrank[tid]);
    uint32_t run = 0;   /* 4-bit per-document counts of this thread's entries placed so far */
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const uint32_t key = ek[j];
        if (key) {
            const uint32_t rel4 = 4u * ((key & 0x7FFFFFFFu) >> sb);
            const uint32_t loc = (uint32_t)lr16[rel4 >> 2] + ((run >> rel4) & 15u);
            run += 1u << rel4;
            S.TK[loc] = key;
            S.TC[loc] = ec[j];
        }
    }
    const unsigned long long rb = S.rec_base, pb = S.part_base;
    sl_write_staged(S, o, gd0, sb, S.fl_nrec, S.fl_npart, rb, pb, rb != ~0ull, pb != ~0ull);
}

/* The LDS count of one round's keys (key32 = 1 << 31 | document in group << sb | vocabulary slot;
 * 0: no token). */
#ifdef SL_STAMPS
#define SL_STC , st_cnt
#define SL_STC_ARG , unsigned long long* st_cnt
#else
#define SL_STC
#define SL_STC_ARG
#endif
__device__ __forceinline__ void lds_count(SlShared& S, const K1Out* o, uint32_t key, uint32_t& wclaims, uint32_t gd0,
                                          uint32_t sb SL_STC_ARG) {
    /* The LDS count, straight-line: ONE bucket read (two ds_read_b128), then one CAS
     * and one add per lane whatever the case — a match CASes its own key over itself,
     * a new key claims a free slot (CAS from 0), every other lane CASes against a
     * value no slot holds (0x7FFFFFFF: keys carry bit 31) and adds 0 */
    const bool over = wclaims >= WAVE_CLAIMS;
    const uint32_t b = bkt_hash(key);
    const BktK kk = bkt_read(S.TK, b);
    /* the key's slot: at most one slot matches, so its index bits are ORs of the lane masks
     * (scalar ORs, three selects; seven selects before) */
    const bool m0 = kk.a.x == key, m1 = kk.a.y == key, m2 = kk.a.z == key, m3 = kk.a.w == key;
    const bool m4 = kk.b.x == key, m5 = kk.b.y == key, m6 = kk.b.z == key, m7 = kk.b.w == key;
    const uint32_t j = ((m1 | m3 | m5 | m7) ? 1u : 0u) | ((m2 | m3 | m6 | m7) ? 2u : 0u) | ((m4 | m5 | m6 | m7) ? 4u : 0u);
    const bool found = m0 | m1 | m2 | m3 | m4 | m5 | m6 | m7;
    const uint32_t pref = bkt_pref(key);
    uint32_t occ = bkt_occ(kk);
    const uint32_t n = bkt_pick(occ, pref);   /* the key's first empty slot (BW: full) */
    const bool hit = key != 0u && found;
    const bool claim = key != 0u && !found && n < BW && !over;
    const uint32_t idx = bkt_slot(b, found ? j : (n & (BW - 1u)));
    /* only a new key waits for an LDS round trip (its CAS); a match adds at once.  The slot
     * holds the key after the CAS exactly when the CAS returned the key (a match, or a peer
     * lane claimed it for the same key first) or returned 0 to a claim */
    const uint32_t old = atomicCAS(&S.TK[idx], hit ? key : (claim ? 0u : 0x7FFFFFFFu), key);
    const bool ok = key != 0u && (old == key || (claim && old == 0u));
    atomicAdd(&S.TC[idx], ok ? 1u : 0u);
    bool claimed = claim && old == 0u;
    bool slow = key != 0u && !ok;
#ifdef SL_STAMPS
    st_cnt[0] += __ballot(slow) != 0ull ? 1u : 0u;
    st_cnt[1] += (uint32_t)__popcll(__ballot(slow));
    st_cnt[2] += (uint32_t)__popcll(__ballot(claim && !ok));
    ++st_cnt[4];
#endif
    /* claims lost to other lanes (of this round: every lane read the bucket before any
     * claimed): inline claims of the key's next empty slots of the snapshot, without
     * re-reading the bucket (a lost CAS returns the slot's key: the same key counts
     * there) */
    uint32_t nn = n;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        if (claim && slow) {
            occ |= 1u << (nn & (BW - 1u));
            nn = bkt_pick(occ, pref);
        }
        const bool lost = claim && slow && nn < BW;
        if (__ballot(lost) == 0ull) break;
        if (lost) {
            const uint32_t i2 = bkt_slot(b, nn);
            const uint32_t o2 = atomicCAS(&S.TK[i2], 0u, key);
            if (o2 == 0u || o2 == key) {
                atomicAdd(&S.TC[i2], 1u);
                slow = false;
                claimed = o2 == 0u;
            }
        }
    }
    /* the home bucket full without the key: one inline probe of the next bucket (a
     * fresh read: match there, else claim its first empty slot) */
    {
        const bool full = slow && !claim && !over && key != 0u;
        if (__ballot(full) != 0ull) {
            if (full) {
                const uint32_t b2 = b + 1u == NB ? 0u : b + 1u;
                const BktK k2 = bkt_read(S.TK, b2);
                const uint32_t j2 = bkt_match(k2, key);
                uint32_t e2 = j2;
                bool ok2 = j2 < BW;
                if (!ok2) {
                    e2 = bkt_pick(bkt_occ(k2), pref);
                    if (e2 < BW) {
                        const uint32_t o2 = atomicCAS(&S.TK[bkt_slot(b2, e2)], 0u, key);
                        ok2 = o2 == 0u || o2 == key;
                        claimed = o2 == 0u;
                    }
                }
                if (ok2) {
                    atomicAdd(&S.TC[bkt_slot(b2, e2)], 1u);
                    slow = false;
                }
            }
        }
    }
#ifdef SL_STAMPS
    st_cnt[3] += __ballot(slow) != 0ull ? 1u : 0u;
    st_cnt[5] += (uint32_t)__popcll(__ballot(slow && claim));            /* lost every retry */
    st_cnt[6] += (uint32_t)__popcll(__ballot(slow && !claim && !over));  /* bucket full */
    st_cnt[7] += (uint32_t)__popcll(__ballot(slow && over));             /* overflow mode */
#endif
    uint32_t claims = claimed ? 1u : 0u;
    if (__ballot(slow) != 0ull) {
        if (slow) claims = bkt_slow(S.TK, S.TC, S.dpart, o, key, b, over, gd0, sb);
    }
    wclaims += (uint32_t)__popcll(__ballot(claims != 0u));
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

/* a round's token between issue (vocabulary loads sent) and count */
struct Round {
    uint32_t k0, k1, k2, k3;   /* identity key (short terms) */
    uint32_t h;                /* even home slot */
    uint32_t rel, kind;        /* document in group; 0 none, 1 short term, 2 long / past the window */
    int32_t ap;                /* token start, relative to b0 (kind 2) */
#ifdef SL_DEBUG
    uint32_t ent;              /* diagnostic build: the token entry */
#endif
    uint4 s0, s1;              /* the pair's two slots */
};

}  // namespace

__global__ __launch_bounds__(NT, WG_PER_CU * NT / 256) void k_tokcount_sl(CorpusDev c, const uint64_t* __restrict__ chunk_start,
                                                               const uint32_t* __restrict__ chunk_doc, uint64_t c0,
                                                               uint64_t c1, VocabDev v, const K1Out* __restrict__ o,
                                                               uint32_t sb, uint32_t gcap) {
    __shared__ __attribute__((aligned(16))) SlShared S;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);   /* wave-uniform: scalar step loop */
    unsigned long long tokens_w = 0;
    bool clean = false;             /* the LDS table is clear (every flush clears what it emits) */
#ifdef SL_STAMPS
    /* diagnostic build: per-wave s_memtime cycles per phase (0 chunk set-up, 1 walk,
     * 2 token list, 3 round build, 4 round finish + loads, 5 the group's last rounds,
     * 6 chunk end, 7 waiting for the other waves before the flush, 8 flush (few-document
     * flushes: its record writes and clear), 9 flush entry counts, 10 flush record-space
     * allocation and its barriers, 11 a round finish's wait for its loads) */
    unsigned long long st_acc[SL_NPH] = {};
    unsigned long long st_t = __builtin_amdgcn_s_memtime(), st_chunks = 0;
    unsigned long long st_cnt[8] = {};   /* rounds with a slow lane, slow lanes, lost claims, rounds
                                            still slow after the inline retries, rounds; lanes
                                            still slow by cause (lost every retry, bucket full,
                                            overflow mode) */
#define SL_STAMP(k)                                                         \
    do {                                                                    \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();         \
        st_acc[k] += t_ - st_t;                                             \
        st_t = t_;                                                          \
    } while (0)
#else
#define SL_STAMP(k) do {} while (0)
#endif
    /* chunks are claimed from a global counter (their sizes vary: a static share leaves a
     * tail of the slowest workgroups); the next claim is sent when a chunk starts, so its
     * round trip is hidden behind the chunk */
    if (tid == 0) S.next_chunk = c0 + gatomic_add(o->chunk_ctr, 1ull);
    lds_barrier();
    unsigned long long claim = 0;
    for (uint64_t chunk = (uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)S.next_chunk) |
                          ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(S.next_chunk >> 32)) << 32);
         chunk < c1;) {
    if (tid == 0) claim = c0 + gatomic_add(o->chunk_ctr, 1ull);
    const uint64_t cs = chunk_start[chunk], ce = chunk_start[chunk + 1];
    const uint32_t dfirst = chunk_doc[chunk], dlast = chunk_doc[chunk + 1];
#ifdef SL_STAMPS
    ++st_chunks;
#endif
    if (cs < ce) {

    /* chunk base and the corpus buffer: byte at chunk-relative p is at buffer offset p + shift */
    const uint64_t b0 = cs & ~(uint64_t)15;
    const uint64_t rb = b0 >= 16 ? b0 - 16 : 0;
    const int32_t shift = (int32_t)(b0 - rb);
    /* the buffer's range check zeroes every dword at or past num_records, so the range is
     * rounded up to whole 16-byte blocks: the block holding the corpus's last byte is read
     * whole (it lies in the same page as that byte: the base is 16-byte aligned), and its
     * bytes past the shard end read as whitespace (outside16) */
    const uint64_t avail = c.nbytes > rb ? ((c.nbytes - rb + 15) & ~(uint64_t)15) : 0;
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(c.bytes + rb), 0, (int)(avail < 0x7FFFFFF0ull ? avail : 0x7FFFFFF0ull), RSRC_WORD3);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)v.keys, 0, (int)((v.mask + 1) * 16),
                                                                         RSRC_WORD3);
    const int32_t span = (int32_t)(ce - b0);                   /* chunk end, relative */
    const int32_t cs_rel = (int32_t)(cs - b0);
    const int32_t lo_rel = c.lo > b0 ? (c.lo - b0 > (uint64_t)span ? span : (int32_t)(c.lo - b0)) : -64;
    const int32_t hi_rel = c.hi - b0 > (uint64_t)span + 64 ? span + 64 : (int32_t)(c.hi - b0);

    /* The first group's document offsets and each wave's first step of corpus bytes are
     * requested before the table is cleared: the group's first step always starts at b0
     * (the chunk starts inside or at the start of its first document), so neither waits for
     * the other or for the clear. */
    const uint32_t ng0 = (dlast + 1 - dfirst) < gcap ? (dlast + 1 - dfirst) : gcap;
    const uint64_t dpre = (uint32_t)tid <= ng0 ? c.doc_off[dfirst + tid] : 0ull;
    uint4 pf = bload16<2>(crs, wid * WSTEP + 16 * lane - 16 + shift);
    /* table + selectors (once per workgroup) */
    if (!clean) {
        uint4* t = reinterpret_cast<uint4*>(S.TK);
        for (int j = tid; j < 2 * TB / 4; j += NT) t[j] = make_uint4(0, 0, 0, 0);   /* TK and TC are adjacent */
        if (tid < 64) {
            const uint32_t n = (uint32_t)tid >> 2, k = (uint32_t)tid & 3u;
            (&S.sel[n].x)[k] = perm_sel(n, k);
        }
        clean = true;
    }
    uint8_t* const stage = reinterpret_cast<uint8_t*>(&S.w.stage[wid][0]);
    uint32_t* const tl = S.w.tl[wid];

    for (uint32_t gd0 = dfirst; gd0 <= dlast; gd0 += gcap) {
        const uint32_t ng = (dlast + 1 - gd0) < gcap ? (dlast + 1 - gd0) : gcap;
        for (uint32_t k = tid; k <= ng; k += NT) {
            const uint64_t d = (gd0 == dfirst && k == (uint32_t)tid) ? dpre : c.doc_off[gd0 + k];
            S.gdoc[k] = d < b0 ? -64 : (d - b0 > (uint64_t)span + 64 ? span + 64 : (int32_t)(d - b0));
        }
        if (tid < GCAP) { S.dsz[tid] = 0; S.dpart[tid] = 0; }
        if (tid == 0) S.step_next = NWAVE;
        lds_barrier();
        if ((uint32_t)tid < ng) S.dfull[tid] = S.gdoc[tid] >= cs_rel && S.gdoc[tid + 1] <= span;
        const int32_t g0 = __builtin_amdgcn_readfirstlane(S.gdoc[0]);
        const int32_t gn = __builtin_amdgcn_readfirstlane(S.gdoc[ng]);
        const int32_t gs = g0 > cs_rel ? g0 : cs_rel;
        const int32_t ge = gn < span ? gn : span;
        SL_STAMP(0);

        Round pend, acc;
        pend.kind = 0;
        pend.k0 = pend.k1 = pend.k2 = pend.k3 = 0;
        pend.h = 0;
        pend.rel = 0;
        pend.ap = 0;
        pend.s0 = pend.s1 = make_uint4(0, 0, 0, 0);
#ifdef SL_DEBUG
        pend.ent = 0;
#endif
        acc = pend;
        uint32_t fill = 0;             /* wave-uniform: built lanes of acc */
        uint32_t wclaims = 0;          /* this wave's LDS table claims (wave-uniform) */

        /* pend takes acc's token and issues its vocabulary loads (two rounds whose roles swap
         * instead, to save the copy, made the compiler select between them through scratch) */
        auto promote = [&](Round& p, const Round& a) {
            p.k0 = a.k0; p.k1 = a.k1; p.k2 = a.k2; p.k3 = a.k3;
            p.h = a.h; p.rel = a.rel; p.kind = a.kind; p.ap = a.ap;
#ifdef SL_DEBUG
            p.ent = a.ent;
#endif
#ifdef SL_ABL_NOVOCAB   /* timing ablation (wrong output): no vocabulary loads, slot = home */
            p.s0 = make_uint4(p.k0, p.k1, p.k2, p.k3);
            p.s1 = p.s0;
#else
            p.s0 = bload16<0>(vrs, (int32_t)(p.h << 4));
            p.s1 = bload16<0>(vrs, (int32_t)(p.h << 4) + 16);
#endif
        };
        auto finish = [&](const Round& r) {
#ifdef SL_STAMPS
            /* diagnostic: the wait for the round's vocabulary loads (and, in order, every
             * older or younger load still in flight) on its own */
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            SL_STAMP(11);
#endif
            /* whole-key compares without short-circuit branches */
            const bool h0 = ((r.s0.x ^ r.k0) | (r.s0.y ^ r.k1) | (r.s0.z ^ r.k2) | (r.s0.w ^ r.k3)) == 0u;
            const bool h1 = ((r.s1.x ^ r.k0) | (r.s1.y ^ r.k1) | (r.s1.z ^ r.k2) | (r.s1.w ^ r.k3)) == 0u;
            uint32_t slot = r.h + (h0 ? 0u : 1u);
#ifdef SL_ABL_NOVOCAB
            const bool need = false;
#else
            const bool need = (r.kind == 2u) | ((r.kind == 1u) & !(h0 | h1));
#endif
            if (__ballot(need) != 0ull) {
                if (need) {
                    const uint64_t p0 = b0 + (uint64_t)(int64_t)r.ap;
                    const uint64_t dend = c.doc_off[gd0 + r.rel + 1];   /* unclamped: long terms cross chunks */
                    slot = resolve_slow(c.bytes, v.keys, v.rep, v.mask, o->status, r.kind, r.k0, r.k1, r.k2, r.k3, p0,
                                        dend);
                }
            }
            const uint32_t key = (r.kind != 0u && slot != INVALID_SLOT) ? (0x80000000u | (r.rel << sb) | slot) : 0u;
#ifdef SL_DEBUG
            if (o->stamps && r.kind != 0u) {   /* diagnostic build: one record per token */
                const unsigned long long q = atomicAdd(&o->stamps[0], 1ull);
                if (q < (K1_DEBUG_WORDS - 8) / 4) {
                    unsigned long long* d = o->stamps + 8 + 4 * q;
                    d[0] = ((unsigned long long)r.ent << 32) | ((uint32_t)r.ap << 8) | r.kind;
                    d[1] = ((unsigned long long)r.k1 << 32) | r.k0;
                    d[2] = ((unsigned long long)r.k3 << 32) | r.k2;
                    d[3] = ((unsigned long long)key << 32) | slot;
                }
            }
#endif
#ifdef SL_ABL_NOCOUNT   /* timing ablation (wrong output): no LDS count */
            wclaims += (uint32_t)__popcll(__ballot(key == 0x12345u));
            return;
#endif
            lds_count(S, o, key, wclaims, gd0, sb SL_STC);
        };
        /* one lane's token into the round being built: its key from the staged bytes */
        auto build = [&](Round& a, uint32_t e, int32_t sbp) {
            const uint32_t pos = e & 1023u, len = (e >> 10) & 31u;
            a.rel = e >> 16;
            a.ap = sbp - 16 + (int32_t)pos;
            a.kind = len >= 16u ? 2u : 1u;   /* 16..31: a long term or one past the window */
#ifdef SL_DEBUG
            a.ent = e;
#endif
            const u32x4u raw = *reinterpret_cast<const u32x4u*>(stage + pos);
            const uint4 sl = S.sel[len & 15u];
            a.k0 = __builtin_amdgcn_perm(0x09090909u, raw.x, sl.x);
            a.k1 = __builtin_amdgcn_perm(0x09090909u, raw.y, sl.y);
            a.k2 = __builtin_amdgcn_perm(0x09090909u, raw.z, sl.z);
            a.k3 = __builtin_amdgcn_perm(0x09090909u, raw.w, sl.w);
            a.h = (uint32_t)key_hash(((uint64_t)a.k1 << 32) | a.k0, ((uint64_t)a.k3 << 32) | a.k2) & (uint32_t)v.mask & ~1u;
        };
        /* acc is full (or the group's last): count pend, then send acc's vocabulary loads
         * straight into the registers pend just released (a loaded value is never copied: a
         * copy would wait for the load at once) */
        auto turn = [&]() {
            finish(pend);
            promote(pend, acc);
            acc.kind = 0u;
            fill = 0u;
        };

        if (gs < ge) {
            const int32_t bs = gs & ~15;
            const int32_t nsteps = (ge - bs + WSTEP - 1) / WSTEP;
            const bool inner_all = bs >= lo_rel + 16 && bs + nsteps * WSTEP + 16 <= hi_rel;
            if (gd0 != dfirst || bs != 0) pf = bload16<2>(crs, bs + wid * WSTEP + 16 * lane - 16 + shift);
            uint32_t wr = 0;                    /* wave-uniform: document containing the step start */
            int32_t wcur = g0, wnext = ng > 1 ? __builtin_amdgcn_readfirstlane(S.gdoc[1]) : gn;
            /* steps claimed from an LDS counter (wave w's first step is w): the waves of a
             * chunk finish within one step of each other whatever their steps cost */
            for (int32_t s = wid, snext = wid; s < nsteps; s = snext) {
                {
                    uint32_t nx = 0;
                    if (lane == 0) nx = atomicAdd(&S.step_next, 1u);
                    snext = __builtin_amdgcn_readfirstlane((int)nx);
                }
                const int32_t sbp = bs + s * WSTEP;              /* first owned byte */
                const int32_t gpos = sbp + 16 * lane - 16;       /* this lane's group */
                const uint4 cur = pf;
#ifdef SL_ABL_L2C   /* timing ablation (wrong output): every step re-reads one of the group's first four steps (L2) */
                pf = bload16<2>(crs, bs + (snext & 3) * WSTEP + 16 * lane - 16 + shift);
#else
                pf = bload16<2>(crs, bs + snext * WSTEP + 16 * lane - 16 + shift);   /* next step (harmless past ge) */
#endif
                reinterpret_cast<uint4*>(stage)[lane] = cur;
                uint32_t lt9 = 0;
                uint32_t ws = ws_mask16_dot(cur, lt9);
                if (!inner_all) ws |= outside16(gpos, lo_rel, hi_rel);
                /* document starts in the window [sbp - 16, sbp + WSTEP + 16), the document
                 * of each lane's first byte; most steps hold none */
                while (wr + 1 < ng && wnext <= sbp) {
                    ++wr;
                    wcur = wnext;
                    wnext = __builtin_amdgcn_readfirstlane(S.gdoc[wr + 1]);
                }
                uint32_t ds = 0, base = wr;
                const bool multi = wnext < sbp + WSTEP + 16 || wcur + 16 >= sbp;
                if (multi) {
                    for (uint32_t k = wr; k <= ng; ++k) {
                        const int32_t sk = __builtin_amdgcn_readfirstlane(S.gdoc[k]);
                        if (sk >= sbp + WSTEP + 16) break;
                        base += (k > wr && sk < gpos) ? 1u : 0u;
                        if (sk >= gpos && sk < gpos + 16) ds |= 1u << (uint32_t)(sk - gpos);
                    }
                }
                const uint32_t prev = (lane_prev(ws) >> 15) & 1u;
                uint32_t own = (lane >= 1 && lane <= 62) ? 0xFFFFu : 0u;
                if (!(sbp >= gs && sbp + WSTEP <= ge) && own) own &= ~outside16(gpos, gs, ge);
                const uint32_t starts = ~ws & ((ws << 1) | prev | ds) & own & 0xFFFFu;
                uint32_t nul = 0;
                const bool nulany = __ballot(lt9 != 0u) != 0ull;
                if (nulany)   /* a byte below 0x09 somewhere: exact NUL mask */
                    nul = compress4(zero_bits(cur.x)) | (compress4(zero_bits(cur.y)) << 4) |
                          (compress4(zero_bits(cur.z)) << 8) | (compress4(zero_bits(cur.w)) << 12);
                const uint32_t stop = ws | ds;
                const uint32_t stop32 = stop | (lane_next(stop) << 16), nul32 = nul | (lane_next(nul) << 16);
                const uint32_t nmine = (uint32_t)__popc(starts);
                const uint32_t incl = wave_incl_scan(nmine);
                const uint32_t ntok = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                SL_STAMP(1);
                if (ntok == 0) continue;
                tokens_w += ntok;
#ifdef SL_ABL_NOROUNDS   /* timing ablation (wrong output): tokenize only */
                if (!multi && lane == 0) atomicAdd(&S.dsz[wr], ntok);
                continue;
#endif
                if (!multi && lane == 0) atomicAdd(&S.dsz[wr], ntok);   /* the whole step is in document wr */
                /* the common step (no document start in its window, no byte below 0x09, one
                 * list pass): a token entry is its start bit, its length as the first stop bit
                 * after it (lengths >= 16 are long terms whatever their value) and one OR into
                 * the lane's loop-invariant (lane, document) bits — 10 VALU per entry with the
                 * loop, against 25 in the general form below */
                const bool fast = !multi && !nulany && ntok <= (uint32_t)TLW;
                for (uint32_t tb = 0; tb < ntok; tb += TLW) {
                    if (fast) {
                        /* bit 31 set: a token with no stop in the window gets length 31 - i >= 16 */
                        const uint32_t eb = ((uint32_t)lane << 4) | (wr << 16), s32 = stop32 | 0x80000000u;
                        uint32_t sm = starts;
                        uint32_t* p = tl + (incl - nmine);
                        while (sm) {
                            const uint32_t i = __builtin_ctz(sm);
                            sm &= sm - 1;
                            *p++ = eb | i | ((uint32_t)__builtin_ctz(s32 >> i) << 10);
                        }
                    } else {
                        uint32_t sm = starts, idx = incl - nmine;
                        while (sm) {
                            const uint32_t i = __builtin_ctz(sm);
                            sm &= sm - 1;
                            if (idx - tb < (uint32_t)TLW) {
                                const uint32_t e = ((stop32 >> i) & ~1u) | (nul32 >> i);
                                const uint32_t len = e ? (uint32_t)__builtin_ctz(e) : LEN_LONG;
                                uint32_t rel = base;
                                if (ds & ((2u << i) - 1u))
                                    while (rel + 1 < ng && S.gdoc[rel + 1] <= gpos + (int32_t)i) ++rel;
                                tl[idx - tb] = ((uint32_t)lane << 4 | i) | ((len < 16u ? len : LEN_LONG) << 10) | (rel << 16);
                                if (multi) atomicAdd(&S.dsz[rel], 1u);
                            }
                            ++idx;
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    const uint32_t cnt = (ntok - tb) < (uint32_t)TLW ? (ntok - tb) : (uint32_t)TLW;
                    SL_STAMP(2);
                    /* rounds are filled across steps: lanes [0, fill) of acc hold tokens built
                     * from earlier steps (their bytes already read, their vocabulary loads sent),
                     * so every counted round is a full 64 except the group's last */
                    for (uint32_t t = 0; t < cnt;) {
                        const uint32_t m = (64u - fill) < (cnt - t) ? (64u - fill) : (cnt - t);
                        if ((uint32_t)lane >= fill && (uint32_t)lane < fill + m) {
                            const uint32_t e = tl[t + (uint32_t)lane - fill];
                            build(acc, e, sbp);
                        }
                        t += m;
                        fill += m;
                        if (fill == 64u) {
                            SL_STAMP(3);
                            turn();
                            SL_STAMP(4);
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            }
        }
        SL_STAMP(3);
        if (fill) turn();   /* the group's last, partial round */
        finish(pend);   /* drain */
#ifdef SL_STAMPS
        SL_STAMP(5);
        lds_barrier();   /* (the flush's first barrier, made explicit to time the wait) */
        SL_STAMP(7);
#endif
#ifdef SL_STAMPS
        if (ng <= FEW) sl_flush_few(S, o, gd0, ng, sb, st_acc, st_t);
#else
        if (ng <= FEW) sl_flush_few(S, o, gd0, ng, sb);
#endif
        else sl_flush(S, o, gd0, ng, sb);
        if ((uint32_t)tid < ng) {
            const uint32_t n = S.dsz[tid];
            if (n) {
                if (S.dfull[tid]) gmem(o->doc_size)[gd0 + tid] = n;
                else atomicAdd(&o->doc_size[gd0 + tid], n);
            }
        }
        lds_barrier();
        SL_STAMP(8);
        if (gd0 + gcap < gd0) break;   /* overflow guard */
    }
    }   /* cs < ce */
    if (tid == 0) S.next_chunk = claim;
    lds_barrier();
    chunk = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)S.next_chunk) |
            ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(S.next_chunk >> 32)) << 32);
    SL_STAMP(6);
    }   /* chunk */
    if (lane == 0 && tokens_w) atomicAdd(o->ntokens, tokens_w);
#ifdef SL_STAMPS
    SL_STAMP(6);
    if (lane == 0 && o->stamps) {
        for (int k = 0; k < SL_NPH; ++k) atomicAdd(&o->stamps[k], st_acc[k]);
        atomicAdd(&o->stamps[SL_NPH], st_chunks);
        atomicAdd(&o->stamps[SL_NPH + 1], 1ull);
        for (int k = 0; k < 8; ++k) atomicAdd(&o->stamps[SL_NPH + 2 + k], st_cnt[k]);
    }
#endif
}

int launch_tokcount_sl(const CorpusDev& c, const uint64_t* chunk_start, const uint32_t* chunk_doc, uint64_t c0,
                       uint64_t c1, const VocabDev& v, const K1Out* o_dev, hipStream_t s) {
    if (c1 <= c0) return 0;
    if (v.mask >= (1ull << SLOT_BITS)) return -3;
    static_assert(sizeof(SlShared) * WG_PER_CU <= 163840, "LDS of WG_PER_CU workgroups per CU");
    static_assert(TB % NT == 0 && TB % BW == 0, "table rows");
    const uint32_t sbits = (uint32_t)__builtin_popcountll(v.mask);
    const uint32_t gcap = (1u << (31u - sbits)) >= (uint32_t)GCAP ? (uint32_t)GCAP : (1u << (31u - sbits));
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const uint64_t wgs = (uint64_t)ncu * WG_PER_CU;
    const uint64_t grid = (c1 - c0) < wgs ? (c1 - c0) : wgs;
    k_tokcount_sl<<<(unsigned)grid, NT, 0, s>>>(c, chunk_start, chunk_doc, c0, c1, v, o_dev, sbits, gcap);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
