/*
 * tokcount_ws.hip — K1 fast path: fused tokenize + per-document term counting for corpora
 * whose documents are whitespace-separated (the byte before every non-empty document
 * is C-locale whitespace, as for text files ending in '\n') and whose base address is
 * 16-byte aligned.  Token boundaries are then whitespace alone (TFIDF.c:142,147
 * fscanf("%s")), so no per-window document-start bitmap is needed; documents only
 * attribute tokens.  tokcount.hip's k_tokcount remains the general path.
 *
 * One 256-thread workgroup per chunk (K0), two workgroups per CU (~70 KB LDS each):
 *   document groups: up to GCAP documents of the chunk at a time, their offsets staged
 *     in LDS (token -> document, containment tests, docSize sums);
 *   windows of 4 KiB (+64 B lookahead): one 16-byte group per lane, loaded one window
 *     ahead into registers by a branch-free clamped global_load_dwordx4 (so the compiler
 *     places no vmcnt wait until the next window uses it), staged to LDS and classified
 *     into a 16-bit whitespace mask; token starts compacted by a block scan into an LDS
 *     list of packed (offset:12 | length:12 | doc:8) words;
 *   docSize: -first index / +(last index + 1) per document and window (no per-token
 *     atomics);
 *   segments: thread 0 cuts the window's tokens where the (doc, term) table must be
 *     flushed — at a document boundary once it holds FLUSH_THR entries, mid-document
 *     only above HARD entries (that document then goes to the partial stream);
 *   insert: three tokens per lane in flight — their key bytes, then their first table
 *     probe (count word and 128-bit key read in the same LDS round trip) — so LDS
 *     latency overlaps; a hit is one 64-bit LDS atomic add, a claim one 64-bit CAS plus
 *     one 128-bit key write;
 *   flush: occupied slots are compacted, each term is resolved to its global
 *     vocabulary slot (first probe loads issued four wide), and (slot, count) records
 *     are written grouped by document (complete documents) or to the partial stream.
 */
#include "dev_common.h"
#include "dev_vocab.h"
#include "kernels.h"

namespace {

constexpr int NT = K1_NT;
constexpr int WIN = K1_WIN;
constexpr int LOOK = 64;
constexpr int NGRP = (WIN + LOOK) / 16;
constexpr int NEXTRA = NGRP - NT;          /* lookahead groups, loaded by lanes 0..NEXTRA-1 */
constexpr int MAXTOK = WIN / 2 + 2;
constexpr int TBL = 2048;
constexpr int HARD = 1536;                 /* above this (load 0.75) the open document is split */
constexpr int FLUSH_THR = 256;             /* above this, flush at the next document boundary */
constexpr int GCAP = 256;                  /* documents per group (token doc field: 8 bits) */
constexpr uint32_t LEN_OPEN = 0xFFFu;      /* token length >= 4095 or end beyond the lookahead */
constexpr int KIL = 3;                     /* tokens in flight per lane during insert */
constexpr unsigned long long TDC_EMPTY = ~0ull;
constexpr uint32_t REL_NONE = 0xFFFFFFFFu;
enum { DEC_INSERT = 0, DEC_FLUSH_CLEAN = 1, DEC_FLUSH_MID = 2 };

__device__ __forceinline__ uint32_t tok_rel(uint32_t t) { return t >> 20; }
__device__ __forceinline__ uint32_t tok_len(uint32_t t) { return (t >> 8) & 0xFFFu; }
__device__ __forceinline__ uint32_t tok_doc(uint32_t t) { return t & 0xFFu; }

/* Diagnostic build only (-DK1_STAMPS, lib/libtfidf_hip_stamps.so): lane 0 accumulates
 * s_memtime cycles per phase; never compiled into the measured library. */
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
#else
struct Stamps {};
#define STAMP(st, k) do { (void)(st); } while (0)
#endif
#ifdef K1_STAMPS
#define CNT(k, n) (cnt_[k] += (n))
#else
#define CNT(k, n) ((void)0)
#endif

struct WsShared {
    uint8_t bytes[WIN + LOOK + 32];
    uint32_t tok[MAXTOK];                  /* packed (offset, length, doc) */
    ulonglong2 key[TBL];                   /* {lo, hi}: written as ONE 128-bit LDS access */
    unsigned long long tdc[TBL];           /* (doc_rel << 32) | count */
    uint16_t wsm[NGRP];
    uint64_t gdoc[GCAP + 1];               /* doc_off of the group's documents */
    uint32_t dsz[GCAP];                    /* docSize accumulators */
    uint32_t dcnt[GCAP];
    uint32_t drun[GCAP];
    uint16_t flist[TBL];
    uint32_t wsum[NT / 64];
    uint32_t fill, npart, pfill, ntok_w, seg_end, decision, open_doc, partial_doc, prev_ws;
    unsigned long long rec_base, part_base;
};

/* Branch-free aligned 16-byte group load: the address is clamped to the last 16-byte
 * block holding corpus bytes (same page as the buffer's end); bytes at or past the
 * corpus end are turned into whitespace by the caller's bounds mask. */
__device__ __forceinline__ uint4 ld16c(const uint8_t* __restrict__ bytes, uint64_t last_blk, uint64_t pos) {
    const uint64_t p = pos < last_blk ? pos : last_blk;
    return *reinterpret_cast<const uint4*>(bytes + p);
}

__device__ __forceinline__ uint32_t bounds_ws(uint64_t pos, uint64_t lo, uint64_t hi) {
    uint32_t m = 0;
    if (pos < lo || pos + 16 > hi)
        for (int i = 0; i < 16; ++i) if (pos + i < lo || pos + i >= hi) m |= 1u << i;
    return m;
}

__device__ __forceinline__ uint32_t tbl_hash(uint64_t lo, uint64_t hi, uint32_t dr) {
    uint32_t h = (uint32_t)lo * 0x9E3779B1u ^ (uint32_t)(lo >> 32) * 0x85EBCA77u ^ (uint32_t)hi * 0xC2B2AE3Du ^
                 (uint32_t)(hi >> 32) * 0x27D4EB2Fu ^ (dr + 1u) * 0x165667B1u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 13;
    return h;
}

/* Full probe/insert of (dr, key) from slot h.  Slots are claimed once per epoch and keys
 * are reset to the EMPTY sentinel at every flush, so a key read is either the sentinel
 * (claimer still writing: retry) or final; keys move as one 128-bit LDS access and no
 * fence is needed. */
__device__ __forceinline__ uint32_t tbl_probe(WsShared& S, uint32_t h, uint32_t dr, uint64_t klo, uint64_t khi,
                                              uint32_t& claims, uint32_t* status) {
    const unsigned long long mine = ((unsigned long long)dr << 32) | 1ull; /* claimed with count 1 */
    for (uint32_t guard = 0;; ++guard) {
        if (guard > (1u << 16)) { atomicOr(status, ST_VOCAB_SPIN); return guard; }
        asm volatile("" ::: "memory");
        unsigned long long w = S.tdc[h];
        if (w == TDC_EMPTY) {
            unsigned long long old = atomicCAS(&S.tdc[h], TDC_EMPTY, mine);
            if (old == TDC_EMPTY) {
                S.key[h] = make_ulonglong2(klo, khi);
                ++claims;
                return guard + 1;
            }
            w = old;
        }
        if ((w >> 32) == dr) {
            const ulonglong2 kk = S.key[h];
            if (kk.y == KEY_EMPTY_HI) { __builtin_amdgcn_s_sleep(1); continue; }
            if (kk.y == khi && kk.x == klo) { atomicAdd(&S.tdc[h], 1ull); return guard + 1; }
        }
        h = (h + 1) & (TBL - 1);
    }
}

/* Key of a token whose bytes are not all in the staged window, or whose term is >= 16
 * bytes: read from global memory (rare).  Long terms are resolved to their global
 * vocabulary slot right away (key = {slot, KEY_GSLOT_TAG}). */
__device__ __noinline__ ulonglong2 slow_key(const CorpusDev& c, const VocabDev& v, uint64_t p0, uint64_t dend,
                                            uint32_t* status) {
    uint64_t klo_, khi_;
    uint64_t* klo = &klo_;
    uint64_t* khi = &khi_;
    uint64_t p = p0;
    while (p < dend && p < c.nbytes && !is_ws(c.bytes[p])) ++p;
    uint64_t n = 0;
    while (p0 + n < p && c.bytes[p0 + n] != 0) ++n;
    if (n < 16) {
        uint64_t lo = 0, hi = 0;
        for (uint32_t k = 0; k < n; ++k) {
            uint64_t b = c.bytes[p0 + k];
            if (k < 8) lo |= b << (8 * k); else hi |= b << (8 * (k - 8));
        }
        make_short_key(lo, hi, (uint32_t)n, klo, khi);
    } else {
        make_long_key(c.bytes + p0, n, klo, khi);
        uint64_t rep = ((n < 0xFFFFFFull ? n : 0xFFFFFFull) << 40) | p0;
        *klo = vocab_insert(v, *klo, *khi, rep, status);
        *khi = KEY_GSLOT_TAG;
    }
    return make_ulonglong2(klo_, khi_);
}

/* Emits every table entry and clears the table.  straddle = group-relative document that
 * continues after this flush, or REL_NONE. */
__device__ void ws_flush(WsShared& S, const VocabDev& v, const K1Out& o, uint32_t gd0, uint64_t cs, uint64_t ce,
                         uint32_t straddle, Stamps& st) {
    const int tid = threadIdx.x;
    __syncthreads();
    STAMP(st, 6);
    /* A: compact occupied slots (8 consecutive slots per lane) */
    uint32_t occ = 0;
#pragma unroll
    for (int k = 0; k < TBL / NT; ++k)
        occ |= (S.tdc[tid * (TBL / NT) + k] != TDC_EMPTY ? 1u : 0u) << k;
    uint32_t nocc;
    uint32_t off = block_excl_scan<NT>((uint32_t)__popc(occ), S.wsum, &nocc);
    for (uint32_t m = occ; m; m &= m - 1) S.flist[off++] = (uint16_t)(tid * (TBL / NT) + __builtin_ctz(m));
    if (tid < GCAP) S.dcnt[tid] = 0;
    if (tid == 0) { S.npart = 0; S.pfill = 0; }
    const uint32_t pdoc = S.partial_doc;
    __syncthreads();
    STAMP(st, 7);
    /* B: resolve each term's global slot (first probe loads issued four wide,
     * unconditionally, so no wait is placed between them) */
    for (uint32_t e0 = tid; e0 < nocc; e0 += 4 * NT) {
        uint32_t sl[4];
        uint64_t lo[4], hi[4], h[4];
        uint4 pk[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t e = e0 + q * NT;
            sl[q] = e < nocc ? S.flist[e] : 0u;
            const ulonglong2 kk = S.key[sl[q]];
            lo[q] = kk.x;
            hi[q] = kk.y;
            h[q] = key_hash(lo[q], hi[q]) & v.mask;
            pk[q] = v.keys[h[q]];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t e = e0 + q * NT;
            if (e >= nocc) continue;
            uint32_t g;
            if (hi[q] == KEY_GSLOT_TAG) {
                g = (uint32_t)lo[q];
            } else {
                uint64_t plo = ((uint64_t)pk[q].y << 32) | pk[q].x, phi = ((uint64_t)pk[q].w << 32) | pk[q].z;
                g = (plo == lo[q] && phi == hi[q]) ? (uint32_t)h[q] : vocab_insert(v, lo[q], hi[q], 0, o.status);
            }
            S.key[sl[q]].x = g;
            uint32_t rel = (uint32_t)(S.tdc[sl[q]] >> 32);
            bool comp = rel != straddle && rel != pdoc && S.gdoc[rel] >= cs && S.gdoc[rel + 1] <= ce;
            if (comp) atomicAdd(&S.dcnt[rel], 1u);
            else atomicAdd(&S.npart, 1u);
        }
    }
    __syncthreads();
    STAMP(st, 8);
    /* C: per-document record offsets; one allocation for records, one for partials */
    uint32_t tot;
    const uint32_t mycnt = tid < GCAP ? S.dcnt[tid] : 0u;
    const uint32_t myoff = block_excl_scan<NT>(mycnt, S.wsum, &tot);
    if (tid < GCAP) S.drun[tid] = myoff;
    if (tid == 0) {
        S.rec_base = tot ? atomicAdd(o.rec_alloc, (unsigned long long)tot) : 0ull;
        S.part_base = S.npart ? atomicAdd(o.part_alloc, (unsigned long long)S.npart) : 0ull;
        if (S.rec_base + tot > o.rec_cap) atomicOr(o.status, ST_REC_FULL);
        if (S.part_base + S.npart > o.part_cap) atomicOr(o.status, ST_PART_FULL);
    }
    __syncthreads();
    const unsigned long long rb = S.rec_base, pb = S.part_base;
    const bool rec_ok = rb + tot <= o.rec_cap, part_ok = pb + S.npart <= o.part_cap;
    STAMP(st, 9);
    if (tid < GCAP && mycnt) {
        o.doc_recoff[gd0 + tid] = rb + myoff;
        o.doc_npairs[gd0 + tid] = mycnt;
    }
    /* D: records */
    for (uint32_t e = tid; e < nocc; e += NT) {
        uint32_t s = S.flist[e];
        unsigned long long w = S.tdc[s];
        uint32_t rel = (uint32_t)(w >> 32), cnt = (uint32_t)w, g = (uint32_t)S.key[s].x;
        bool comp = rel != straddle && rel != pdoc && S.gdoc[rel] >= cs && S.gdoc[rel + 1] <= ce;
        if (comp) {
            uint64_t pos = rb + atomicAdd(&S.drun[rel], 1u);
            if (rec_ok) { o.rec_slot[pos] = g; o.rec_cnt[pos] = cnt; }
        } else {
            uint64_t pos = pb + atomicAdd(&S.pfill, 1u);
            if (part_ok) { o.part_doc[pos] = gd0 + rel; o.part_slot[pos] = g; o.part_cnt[pos] = cnt; }
            o.doc_flags[gd0 + rel] = DF_PARTIAL;
        }
        /* E: clear the slot */
        S.tdc[s] = TDC_EMPTY;
        S.key[s] = make_ulonglong2(0ull, KEY_EMPTY_HI);
    }
    __syncthreads();
    if (tid == 0) {
        S.fill = 0;
        S.open_doc = REL_NONE;
        if (straddle != REL_NONE) S.partial_doc = straddle;
    }
    __syncthreads();
    STAMP(st, 10);
}

}  // namespace

/* flag = 1 unless every non-empty document is preceded by whitespace (or the corpus
 * start): the fast path's precondition. */
__global__ void k_docs_ws_sep(CorpusDev c, uint32_t* __restrict__ flag) {
    uint32_t d = blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (d >= c.ndocs) return;
    uint64_t s = c.doc_off[d];
    if (c.doc_off[d + 1] > s && s > c.lo && !is_ws(c.bytes[s - 1])) atomicOr(flag, 1u);
}
int launch_docs_ws_sep(const CorpusDev& c, uint32_t* flag, hipStream_t s) {
    if (c.ndocs > 1) k_docs_ws_sep<<<(c.ndocs + 255) / 256, 256, 0, s>>>(c, flag);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ __launch_bounds__(NT, 2) void k_tokcount_ws(CorpusDev c, const uint64_t* __restrict__ chunk_start,
                                                       const uint32_t* __restrict__ chunk_doc, uint64_t c0,
                                                       VocabDev v, K1Out o) {
    __shared__ __attribute__((aligned(16))) WsShared S;
    const int tid = threadIdx.x, lane = tid & 63;
    const uint64_t chunk = c0 + blockIdx.x;
    const uint64_t cs = chunk_start[chunk], ce = chunk_start[chunk + 1];
    if (cs >= ce) return;
    const uint32_t dfirst = chunk_doc[chunk], dlast = chunk_doc[chunk + 1];
    const uint64_t last_blk = c.nbytes ? ((c.nbytes - 1) & ~(uint64_t)15) : 0;

    for (int s = tid; s < TBL; s += NT) { S.tdc[s] = TDC_EMPTY; S.key[s] = make_ulonglong2(0ull, KEY_EMPTY_HI); }
    if (tid == 0) { S.fill = 0; S.open_doc = REL_NONE; }
    unsigned long long tokens_chunk = 0;
    Stamps st;
#ifdef K1_STAMPS
    st.prev = 0;
    for (int k = 0; k < K1_NSTAMP; ++k) st.acc[k] = 0;
    uint32_t cnt_[K1_NCOUNT] = {0, 0, 0, 0};
#endif
    STAMP(st, 11);

    for (uint32_t gd0 = dfirst; gd0 <= dlast; gd0 += GCAP) {
        const uint32_t ng = (dlast + 1 - gd0) < (uint32_t)GCAP ? (dlast + 1 - gd0) : (uint32_t)GCAP;
        for (uint32_t k = tid; k <= ng; k += NT) S.gdoc[k] = c.doc_off[gd0 + k];
        if (tid < GCAP) S.dsz[tid] = 0;
        if (tid == 0) S.partial_doc = REL_NONE;
        __syncthreads();
        STAMP(st, 0);
        const uint64_t gs = S.gdoc[0] > cs ? S.gdoc[0] : cs;
        const uint64_t ge = S.gdoc[ng] < ce ? S.gdoc[ng] : ce;
        if (gs < ge) {
            const uint64_t wbase0 = gs & ~(uint64_t)15;
            if (tid == 0) {
                uint32_t pw = 1;
                if (wbase0 > c.lo && wbase0 - 1 < c.hi) pw = is_ws(c.bytes[wbase0 - 1]) ? 1u : 0u;
                S.prev_ws = pw;
            }
            uint4 pf0 = ld16c(c.bytes, last_blk, wbase0 + 16ull * tid);
            uint4 pf1 = ld16c(c.bytes, last_blk, wbase0 + 16ull * (NT + (tid & (NEXTRA - 1))));
            for (uint64_t wbase = wbase0; wbase < ge; wbase += WIN) {
                /* ---- stage + classify (this window was prefetched) ---- */
                const uint64_t own_lo = wbase > gs ? wbase : gs;
                const uint64_t own_hi = (wbase + WIN) < ge ? (wbase + WIN) : ge;
                uint32_t my_ws;
                {
                    *reinterpret_cast<uint4*>(&S.bytes[16 * tid]) = pf0;
                    const uint64_t pos = wbase + 16ull * tid;
                    my_ws = ws_mask16(pf0) | bounds_ws(pos, c.lo, c.hi);
                    S.wsm[tid] = (uint16_t)my_ws;
                    if (tid < NEXTRA) {
                        *reinterpret_cast<uint4*>(&S.bytes[16 * (NT + tid)]) = pf1;
                        const uint64_t p1 = wbase + 16ull * (NT + tid);
                        S.wsm[NT + tid] = (uint16_t)(ws_mask16(pf1) | bounds_ws(p1, c.lo, c.hi));
                    }
                }
                /* prefetch the next window while this one is processed (harmless past ge) */
                pf0 = ld16c(c.bytes, last_blk, wbase + WIN + 16ull * tid);
                pf1 = ld16c(c.bytes, last_blk, wbase + WIN + 16ull * (NT + (tid & (NEXTRA - 1))));
                __syncthreads();
                STAMP(st, 1);
                /* ---- token starts, compaction, document of each token ---- */
                {
                    const uint64_t gpos = wbase + 16ull * tid;
                    const uint32_t prevw = tid ? ((S.wsm[tid - 1] >> 15) & 1u) : S.prev_ws;
                    uint32_t owned = 0;
                    if (gpos + 16 > own_lo && gpos < own_hi) {
                        uint32_t a = gpos < own_lo ? (uint32_t)(own_lo - gpos) : 0u;
                        uint32_t b = gpos + 16 > own_hi ? (uint32_t)(own_hi - gpos) : 16u;
                        owned = ((1u << b) - 1u) & ~((1u << a) - 1u);
                    }
                    uint32_t starts = ~my_ws & ((my_ws << 1) | prevw) & owned & 0xFFFFu;
                    uint32_t tot;
                    uint32_t off = block_excl_scan<NT>((uint32_t)__popc(starts), S.wsum, &tot);
                    if (starts) {
                        /* document of this lane's group: one search per lane, then walk */
                        const uint64_t first = gpos + __builtin_ctz(starts);
                        uint32_t lo = 0, hi = ng;
                        while (hi - lo > 1) {
                            uint32_t mid = (lo + hi) >> 1;
                            if (S.gdoc[mid] <= first) lo = mid; else hi = mid;
                        }
                        uint64_t next_start = S.gdoc[lo + 1];
                        const uint32_t nxt_ws = (tid + 1 < NGRP) ? S.wsm[tid + 1] : 0xFFFFu;
                        while (starts) {
                            const uint32_t i = __builtin_ctz(starts);
                            starts &= starts - 1;
                            uint32_t len = LEN_OPEN;
                            const uint32_t m = (my_ws >> (i + 1)) & 0xFFFFu;
                            if (m) {
                                len = __builtin_ctz(m) + 1;
                            } else if (nxt_ws) {
                                len = 16u - i + __builtin_ctz(nxt_ws);
                            } else {
                                for (int gg = tid + 2; gg < NGRP; ++gg) {
                                    uint32_t sm = S.wsm[gg];
                                    if (sm) { len = 16u * (gg - tid) + __builtin_ctz(sm) - i; break; }
                                }
                            }
                            const uint64_t ap = gpos + i;
                            while (ap >= next_start) { ++lo; next_start = S.gdoc[lo + 1]; }
                            const uint32_t rel = 16u * tid + i;
                            S.tok[off++] = (rel << 20) | ((len < LEN_OPEN ? len : LEN_OPEN) << 8) | lo;
                        }
                    }
                    if (tid == 0) S.ntok_w = tot;
                }
                __syncthreads();
                STAMP(st, 2);
                const uint32_t ntok = S.ntok_w;
                tokens_chunk += ntok;
                /* ---- docSize: - first index, + (last index + 1) per document ---- */
                for (uint32_t i = tid; i < ntok; i += NT) {
                    const uint32_t dr = tok_doc(S.tok[i]);
                    if (i == 0 || tok_doc(S.tok[i - 1]) != dr) atomicSub(&S.dsz[dr], i);
                    if (i + 1 == ntok || tok_doc(S.tok[i + 1]) != dr) atomicAdd(&S.dsz[dr], i + 1);
                }
                STAMP(st, 3);
                /* ---- segments ---- */
                uint32_t pos = 0;
                while (pos < ntok) {
                    if (tid == 0) {
                        /* Flush cleanly at a document boundary once the table holds
                         * FLUSH_THR entries; split the open document only above HARD.  A
                         * segment never adds more tokens than the table has slots left
                         * (minus a margin), so inserts cannot overflow. */
                        const uint32_t fill0 = S.fill, open = S.open_doc;
                        const uint32_t cur = tok_doc(S.tok[pos]);
                        const bool at_boundary = open == REL_NONE || cur != open;
                        uint32_t e = ntok, dec = DEC_INSERT;
                        if (fill0 > (uint32_t)FLUSH_THR && at_boundary) {
                            dec = DEC_FLUSH_CLEAN;
                        } else if (fill0 > (uint32_t)HARD) {
                            dec = DEC_FLUSH_MID; /* mid-document (at_boundary is false here) */
                        } else {
                            const uint32_t room = (uint32_t)(TBL - 64) - fill0;
                            if (e > pos + room) e = pos + room;
                            if (fill0 + (e - pos) > (uint32_t)FLUSH_THR) {
                                /* will cross the threshold: stop at the end of the current
                                 * document so the next decision can flush cleanly */
                                uint32_t lo = pos, hi = e;
                                while (lo < hi) {
                                    uint32_t mid = (lo + hi) >> 1;
                                    if (tok_doc(S.tok[mid]) > cur) hi = mid; else lo = mid + 1;
                                }
                                e = lo;
                            }
                        }
                        S.decision = dec;
                        S.seg_end = e;
                        if (dec == DEC_INSERT) S.open_doc = tok_doc(S.tok[e - 1]);
                    }
                    __syncthreads();
                    STAMP(st, 4);
                    const uint32_t dec = S.decision, e = S.seg_end;
                    if (tid == 0) CNT(dec == DEC_INSERT ? 0 : 1, 1);
                    if (dec != DEC_INSERT) {
                        ws_flush(S, v, o, gd0, cs, ce, dec == DEC_FLUSH_MID ? S.open_doc : REL_NONE, st);
                        continue;
                    }
                    uint32_t claims = 0;
                    for (uint32_t i0 = pos + tid; i0 < e; i0 += KIL * NT) {
                        uint32_t dr[KIL], h[KIL];
                        uint64_t klo[KIL], khi[KIL];
                        bool val[KIL];
                        /* key bytes of KIL tokens (independent LDS reads) */
#pragma unroll
                        for (int k = 0; k < KIL; ++k) {
                            const uint32_t i = i0 + k * NT;
                            val[k] = i < e;
                            const uint32_t tw = val[k] ? S.tok[i] : 0u;
                            const uint32_t rel = tok_rel(tw), len = tok_len(tw);
                            dr[k] = tok_doc(tw);
                            const uint32_t a = rel & ~7u;
                            const uint64_t* q = reinterpret_cast<const uint64_t*>(&S.bytes[a]);
                            const uint64_t w0 = q[0], w1 = q[1], w2 = q[2];
                            const uint32_t sh = (rel & 7u) * 8u;
                            const uint64_t lo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
                            const uint64_t hi = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
                            bool slow = len == LEN_OPEN;
                            if (!slow) slow = make_short_key(lo, hi, len, &klo[k], &khi[k]) >= 16u;
                            if (val[k] && slow) {
                                const ulonglong2 sk = slow_key(c, v, wbase + rel, S.gdoc[dr[k] + 1], o.status);
                                klo[k] = sk.x;
                                khi[k] = sk.y;
                            }
                            h[k] = tbl_hash(klo[k], khi[k], dr[k]) & (TBL - 1);
                        }
                        /* first probe of KIL tokens: count word and key in one round trip */
                        unsigned long long tw8[KIL];
                        ulonglong2 kk[KIL];
#pragma unroll
                        for (int k = 0; k < KIL; ++k) {
                            tw8[k] = S.tdc[h[k]];
                            kk[k] = S.key[h[k]];
                        }
                        /* hits: one non-returning atomic add each; empty slots: claim with a
                         * count of 1 (the CASes of all KIL tokens in flight together) */
                        unsigned long long cas[KIL];
#pragma unroll
                        for (int k = 0; k < KIL; ++k) {
                            const bool mine = (uint32_t)(tw8[k] >> 32) == dr[k];
                            const bool hit = val[k] && tw8[k] != TDC_EMPTY && mine && kk[k].y == khi[k] && kk[k].x == klo[k];
                            if (hit) atomicAdd(&S.tdc[h[k]], 1ull);
                            cas[k] = 0;
                            if (val[k] && tw8[k] == TDC_EMPTY)
                                cas[k] = atomicCAS(&S.tdc[h[k]], TDC_EMPTY, ((unsigned long long)dr[k] << 32) | 1ull);
                            else if (hit)
                                val[k] = false;
                        }
                        /* publish every key claimed above BEFORE any lane starts a full probe:
                         * a probing lane may spin on one of these slots, and the claiming lane
                         * must not be waiting behind it (same wave, or a later k) */
#pragma unroll
                        for (int k = 0; k < KIL; ++k) {
                            if (val[k] && tw8[k] == TDC_EMPTY && cas[k] == TDC_EMPTY) {
                                S.key[h[k]] = make_ulonglong2(klo[k], khi[k]);
                                ++claims;
                                val[k] = false;
                            }
                        }
#pragma unroll
                        for (int k = 0; k < KIL; ++k) {
                            if (!val[k]) continue;
                            const uint32_t it = tbl_probe(S, h[k], dr[k], klo[k], khi[k], claims, o.status);
                            CNT(2, 1);
                            CNT(3, it);
                            (void)it;
                        }
                    }
                    /* wave-aggregated fill counter */
                    for (int off2 = 32; off2 > 0; off2 >>= 1) claims += __shfl_xor(claims, off2, 64);
                    if (lane == 0 && claims) atomicAdd(&S.fill, claims);
                    __syncthreads();
                    STAMP(st, 5);
                    pos = e;
                }
                if (tid == 0) S.prev_ws = (S.wsm[NT - 1] >> 15) & 1u;
                __syncthreads();
            }
        }
        /* group end is a document boundary: flush, then docSize of the group's documents */
        ws_flush(S, v, o, gd0, cs, ce, REL_NONE, st);
        if ((uint32_t)tid < ng) {
            uint32_t n = S.dsz[tid];
            if (n) {
                uint32_t d = gd0 + tid;
                if (S.gdoc[tid] >= cs && S.gdoc[tid + 1] <= ce) o.doc_size[d] = n;
                else atomicAdd(&o.doc_size[d], n);
            }
        }
        __syncthreads();
        if (gd0 + GCAP < gd0) break; /* overflow guard */
    }
    if (tid == 0) atomicAdd(o.ntokens, tokens_chunk);
#ifdef K1_STAMPS
    STAMP(st, 11);
    if (tid == 0 && o.stamps) {
        for (int k = 0; k < K1_NSTAMP; ++k) atomicAdd(&o.stamps[k], (unsigned long long)st.acc[k]);
        atomicAdd(&o.stamps[K1_NSTAMP], 1ull);
    }
    if (o.stamps)
        for (int k = 0; k < K1_NCOUNT; ++k)
            if (cnt_[k]) atomicAdd(&o.stamps[K1_NSTAMP + 1 + k], (unsigned long long)cnt_[k]);
#endif
}

int launch_tokcount_ws(const CorpusDev& c, const uint64_t* chunk_start, const uint32_t* chunk_doc, uint64_t c0,
                       uint64_t c1, const VocabDev& v, const K1Out& o, hipStream_t s) {
    if (c1 <= c0) return 0;
    k_tokcount_ws<<<(unsigned)(c1 - c0), NT, 0, s>>>(c, chunk_start, chunk_doc, c0, v, o);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
