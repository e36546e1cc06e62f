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
 *             (__shfl_down), hashed, and looked up in the HBM vocabulary (one 16-byte
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

__device__ __forceinline__ uint4 ld16c(const uint8_t* __restrict__ bytes, uint64_t last_blk, uint64_t pos) {
    const uint64_t p = pos < last_blk ? pos : last_blk;
    return *reinterpret_cast<const uint4*>(bytes + p);
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

/* counts (key, +n) into the table (entry claimed with count n or added to) */
__device__ __forceinline__ bool tbl_add(VsShared& S, uint64_t key, uint32_t n, uint32_t* status) {
    uint32_t h = tbl_hash(key) & (TB - 1);
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

/* Term slot of a token whose term is >= 16 bytes or whose end lies past the 32 bytes a
 * lane holds: the token is re-read from HBM (rare for text). */
__device__ __noinline__ uint32_t slow_slot(const CorpusDev& c, const VocabDev& v, uint64_t p0, uint64_t dend,
                                           uint32_t* status) {
    uint64_t p = p0;
    while (p < dend && !is_ws(c.bytes[p])) ++p;
    uint64_t n = 0;
    while (p0 + n < p && c.bytes[p0 + n] != 0) ++n;
    uint64_t klo, khi;
    if (n < 16) {
        uint64_t lo = 0, hi = 0;
        for (uint32_t k = 0; k < n; ++k) {
            const uint64_t b = c.bytes[p0 + k];
            if (k < 8) lo |= b << (8 * k); else hi |= b << (8 * (k - 8));
        }
        make_short_key(lo, hi, (uint32_t)n, &klo, &khi);
        return vocab_insert(v, klo, khi, 0, status);
    }
    make_long_key(c.bytes + p0, n, &klo, &khi);
    const uint64_t rep = ((n < 0xFFFFFFull ? n : 0xFFFFFFull) << 40) | p0;
    return vocab_insert(v, klo, khi, rep, status);
}

/* Vocabulary slot of a short key: first probe inline, the rest in vocab_insert. */
__device__ __forceinline__ uint32_t vocab_slot(const VocabDev& v, uint64_t klo, uint64_t khi, uint32_t* status) {
    const uint64_t h = key_hash(klo, khi) & v.mask;
    const uint4 s = v.keys[h];
    if (s.x == (uint32_t)klo && s.y == (uint32_t)(klo >> 32) && s.z == (uint32_t)khi && s.w == (uint32_t)(khi >> 32))
        return (uint32_t)h;
    return vocab_insert(v, klo, khi, 0, status);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
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
        const unsigned long long rb = nrec ? atomicAdd(o.rec_alloc, (unsigned long long)nrec) : 0ull;
        const unsigned long long pb = npart ? atomicAdd(o.part_alloc, (unsigned long long)npart) : 0ull;
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
    /* pass 2: scatter emitted entries, clear the table, remember kept ones */
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        if (!e[j]) continue;
        const uint32_t rel = (uint32_t)(e[j] >> (CNT_BITS + SLOT_BITS));
        const uint32_t slot = (uint32_t)(e[j] >> CNT_BITS) & ((1u << SLOT_BITS) - 1u);
        const uint32_t cnt = (uint32_t)(e[j] & CNT_MASK);
        const uint8_t st = S.dstate[rel];
        if (st == 3) { keep |= 1u << j; continue; }
        const uint32_t k = atomicAdd(&S.drun[rel], 1u);
        const uint32_t dof = S.doff[rel];
        if (st == 2) {
            const uint64_t p = rb + (dof & 0xFFFFu) + k;
            if (rec_ok) { o.rec_slot[p] = slot; o.rec_cnt[p] = cnt; }
        } else {
            const uint64_t p = pb + (dof >> 16) + k;
            if (part_ok) { o.part_doc[p] = gd0 + rel; o.part_slot[p] = slot; o.part_cnt[p] = cnt; }
        }
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j) S.T[j * NT + tid] = 0ull;
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

__global__ __launch_bounds__(NT, 4) void k_tokcount_vs(CorpusDev c, const uint64_t* __restrict__ chunk_start,
                                                       const uint32_t* __restrict__ chunk_doc, uint64_t c0,
                                                       VocabDev v, K1Out o) {
    __shared__ __attribute__((aligned(16))) VsShared S;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t chunk = c0 + blockIdx.x;
    const uint64_t cs = chunk_start[chunk], ce = chunk_start[chunk + 1];
    if (cs >= ce) return;
    const uint32_t dfirst = chunk_doc[chunk], dlast = chunk_doc[chunk + 1];
    const uint64_t last_blk = c.nbytes ? ((c.nbytes - 1) & ~(uint64_t)15) : 0;

#pragma unroll
    for (int j = 0; j < EPT; ++j) S.T[j * NT + tid] = 0ull;
    unsigned long long tokens_chunk = 0;
    uint32_t step = 0;  /* global step counter: buffer parity */
    if (tid < NT / 64) { S.wcl[0][tid] = 0; S.wcl[1][tid] = 0; }

    for (uint32_t gd0 = dfirst; gd0 <= dlast; gd0 += GCAP) {
        const uint32_t ng = (dlast + 1 - gd0) < (uint32_t)GCAP ? (dlast + 1 - gd0) : (uint32_t)GCAP;
        for (uint32_t k = tid; k <= ng; k += NT) S.gdoc[k] = c.doc_off[gd0 + k];
        if (tid < GCAP) { S.dsz[tid] = 0; S.dpart[tid] = 0; }
        __syncthreads();
        const uint64_t gs = S.gdoc[0] > cs ? S.gdoc[0] : cs;
        const uint64_t ge = S.gdoc[ng] < ce ? S.gdoc[ng] : ce;
        uint32_t fill = 0; /* table entries, identical in every thread */
        if (gs < ge) {
            const uint64_t wbase0 = gs & ~(uint64_t)15;
            uint4 pf = ld16c(c.bytes, last_blk, wbase0 + 16ull * tid);
            for (uint64_t sbase = wbase0; sbase < ge; sbase += STEP, ++step) {
                const uint32_t par = step & 1u;
                const uint64_t gpos = sbase + 16ull * tid;
                const uint4 cur = pf;
                pf = ld16c(c.bytes, last_blk, gpos + STEP); /* next step, harmless past ge */
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
                uint32_t prev = __shfl_up(ws >> 15, 1, 64) & 1u;
                if (lane == 0) {
                    prev = 1u;
                    if (gpos > c.lo && gpos - 1 < c.hi) prev = is_ws(c.bytes[gpos - 1]) ? 1u : 0u;
                }
                const uint32_t starts = ~ws & (((ws << 1) | prev) | ds) & own & 0xFFFFu;
                /* the neighbour's 16 bytes and stop mask (tokens running into it) */
                uint4 nxt;
                nxt.x = __shfl_down(cur.x, 1, 64);
                nxt.y = __shfl_down(cur.y, 1, 64);
                nxt.z = __shfl_down(cur.z, 1, 64);
                nxt.w = __shfl_down(cur.w, 1, 64);
                uint32_t nstop = __shfl_down(stop, 1, 64);
                if (lane == 63 && starts) {
                    nxt = ld16c(c.bytes, last_blk, gpos + 16);
                    nstop = ws_mask16(nxt) | bounds_ws(gpos + 16, c.lo, c.hi) | doc_start_bits(S, ng, r0, gpos + 16);
                }
                /* ---- step token count -> flush decision (identical in every thread) ---- */
                const uint32_t wt = wave_sum((uint32_t)__popc(starts));
                if (lane == 0) S.wtok[par][wid] = wt;
                __syncthreads();
                uint32_t ntok = 0, ncl = 0;
#pragma unroll
                for (int q = 0; q < NT / 64; ++q) { ntok += S.wtok[par][q]; ncl += S.wcl[par ^ 1u][q]; }
                fill += ncl;
                tokens_chunk += ntok;
                if (fill + ntok > SOFT) fill = vs_flush(S, o, gd0, ng, cs, ce, sbase, false, ntok);
                /* ---- resolve + insert this lane's tokens ---- */
                uint32_t claims = 0;
                if (starts) {
                    const uint64_t q0 = ((uint64_t)cur.y << 32) | cur.x, q1 = ((uint64_t)cur.w << 32) | cur.z;
                    const uint64_t q2 = ((uint64_t)nxt.y << 32) | nxt.x, q3 = ((uint64_t)nxt.w << 32) | nxt.z;
                    const uint32_t s32 = stop | (nstop << 16);
                    uint32_t rel = r0;
                    uint64_t nstart = S.gdoc[rel + 1];
                    uint32_t run_rel = rel, run_n = 0;
                    uint32_t sm = starts;
                    while (sm) {
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
                        uint64_t klo, khi;
                        uint32_t slot;
                        if (make_short_key(lo, hi, len, &klo, &khi) < 16u)
                            slot = vocab_slot(v, klo, khi, o.status);
                        else
                            slot = slow_slot(c, v, ap, nstart, o.status);
                        if (rel != run_rel) {
                            if (run_n) atomicAdd(&S.dsz[run_rel], run_n);
                            run_rel = rel;
                            run_n = 0;
                        }
                        ++run_n;
                        if (slot == INVALID_SLOT) continue; /* status flagged: the run is retried */
                        if (tbl_add(S, ((uint64_t)rel << SLOT_BITS) | slot, 1u, o.status)) ++claims;
                    }
                    if (run_n) atomicAdd(&S.dsz[run_rel], run_n);
                }
                const uint32_t wc = wave_sum(claims);
                if (lane == 0) S.wcl[par][wid] = wc;
            }
        }
        /* group end is a document boundary (or the chunk end): emit everything */
        vs_flush(S, o, gd0, ng, cs, ce, ge, true, 0);
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
        if (gd0 + GCAP < gd0) break; /* overflow guard */
    }
    if (tid == 0) atomicAdd(o.ntokens, tokens_chunk);
}

int launch_tokcount_vs(const CorpusDev& c, const uint64_t* chunk_start, const uint32_t* chunk_doc, uint64_t c0,
                       uint64_t c1, const VocabDev& v, const K1Out& o, hipStream_t s) {
    if (c1 <= c0) return 0;
    if (v.mask >= (1ull << SLOT_BITS)) return -3; /* slot must fit the LDS entry */
    k_tokcount_vs<<<(unsigned)(c1 - c0), NT, 0, s>>>(c, chunk_start, chunk_doc, c0, v, o);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
