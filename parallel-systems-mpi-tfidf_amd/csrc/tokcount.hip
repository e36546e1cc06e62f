/*
 * tokcount.hip — K0 (chunk plan) and K1 (fused tokenize + per-document term count).
 *
 * Replaces the reference's per-rank hot loop TFIDF.c:130-196: fscanf("%s") tokenising
 * (:141-147), the O(P) strcmp search/append of (word, doc) records (:151-167) and the
 * per-rank DF table (:169-188).  Here one 256-thread workgroup owns one chunk of the
 * HBM-resident corpus:
 *   window loop (4 KiB + 64 B lookahead per window):
 *     - each lane loads one 16-byte group (coalesced global_load_dwordx4), stages it in
 *       LDS and classifies it into a 16-bit whitespace mask;
 *     - document starts of the window become a bitmap (token boundaries) and a sorted
 *       (offset, doc) list for the token -> document lookup;
 *     - token starts = non-ws & (previous byte ws | document start); the block scan of
 *       per-lane start counts compacts (offset, length) tokens into an LDS list;
 *     - tokens are consumed 256 at a time: a 128-bit term key is assembled from LDS
 *       (dev_common.h) and (doc, key) is counted in an LDS open-addressing table
 *       (2048 slots, linear probing, CAS-claimed by document id);
 *   flushes happen at document boundaries once the table is over FLUSH_THR entries
 *   (or when it would overflow, splitting the open document): every (doc, term) entry
 *   is resolved to a slot of the global HBM vocabulary (lock-free 128-bit insert, see
 *   vocab_insert) and written as a (slot, count) record grouped by document.  Documents
 *   that straddle a flush or a chunk boundary go to the partial stream and are merged by
 *   a radix sort later (finalize.hip).
 */
#include "dev_common.h"
#include "dev_vocab.h"
#include "kernels.h"

namespace {

constexpr int NT = K1_NT;
constexpr int WIN = K1_WIN;
constexpr int LOOK = 64;
constexpr int NGRP = (WIN + LOOK) / 16;     /* staged 16-byte groups */
constexpr int MAXTOK = WIN / 2 + 2;         /* tokens starting in one window */
constexpr int TBL = 2048;                   /* LDS (doc, term) table slots */
constexpr int TBL_HARD = 1600;              /* never exceed this many entries */
constexpr int FLUSH_THR = 384;              /* flush at the next document boundary above this */
constexpr int FDOCS = 256;                  /* documents per flush epoch */
constexpr int WDS_CAP = 256;                /* document starts listed per window */
constexpr uint32_t LEN_OPEN = 0xFFFFu;      /* token end not within the staged bytes */

/* upper_bound(doc_off[lo..hi), x) - 1 : document containing absolute byte x */
__device__ uint32_t doc_containing(const uint64_t* __restrict__ doc_off, uint32_t lo, uint32_t hi, uint64_t x) {
    while (lo < hi) {
        uint32_t mid = lo + ((hi - lo) >> 1);
        if (doc_off[mid] <= x) lo = mid + 1; else hi = mid;
    }
    return lo - 1;
}

__device__ __forceinline__ uint4 load16_guarded(const uint8_t* __restrict__ bytes, uint64_t nbytes, uint64_t pos) {
    uint4 v = make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
    if (pos + 16 <= nbytes && (((uintptr_t)(bytes + pos)) & 15u) == 0) {
        v = *reinterpret_cast<const uint4*>(bytes + pos);
    } else {
        uint32_t w[4] = {0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u};
        for (int i = 0; i < 16; ++i) {
            uint64_t p = pos + i;
            if (p < nbytes) {
                uint32_t sh = 8 * (i & 3);
                w[i >> 2] = (w[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)bytes[p] << sh);
            }
        }
        v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return v;
}

}  // namespace

/* ----------------------------------------------------------------- K0 ----- */

/* Also lists the documents longer than DENSE_DOC (each registered once, by the first grid
 * point inside it): their partial records are summed in a dense per-document array by
 * the merge stage instead of being sorted (finalize.hip, k_part_dense). */
__global__ void k_plan_chunks(CorpusDev c, uint64_t nchunks, uint32_t cb, uint64_t* __restrict__ chunk_start,
                              uint32_t* __restrict__ chunk_doc, uint32_t* __restrict__ big_list,
                              unsigned long long* __restrict__ big_ctr) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > nchunks) return;
    uint64_t b = c.lo + i * (uint64_t)cb;
    if (i == nchunks || b >= c.hi) {
        chunk_start[i] = c.hi;
        chunk_doc[i] = c.ndocs ? c.ndocs - 1 : 0;
        return;
    }
    uint32_t d = doc_containing(c.doc_off, 0, c.ndocs + 1, b); /* doc_off[d] <= b < doc_off[d+1] */
    uint64_t s0 = c.doc_off[d], s1 = c.doc_off[d + 1];
    chunk_start[i] = (s1 - s0 <= BIG_DOC) ? s0 : b;
    chunk_doc[i] = d;
    if (big_list && s1 - s0 > DENSE_DOC && (i == 0 || b - cb < s0)) {
        const unsigned long long k = atomicAdd(big_ctr, 1ull);
        if (k < BIG_LIST_CAP) big_list[k] = d;
    }
}

int launch_plan_chunks(const CorpusDev& c, uint64_t nchunks, uint32_t chunk_bytes, uint64_t* chunk_start,
                       uint32_t* chunk_doc, uint32_t* big_list, unsigned long long* big_ctr, hipStream_t s) {
    uint64_t n = nchunks + 1;
    k_plan_chunks<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(c, nchunks, chunk_bytes, chunk_start, chunk_doc, big_list,
                                                              big_ctr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* ----------------------------------------------------------------- K1 ----- */

struct K1Shared {
    uint8_t bytes[WIN + LOOK + 32];     /* staged window (16-B aligned) */
    uint32_t tok[MAXTOK];               /* (offset << 16) | length */
    ulonglong2 key[TBL];                /* {lo, hi}: one 128-bit LDS write publishes a key */
    uint32_t tdoc[TBL];
    uint32_t tcnt[TBL];
    uint16_t ws[NGRP];                  /* whitespace mask per group */
    uint16_t stop[NGRP];                /* whitespace | document start */
    uint32_t dsbits[(WIN + LOOK) / 32]; /* document starts in the staged range */
    uint16_t wds_start[WDS_CAP];
    uint32_t wds_doc[WDS_CAP];
    uint32_t dsize[FDOCS];              /* tokens per document of the epoch */
    uint32_t dcnt[FDOCS];               /* complete records per document */
    uint32_t doff[FDOCS];
    uint32_t dfill[FDOCS];
    uint8_t dcomplete[FDOCS];
    uint32_t wsum[NT / 64];
    /* block-uniform state */
    uint32_t fill, npart, pfill, ntok_w, nwds, wds_over, cut, carry_next, base_doc_tok;
    uint32_t open_doc, epoch_lo, partial_doc, prev_ws, more;
    unsigned long long rec_base, part_base;
};

__device__ __forceinline__ bool k1_contained(const CorpusDev& c, uint32_t d, uint64_t cs, uint64_t ce) {
    return c.doc_off[d] >= cs && c.doc_off[d + 1] <= ce;
}

/* Emits every table entry as a record and clears the table.  straddle = document that
 * continues after this flush (DOC_NONE for a flush at a document boundary). */
__device__ void k1_flush(K1Shared& S, const CorpusDev& c, const VocabDev& v, const K1Out& o, uint64_t cs,
                         uint64_t ce, uint32_t straddle) {
    const int tid = threadIdx.x;
    __syncthreads();
    const uint32_t elo = S.epoch_lo;
    if (elo != DOC_NONE) {
        /* A0: which documents of the epoch are complete here */
        {
            uint32_t d = elo + tid;
            bool comp = false;
            if (tid < FDOCS && S.dsize[tid] > 0)
                comp = d != straddle && d != S.partial_doc && k1_contained(c, d, cs, ce);
            if (tid < FDOCS) { S.dcomplete[tid] = comp ? 1 : 0; S.dcnt[tid] = 0; S.dfill[tid] = 0; }
        }
        if (tid == 0) { S.npart = 0; S.pfill = 0; }
        __syncthreads();
        /* A: resolve terms to global vocabulary slots, count records */
        for (int s = tid; s < TBL; s += NT) {
            uint32_t d = S.tdoc[s];
            if (d == DOC_NONE) continue;
            uint64_t lo = S.key[s].x, hi = S.key[s].y;
            uint32_t g = (hi == KEY_GSLOT_TAG) ? (uint32_t)lo : vocab_insert(v, lo, hi, 0, o.status);
            S.key[s].x = g;
            uint32_t rel = d - elo;
            if (S.dcomplete[rel]) atomicAdd(&S.dcnt[rel], 1u);
            else atomicAdd(&S.npart, 1u);
        }
        __syncthreads();
        /* B: per-document offsets, one global allocation each for records and partials */
        uint32_t tot;
        uint32_t mine = tid < FDOCS ? S.dcnt[tid] : 0u;
        uint32_t ex = block_excl_scan<NT>(mine, S.wsum, &tot);
        if (tid < FDOCS) S.doff[tid] = ex;
        if (tid == 0) {
            S.rec_base = tot ? atomicAdd(o.rec_alloc, (unsigned long long)tot) : 0ull;
            S.part_base = S.npart ? atomicAdd(o.part_alloc, (unsigned long long)S.npart) : 0ull;
            if (S.rec_base + tot > o.rec_cap) atomicOr(o.status, ST_REC_FULL);
            if (S.part_base + S.npart > o.part_cap) atomicOr(o.status, ST_PART_FULL);
        }
        __syncthreads();
        const unsigned long long rb = S.rec_base, pb = S.part_base;
        const bool rec_ok = rb + tot <= o.rec_cap, part_ok = pb + S.npart <= o.part_cap;
        /* C: write records */
        for (int s = tid; s < TBL; s += NT) {
            uint32_t d = S.tdoc[s];
            if (d == DOC_NONE) continue;
            uint32_t g = (uint32_t)S.key[s].x, cnt = S.tcnt[s], rel = d - elo;
            if (S.dcomplete[rel]) {
                uint64_t pos = rb + S.doff[rel] + atomicAdd(&S.dfill[rel], 1u);
                if (rec_ok) { o.rec_slot[pos] = g; o.rec_cnt[pos] = cnt; }
            } else {
                uint64_t pos = pb + atomicAdd(&S.pfill, 1u);
                if (part_ok) { o.part_doc[pos] = d; o.part_slot[pos] = g; o.part_cnt[pos] = cnt; }
            }
        }
        /* document metadata */
        if (tid < FDOCS && S.dsize[tid] > 0) {
            uint32_t d = elo + tid;
            if (S.dcomplete[tid]) {
                o.doc_recoff[d] = rb + S.doff[tid];
                o.doc_npairs[d] = S.dcnt[tid];
                o.doc_size[d] = S.dsize[tid];
            } else {
                atomicAdd(&o.doc_size[d], S.dsize[tid]);
                o.doc_flags[d] = DF_PARTIAL;
            }
        }
        __syncthreads();
    }
    /* clear */
    for (int s = tid; s < TBL; s += NT) {
        S.tdoc[s] = DOC_NONE;
        S.tcnt[s] = 0;
        S.key[s] = make_ulonglong2(0ull, KEY_EMPTY_HI);
    }
    if (tid < FDOCS) S.dsize[tid] = 0;
    if (tid == 0) {
        S.fill = 0;
        S.epoch_lo = DOC_NONE;
        if (straddle != DOC_NONE) S.partial_doc = straddle;
    }
    __syncthreads();
}

__global__ __launch_bounds__(NT, 2) void k_tokcount(CorpusDev c, const uint64_t* __restrict__ chunk_start,
                                                    const uint32_t* __restrict__ chunk_doc, uint64_t c0,
                                                    VocabDev v, K1Out o) {
    __shared__ __attribute__((aligned(16))) K1Shared S;
    const int tid = threadIdx.x, lane = tid & 63;
    const uint64_t chunk = c0 + blockIdx.x;
    const uint64_t cs = chunk_start[chunk], ce = chunk_start[chunk + 1];
    if (cs >= ce) return;
    const uint64_t wbase0 = cs & ~(uint64_t)15;
    uint32_t carry = chunk_doc[chunk]; /* document containing byte cs */

    for (int s = tid; s < TBL; s += NT) {
        S.tdoc[s] = DOC_NONE; S.tcnt[s] = 0; S.key[s] = make_ulonglong2(0ull, KEY_EMPTY_HI);
    }
    if (tid < FDOCS) S.dsize[tid] = 0;
    if (tid == 0) {
        S.fill = 0; S.epoch_lo = DOC_NONE; S.partial_doc = DOC_NONE; S.open_doc = DOC_NONE;
        /* byte before the first group: whitespace if outside the corpus */
        uint32_t pw = 1;
        if (wbase0 > c.lo && wbase0 - 1 < c.hi && wbase0 - 1 < c.nbytes) pw = is_ws(c.bytes[wbase0 - 1]) ? 1u : 0u;
        S.prev_ws = pw;
    }
    unsigned long long tokens_chunk = 0;

    for (uint64_t wbase = wbase0; wbase < ce; wbase += WIN) {
        const uint64_t win_lo = wbase > cs ? wbase : cs;
        const uint64_t win_hi = (wbase + WIN) < ce ? (wbase + WIN) : ce;
        const uint64_t stage_hi = wbase + WIN + LOOK;
        /* ---- 1. stage + classify ---- */
        uint32_t my_ws = 0;
        for (int g = tid; g < NGRP; g += NT) {
            uint64_t pos = wbase + 16ull * g;
            uint4 val = load16_guarded(c.bytes, c.nbytes, pos);
            *reinterpret_cast<uint4*>(&S.bytes[16 * g]) = val;
            uint32_t m = ws_mask16(val);
            /* bytes outside [lo, hi) belong to no document: whitespace */
            if (pos < c.lo || pos + 16 > c.hi) {
                for (int i = 0; i < 16; ++i) {
                    uint64_t p = pos + i;
                    if (p < c.lo || p >= c.hi) m |= 1u << i;
                }
            }
            S.ws[g] = (uint16_t)m;
            if (g == tid) my_ws = m;
        }
        for (int k = tid; k < (WIN + LOOK) / 32; k += NT) S.dsbits[k] = 0;
        if (tid == 0) { S.nwds = 0; S.wds_over = 0; S.carry_next = carry; }
        __syncthreads();
        /* ---- 2. document starts in [wbase, stage_hi), from the carried document on ---- */
        for (uint32_t d0 = carry;; d0 += NT) {
            uint32_t d = d0 + tid;
            bool valid = d < c.ndocs && c.doc_off[d] < stage_hi;
            uint64_t st = valid ? c.doc_off[d] : 0;
            bool nonempty = valid && c.doc_off[d + 1] > st && st >= wbase;
            uint32_t rel = nonempty ? (uint32_t)(st - wbase) : 0u;
            if (nonempty) atomicOr(&S.dsbits[rel >> 5], 1u << (rel & 31));
            if (nonempty && rel <= (uint32_t)WIN) atomicMax(&S.carry_next, d);
            bool listed = nonempty && rel < (uint32_t)WIN;
            uint32_t tot;
            uint32_t pos = block_excl_scan<NT>(listed ? 1u : 0u, S.wsum, &tot);
            uint32_t base = S.nwds;
            if (listed && base + pos < WDS_CAP) { S.wds_start[base + pos] = (uint16_t)rel; S.wds_doc[base + pos] = d; }
            __syncthreads();
            if (tid == 0) {
                S.nwds = base + tot;
                S.more = (d0 + NT - 1 < c.ndocs && c.doc_off[d0 + NT - 1] < stage_hi) ? 1u : 0u;
            }
            __syncthreads();
            if (!S.more) break;
        }
        if (tid == 0 && S.nwds > WDS_CAP) S.wds_over = 1;
        /* ---- 3. stop masks ---- */
        for (int g = tid; g < NGRP; g += NT) {
            uint32_t dsm = (S.dsbits[g >> 1] >> ((g & 1) * 16)) & 0xFFFFu;
            S.stop[g] = (uint16_t)(S.ws[g] | dsm);
        }
        __syncthreads();
        /* ---- 4. token starts of this lane's group, compaction ---- */
        {
            const int g = tid;
            const uint64_t gpos = wbase + 16ull * g;
            uint32_t ds16 = (S.dsbits[g >> 1] >> ((g & 1) * 16)) & 0xFFFFu;
            uint32_t prevw = g ? ((S.ws[g - 1] >> 15) & 1u) : S.prev_ws;
            uint32_t boundary = (((my_ws << 1) | prevw) | ds16) & 0xFFFFu;
            uint32_t owned = 0;
            if (gpos + 16 > win_lo && gpos < win_hi) {
                uint32_t a = gpos < win_lo ? (uint32_t)(win_lo - gpos) : 0u;
                uint32_t b = gpos + 16 > win_hi ? (uint32_t)(win_hi - gpos) : 16u;
                owned = ((1u << b) - 1u) & ~((1u << a) - 1u);
            }
            uint32_t starts = ~my_ws & boundary & owned & 0xFFFFu;
            uint32_t tot;
            uint32_t off = block_excl_scan<NT>((uint32_t)__popc(starts), S.wsum, &tot);
            const uint32_t stop16 = S.stop[g];
            while (starts) {
                uint32_t i = __builtin_ctz(starts);
                starts &= starts - 1;
                uint32_t len = LEN_OPEN;
                uint32_t m = (stop16 >> (i + 1)) & 0xFFFFu;
                if (m) {
                    len = __builtin_ctz(m) + 1;
                } else {
                    for (int gg = g + 1; gg < NGRP; ++gg) {
                        uint32_t sm = S.stop[gg];
                        if (sm) { len = 16u * (gg - g) + __builtin_ctz(sm) - i; break; }
                    }
                }
                S.tok[off++] = ((16u * g + i) << 16) | (len > 0xFFFEu ? LEN_OPEN : len);
            }
            if (tid == 0) S.ntok_w = tot;
        }
        __syncthreads();
        const uint32_t ntok_w = S.ntok_w;
        tokens_chunk += ntok_w;
        const uint32_t nwds = S.nwds < WDS_CAP ? S.nwds : WDS_CAP;
        const bool wds_over = S.wds_over != 0;
        /* ---- 5. count tokens in batches ---- */
        uint32_t base = 0;
        while (base < ntok_w) {
            const uint32_t i = base + tid;
            const bool has = i < ntok_w;
            uint32_t rel = 0, len = 0, d = DOC_NONE;
            if (has) {
                uint32_t tw = S.tok[i];
                rel = tw >> 16;
                len = tw & 0xFFFFu;
                if (!wds_over) {
                    uint32_t lo = 0, hi = nwds;
                    while (lo < hi) {
                        uint32_t mid = (lo + hi) >> 1;
                        if (S.wds_start[mid] <= rel) lo = mid + 1; else hi = mid;
                    }
                    d = lo ? S.wds_doc[lo - 1] : carry;
                } else {
                    d = doc_containing(c.doc_off, carry, c.ndocs + 1, wbase + rel);
                }
            }
            if (tid == 0) {
                S.cut = 0xFFFFFFFFu;
                if (S.epoch_lo == DOC_NONE) S.epoch_lo = d; /* thread 0 holds token `base` */
                S.base_doc_tok = d;
            }
            __syncthreads();
            /* Block-uniform decisions use values captured here, between two barriers with
             * no writers: the insert phase below updates fill/open_doc while slower waves
             * could still be deciding. */
            const uint32_t elo = S.epoch_lo, fill0 = S.fill, open0 = S.open_doc, dbase = S.base_doc_tok;
            /* cut the batch at the first token whose document must start a new epoch */
            {
                uint32_t cut_doc = elo + FDOCS;
                if (fill0 > (uint32_t)FLUSH_THR && open0 != DOC_NONE && open0 + 1 < cut_doc) cut_doc = open0 + 1;
                bool f = has && d >= cut_doc;
                uint64_t bm = __ballot(f);
                if (bm && lane == (int)__builtin_ctzll(bm)) atomicMin(&S.cut, i);
            }
            __syncthreads();
            uint32_t end = base + NT < ntok_w ? base + NT : ntok_w;
            const uint32_t cut = S.cut;
            if (cut < end) end = cut;
            if (end == base) { /* document boundary at `base`: flush the epoch cleanly */
                k1_flush(S, c, v, o, cs, ce, DOC_NONE);
                continue;
            }
            if (fill0 + (end - base) > (uint32_t)TBL_HARD) {
                /* cannot fit: flush now; the open document straddles iff it continues at base */
                k1_flush(S, c, v, o, cs, ce, (open0 == dbase) ? dbase : DOC_NONE);
                continue;
            }
            /* ---- insert tokens [base, end) ---- */
            if (i < end) {
                uint64_t klo = 0, khi = 0;
                bool is_long = (len == LEN_OPEN);
                if (!is_long) {
                    const uint32_t a = rel & ~7u;
                    const uint64_t* q = reinterpret_cast<const uint64_t*>(&S.bytes[a]);
                    uint64_t w0 = q[0], w1 = q[1], w2 = q[2];
                    uint32_t sh = (rel & 7u) * 8u;
                    uint64_t lo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
                    uint64_t hi = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
                    uint32_t n = make_short_key(lo, hi, len, &klo, &khi);
                    is_long = n >= 16u;
                }
                if (is_long) {
                    /* slow path (rare): term >= 16 bytes, hashed from global memory and
                     * resolved to its global slot right away */
                    uint64_t p0 = wbase + rel;
                    uint64_t dend = c.doc_off[d + 1];
                    uint64_t p = p0;
                    while (p < dend && p < c.nbytes && !is_ws(c.bytes[p])) ++p;
                    uint64_t tlen = p - p0, n = 0;
                    while (n < tlen && c.bytes[p0 + n] != 0) ++n;
                    if (n < 16) { /* NUL-truncated to a short term */
                        uint64_t lo = 0, hi = 0;
                        for (uint32_t k = 0; k < n; ++k) {
                            uint64_t b = c.bytes[p0 + k];
                            if (k < 8) lo |= b << (8 * k); else hi |= b << (8 * (k - 8));
                        }
                        make_short_key(lo, hi, (uint32_t)n, &klo, &khi);
                    } else {
                        make_long_key(c.bytes + p0, n, &klo, &khi);
                        if (n >= 0xFFFFFFull) atomicOr(o.status, ST_TERM_LONG); /* rep holds 24 length bits */
                        uint64_t rep = ((n < 0xFFFFFFull ? n : 0xFFFFFFull) << 40) | p0;
                        uint32_t g = vocab_insert(v, klo, khi, rep, o.status, c.bytes);
                        klo = g;
                        khi = KEY_GSLOT_TAG;
                    }
                }
                /* LDS (doc, key) table */
                uint32_t h = (uint32_t)key_hash(klo ^ ((uint64_t)d * 0x9E3779B97F4A7C15ull), khi) & (TBL - 1);
                /* claim-once slots, keys published by one 128-bit LDS write; a reader sees
                 * the EMPTY sentinel (retry) or the final key (see tokcount_ws.hip) */
                for (uint32_t guard = 0;; ++guard) {
                    if (guard > (1u << 16)) { atomicOr(o.status, ST_VOCAB_SPIN); break; }
                    asm volatile("" ::: "memory");
                    uint32_t td = S.tdoc[h];
                    if (td == DOC_NONE) {
                        uint32_t old = atomicCAS(&S.tdoc[h], DOC_NONE, d);
                        if (old == DOC_NONE) {
                            S.key[h] = make_ulonglong2(klo, khi);
                            atomicAdd(&S.tcnt[h], 1u);
                            atomicAdd(&S.fill, 1u);
                            break;
                        }
                        td = old;
                    }
                    if (td == d) {
                        const ulonglong2 kk = S.key[h];
                        if (kk.y == KEY_EMPTY_HI) { __builtin_amdgcn_s_sleep(1); continue; }
                        if (kk.y == khi && kk.x == klo) { atomicAdd(&S.tcnt[h], 1u); break; }
                    }
                    h = (h + 1) & (TBL - 1);
                }
                atomicAdd(&S.dsize[d - S.epoch_lo], 1u);
            }
            if (i + 1 == end) S.open_doc = d;
            __syncthreads();
            base = end;
        }
        /* ---- carry state to the next window ---- */
        __syncthreads();
        if (tid == 0) S.prev_ws = (S.ws[NT - 1] >> 15) & 1u;
        carry = S.carry_next;
        __syncthreads();
    }
    k1_flush(S, c, v, o, cs, ce, DOC_NONE);
    if (tid == 0) atomicAdd(o.ntokens, tokens_chunk);
}

int launch_tokcount(const CorpusDev& c, const uint64_t* chunk_start, const uint32_t* chunk_doc, uint64_t c0,
                    uint64_t c1, const VocabDev& v, const K1Out& o, hipStream_t s) {
    if (c1 <= c0) return 0;
    k_tokcount<<<(unsigned)(c1 - c0), NT, 0, s>>>(c, chunk_start, chunk_doc, c0, v, o);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
