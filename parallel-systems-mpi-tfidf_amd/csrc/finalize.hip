/*
 * finalize.hip — everything after K1 (tokenize + count):
 *
 *   vocabulary   compact the HBM hash table, radix-sort the strcmp("word\t") keys,
 *                rank_of_slot / slot_of_rank                 (replaces TFIDF.c:227-234 joins)
 *   partials     documents split across flushes/chunks: radix sort on (doc, rank) and
 *                reduce-by-key into presorted record runs     (TFIDF.c:151-167 semantics)
 *   DF           histogram of records per term rank: #documents containing the term
 *                (TFIDF.c:169-188 + CustomReduce TFIDF.c:291-319)
 *   order+score  documents in "docN@" strcmp order (base-11 keys), terms by rank inside a
 *                document (LDS bitonic sort), tf = wc/ds, score = tf * idf   (TFIDF.c:202,
 *                243-245,273)
 *   multi-GPU    identity-key union + dense DF vector for the RCCL all-reduce
 *   synthetic    device-side corpus generation (csrc/synth.h)
 */
#include "dev_common.h"
#include "dev_vocab.h"
#include "kernels.h"
#include "synth.h"

#include <type_traits>
/* global (address space 1) view of a pointer: K5Args travels by reference into helpers, so
 * its pointers reach loads as generic (flat) pointers, whose loads also count in lgkmcnt and
 * make every LDS wait wait for them too */
#define G(p) ((GLOBAL_AS std::remove_pointer_t<decltype(p)>*)(p))
/* K5's outputs: plain stores.  Non-temporal ones measured c2's score stage 0.753 -> 0.727
 * ms but c4's 3.05 -> 4.1 ms, non-temporal record loads no change on either
 * (profiles/r03_nt_emit_ab.txt) */
template <class T> __device__ __forceinline__ void sto(T* p, T v) { *(GLOBAL_AS T*)p = v; }

namespace {
constexpr int NT = 256;
/* at least one workgroup: an empty launch is an error, every kernel bounds-checks its index */
inline unsigned grid_for(uint64_t n, int nt = NT) { return n ? (unsigned)((n + nt - 1) / nt) : 1u; }
inline int ok() { return hipGetLastError() == hipSuccess ? 0 : -1; }

__device__ __forceinline__ uint4 u128_from(uint64_t lo, uint64_t hi) {
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
__device__ __forceinline__ bool u128_eq(uint4 a, uint4 b) { return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w; }
}  // namespace

/* ------------------------------------------------------------ vocabulary -- */

__global__ void k_vocab_flags(VocabDev v, uint64_t cap, uint32_t* __restrict__ flags) {
    uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap) return;
    uint4 k = v.keys[s];
    uint64_t hi = ((uint64_t)k.w << 32) | k.z;
    flags[s] = (hi != KEY_EMPTY_HI && hi != KEY_PENDING_HI) ? 1u : 0u;
}
int launch_vocab_flags(const VocabDev& v, uint64_t cap, uint32_t* flags, hipStream_t s) {
    k_vocab_flags<<<grid_for(cap), NT, 0, s>>>(v, cap, flags);
    return ok();
}

/* sort key = the term's bytes big-endian: short terms "w\t0..", long terms their first 16 bytes */
__global__ void k_vocab_compact(VocabDev v, uint64_t cap, const uint32_t* __restrict__ dense_of_slot, CorpusDev c,
                                uint32_t* __restrict__ vslot, uint4* __restrict__ sortkey, uint32_t* __restrict__ seq) {
    uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap) return;
    uint32_t dn = dense_of_slot[s];
    if (dense_of_slot[s + 1] == dn) return; /* empty slot */
    uint4 k = v.keys[s];
    uint64_t lo = ((uint64_t)k.y << 32) | k.x, hi = ((uint64_t)k.w << 32) | k.z;
    uint64_t skhi, sklo;
    if ((hi >> 56) == 0xFFu) {
        uint64_t rep = v.rep[s], off = rep & 0xFFFFFFFFFFull;
        uint64_t a = 0, b = 0;
        for (int i = 0; i < 8; ++i) a = (a << 8) | c.bytes[off + i];
        for (int i = 8; i < 16; ++i) b = (b << 8) | c.bytes[off + i];
        skhi = a; sklo = b;
    } else {
        skhi = bswap64(lo);
        sklo = bswap64(hi);
    }
    vslot[dn] = (uint32_t)s;
    sortkey[dn] = u128_from(sklo, skhi);
    seq[dn] = dn;
}
int launch_vocab_compact(const VocabDev& v, uint64_t cap, const uint32_t* dense_of_slot, const CorpusDev& c,
                         uint32_t* vslot, uint4* sortkey, uint32_t* seq, hipStream_t s) {
    k_vocab_compact<<<grid_for(cap), NT, 0, s>>>(v, cap, dense_of_slot, c, vslot, sortkey, seq);
    return ok();
}

__global__ void k_vocab_rank(const uint32_t* __restrict__ sorted_dense, const uint32_t* __restrict__ vslot, uint32_t V,
                             uint32_t* __restrict__ rank_of_slot, uint32_t* __restrict__ slot_of_rank,
                             uint16_t* __restrict__ rank16) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= V) return;
    uint32_t s = vslot[sorted_dense[r]];
    rank_of_slot[s] = r;
    slot_of_rank[r] = s;
    if (rank16) rank16[s] = (uint16_t)r;
}

/* The vocabulary sort of large V as two u64 LSD sorts (the low 8 bytes of the 16-byte
 * strcmp keys, then, stable, the high 8 in that order): every digit pass moves 12-byte
 * (key half, id) pairs instead of 20-byte (key, id) pairs, for one 8-byte gather of the
 * high halves between the two sorts.  out[i] = half of k[seq ? seq[i] : i]. */
__global__ void k_sortkey_half(const uint4* __restrict__ k, uint64_t n, const uint32_t* __restrict__ seq, int hi,
                               uint64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 x = k[seq ? seq[i] : i];
    out[i] = hi ? (((uint64_t)x.w << 32) | x.z) : (((uint64_t)x.y << 32) | x.x);
}
int launch_sortkey_half(const uint4* k, uint64_t n, const uint32_t* seq, int hi, uint64_t* out, hipStream_t s) {
    if (!n) return 0;
    k_sortkey_half<<<grid_for(n), NT, 0, s>>>(k, n, seq, hi, out);
    return ok();
}
__global__ void k_gather_u128(const uint4* __restrict__ k, const uint32_t* __restrict__ seq, uint64_t n,
                              uint4* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = k[seq[i]];
}
/* one grid-stride pass over all segments' 16-byte blocks (off: their prefix counts, in
 * 16-byte units), then each segment's tail bytes */
struct FillRun {
    FillList l;
    uint64_t off[FILL_MAX + 1];
};
__global__ void k_fill_multi(const FillRun f) {
    const uint64_t total = f.off[f.l.n];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        uint32_t g = 0;
        while (i >= f.off[g + 1]) ++g;
        const uint32_t v = f.l.val[g];
        reinterpret_cast<uint4*>(f.l.p[g])[i - f.off[g]] = make_uint4(v, v, v, v);
    }
    if (blockIdx.x == 0 && threadIdx.x < 16u * f.l.n) {
        const uint32_t g = threadIdx.x / 16u, t = threadIdx.x % 16u;
        const uint64_t nb = f.l.bytes[g];
        if (t < (nb & 15u)) ((uint8_t*)f.l.p[g])[(nb & ~15ull) + t] = (uint8_t)f.l.val[g];
    }
}
int launch_fill_multi(const FillList& l, hipStream_t s) {
    if (l.n == 0) return 0;
    if (l.n > (uint32_t)FILL_MAX) return -3;
    FillRun f;
    f.l = l;
    f.off[0] = 0;
    for (uint32_t g = 0; g < l.n; ++g) {
        if (((uintptr_t)l.p[g] & 15u) != 0) return -3;
        f.off[g + 1] = f.off[g] + l.bytes[g] / 16;
    }
    uint64_t nbx = (f.off[l.n] + NT - 1) / NT;
    if (nbx < 1) nbx = 1;
    if (nbx > 2048) nbx = 2048;
    k_fill_multi<<<(unsigned)nbx, NT, 0, s>>>(f);
    return ok();
}

/* dst[i] = the i-th word, zero-extended; dst is pinned host memory (visible to the host
 * after the stream synchronises) */
__global__ void k_words_to_host(const WordList l, uint64_t* dst) {
    const uint32_t i = threadIdx.x;
    if (i < l.n)
        *(volatile uint64_t*)&dst[i] =
            l.bytes[i] == 8 ? *(const volatile uint64_t*)l.src[i] : (uint64_t) * (const volatile uint32_t*)l.src[i];
    if (l.token) {
        __threadfence_system();   /* every lane's word reaches the host before the token */
        __syncthreads();
        if (i == 0) {
            __threadfence_system();
            *(volatile uint64_t*)&dst[l.n] = l.token;
        }
    }
}
int launch_words_to_host(const WordList& l, uint64_t* host_dst, hipStream_t s) {
    if (l.n == 0) return 0;
    if (l.n > (uint32_t)WORDS_MAX) return -3;
    k_words_to_host<<<1, 64, 0, s>>>(l, host_dst);
    return ok();
}

int launch_gather_u128(const uint4* k, const uint32_t* seq, uint64_t n, uint4* out, hipStream_t s) {
    if (!n) return 0;
    k_gather_u128<<<grid_for(n), NT, 0, s>>>(k, seq, n, out);
    return ok();
}
int launch_vocab_rank(const uint32_t* sorted_dense, const uint32_t* vslot, uint32_t V, uint32_t* rank_of_slot,
                      uint32_t* slot_of_rank, uint16_t* rank16, hipStream_t s) {
    k_vocab_rank<<<grid_for(V), NT, 0, s>>>(sorted_dense, vslot, V, rank_of_slot, slot_of_rank, rank16);
    return ok();
}

/* long terms sharing their first 16 bytes: order the tie run by full byte compare
 * (strcmp of "w\t": a word sorts before its extensions unless the next byte < 0x09) */
__device__ int long_cmp(const CorpusDev& c, uint64_t ra, uint64_t rb) {
    uint64_t oa = ra & 0xFFFFFFFFFFull, la = ra >> 40, ob = rb & 0xFFFFFFFFFFull, lb = rb >> 40;
    uint64_t n = la < lb ? la : lb;
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t x = c.bytes[oa + i], y = c.bytes[ob + i];
        if (x != y) return x < y ? -1 : 1;
    }
    if (la == lb) return 0;
    uint32_t nx = la < lb ? 0x09u : c.bytes[oa + n];
    uint32_t ny = la < lb ? c.bytes[ob + n] : 0x09u;
    return nx < ny ? -1 : 1;
}
__global__ void k_vocab_long_fixup(const uint4* __restrict__ sk, uint32_t* __restrict__ sorted_dense,
                                   const uint32_t* __restrict__ vslot, VocabDev v, CorpusDev c, uint32_t V) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i + 1 >= V) return;
    bool head = (i == 0 || !u128_eq(sk[i], sk[i - 1])) && u128_eq(sk[i], sk[i + 1]);
    if (!head) return;
    uint32_t e = i + 1;
    while (e < V && u128_eq(sk[e], sk[i])) ++e;
    for (uint32_t a = i + 1; a < e; ++a) { /* insertion sort of the tie run */
        uint32_t x = sorted_dense[a];
        uint64_t rx = v.rep[vslot[x]];
        uint32_t b = a;
        while (b > i && long_cmp(c, v.rep[vslot[sorted_dense[b - 1]]], rx) > 0) {
            sorted_dense[b] = sorted_dense[b - 1];
            --b;
        }
        sorted_dense[b] = x;
    }
}
/* ---- long terms sharing their first 16 bytes, in parallel ----
 * The vocabulary sort orders long terms by their first 16 bytes only.  Ties (URLs, paths,
 * identifiers with a common prefix: runs of 1e5+ terms are possible) are resolved by
 * iterated re-keying, each round a segmented sort on the next 16 bytes:
 *   h[i]   = 1 where sorted position i starts a group of equal keys so far (h[V] = 1);
 *   round k: the positions in groups of two or more are compacted (pos[]), each gets
 *   key = bytes [16k, 16k + 16) of its term ("w\t" then zeros: strcmp of "w\t",
 *   TFIDF.c:49,245) and seg = its group ordinal; a stable LSD sort by key, then by seg,
 *   reorders every group in place (groups are contiguous in both orders), and new group
 *   starts are set where (seg, key) changes.
 * The loop ends when no group of two or more is left: ceil(common prefix / 16) rounds.
 * After VLF_MAX_ROUNDS (a 16 KiB common prefix) the single-thread insertion sort above
 * finishes whatever is left. */
constexpr uint32_t VLF_MAX_ROUNDS = 1024;

__global__ void k_vlf_heads(const uint4* __restrict__ sk, uint32_t V, uint32_t* __restrict__ h) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > V) return;
    h[i] = (i == 0 || i == V || !u128_eq(sk[i], sk[i - 1])) ? 1u : 0u;
}
/* tied[i]: position i is in a group of two or more */
__global__ void k_vlf_tied(const uint32_t* __restrict__ h, uint32_t V, uint32_t* __restrict__ tied) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < V) tied[i] = (h[i] && h[i + 1]) ? 0u : 1u;
}
__device__ __forceinline__ uint4 vlf_key(const CorpusDev& c, uint64_t rep, uint64_t k) {
    const uint64_t off = rep & 0xFFFFFFFFFFull, len = rep >> 40;
    uint64_t a = 0, b = 0;
    for (int t = 0; t < 16; ++t) {
        const uint64_t p = 16 * k + (uint64_t)t;
        const uint64_t x = p < len ? c.bytes[off + p] : (p == len ? 0x09u : 0u);
        if (t < 8) a = (a << 8) | x; else b = (b << 8) | x;
    }
    return u128_from(b, a);
}
__global__ void k_vlf_keys(const uint32_t* __restrict__ tied_scan, const uint32_t* __restrict__ hscan,
                           const uint32_t* __restrict__ h, const uint32_t* __restrict__ sorted_dense,
                           const uint32_t* __restrict__ vslot, VocabDev v, CorpusDev c, uint32_t V, uint64_t k,
                           uint32_t* __restrict__ pos, uint4* __restrict__ key, uint4* __restrict__ key_orig,
                           uint32_t* __restrict__ val, uint64_t* __restrict__ seg, uint32_t* __restrict__ dense_copy) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= V || tied_scan[i + 1] == tied_scan[i]) return;
    const uint32_t j = tied_scan[i];
    const uint32_t d = sorted_dense[i];
    const uint4 kk = vlf_key(c, v.rep[vslot[d]], k);
    pos[j] = i;
    key[j] = kk;
    key_orig[j] = kk;
    val[j] = j;
    seg[j] = hscan[i] + h[i];   /* group ordinal (inclusive count of group starts) */
    dense_copy[j] = d;
}
/* item j of the (key, seg)-sorted order came from compacted index o = vals[j] */
__global__ void k_vlf_seg_of(const uint32_t* __restrict__ vals, const uint64_t* __restrict__ seg, uint32_t m,
                             uint64_t* __restrict__ seg_sorted) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) seg_sorted[j] = seg[vals[j]];
}
__global__ void k_vlf_apply(const uint32_t* __restrict__ final_idx, uint32_t m, const uint32_t* __restrict__ pos,
                            const uint32_t* __restrict__ dense_copy, const uint64_t* __restrict__ seg,
                            const uint4* __restrict__ key_orig, uint32_t* __restrict__ sorted_dense,
                            uint32_t* __restrict__ h) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint32_t o = final_idx[j], i = pos[j];
    sorted_dense[i] = dense_copy[o];
    bool head = j == 0;
    if (!head) {
        const uint32_t p = final_idx[j - 1];
        head = seg[o] != seg[p] || !u128_eq(key_orig[o], key_orig[p]);
    }
    h[i] = head ? 1u : 0u;
}

int launch_vocab_long_fixup(const uint4* sorted_keys, uint32_t* sorted_dense, const uint32_t* vslot,
                            const VocabDev& v, const CorpusDev& c, uint32_t V, Arena& ar, hipStream_t s) {
    if (V < 2) return 0;
    const size_t m0 = ar.mark();
    uint32_t* h = (uint32_t*)ar.get(((size_t)V + 1) * 4);
    uint32_t* hs = (uint32_t*)ar.get(((size_t)V + 2) * 4);
    uint32_t* ts = (uint32_t*)ar.get(((size_t)V + 2) * 4);
    if (!h || !hs || !ts) return -2;
    k_vlf_heads<<<grid_for((uint64_t)V + 1), NT, 0, s>>>(sorted_keys, V, h);
    uint32_t round = 1;
    for (; round <= VLF_MAX_ROUNDS; ++round) {
        k_vlf_tied<<<grid_for(V), NT, 0, s>>>(h, V, ts);
        if (scan_excl_u32(ts, ts, V, ar, s)) return -2;
        uint32_t m = 0;
        if (hipMemcpyAsync(&m, ts + V, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
        if (hipStreamSynchronize(s) != hipSuccess) return -1;
        if (m == 0) break;
        if (scan_excl_u32(h, hs, V, ar, s)) return -2;
        const size_t mr = ar.mark();
        uint32_t* pos = (uint32_t*)ar.get((size_t)m * 4);
        uint4* k0 = (uint4*)ar.get((size_t)m * 16);
        uint4* k1 = (uint4*)ar.get((size_t)m * 16);
        uint4* ko = (uint4*)ar.get((size_t)m * 16);
        uint32_t* v0 = (uint32_t*)ar.get((size_t)m * 4);
        uint32_t* v1 = (uint32_t*)ar.get((size_t)m * 4);
        uint64_t* sg = (uint64_t*)ar.get((size_t)m * 8);
        uint64_t* s0 = (uint64_t*)ar.get((size_t)m * 8);
        uint64_t* s1 = (uint64_t*)ar.get((size_t)m * 8);
        uint32_t* dc = (uint32_t*)ar.get((size_t)m * 4);
        if (!pos || !k0 || !k1 || !ko || !v0 || !v1 || !sg || !s0 || !s1 || !dc) return -2;
        k_vlf_keys<<<grid_for(V), NT, 0, s>>>(ts, hs, h, sorted_dense, vslot, v, c, V, round, pos, k0, ko, v0, sg, dc);
        uint32_t vm = 0;
        if (key_varying_bytes_u128(k0, m, &vm, ar, s)) return -2;
        int cur = radix_sort_u128(k0, v0, k1, v1, m, vm, ar, s);
        if (cur < 0) return cur;
        uint32_t* vk = cur ? v1 : v0;
        uint32_t* vo = cur ? v0 : v1;
        k_vlf_seg_of<<<grid_for(m), NT, 0, s>>>(vk, sg, m, s0);
        /* groups are < 2^32 and numbered in position order: a stable sort on seg */
        const uint32_t segbytes = 0x0Fu;
        int cs = radix_sort_u64(s0, vk, s1, vo, m, segbytes, ar, s);
        if (cs < 0) return cs;
        const uint32_t* fin = cs ? vo : vk;
        k_vlf_apply<<<grid_for(m), NT, 0, s>>>(fin, m, pos, dc, sg, ko, sorted_dense, h);
        if (ok()) return -1;
        ar.release(mr);
    }
    if (round > VLF_MAX_ROUNDS)   /* absurdly long shared prefixes: finish serially */
        k_vocab_long_fixup<<<grid_for(V), NT, 0, s>>>(sorted_keys, sorted_dense, vslot, v, c, V);
    ar.release(m0);
    return ok();
}

/* ---- large-V vocabulary sort, prefix first: the keys sorted by their first 8 bytes
 * (the high halves) only; positions whose high half equals a neighbour's are "tied" and
 * re-ordered by their low halves within each run of equal prefixes.  Tied positions are
 * numbered in position order and the (run, low half)-sorted tied items are written back
 * to them in that order, so item j of the sorted list lands at the j-th tied position.
 * Most terms differ in their first 8 bytes (c4: 9.75 M terms, 13 radix passes -> 8 + a
 * fix-up of the few tied ones). */
__global__ void k_pt_flags(const uint64_t* __restrict__ hi, uint32_t V, uint32_t* __restrict__ tied,
                           uint32_t* __restrict__ head) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= V) return;
    const bool prev = i > 0 && hi[i] == hi[i - 1];
    const bool next = i + 1 < V && hi[i] == hi[i + 1];
    tied[i] = (prev || next) ? 1u : 0u;
    head[i] = (!prev && next) ? 1u : 0u;
}
__global__ void k_pt_collect(const uint32_t* __restrict__ tied_scan, const uint32_t* __restrict__ head_scan,
                             const uint32_t* __restrict__ head, const uint32_t* __restrict__ sorted_dense,
                             const uint4* __restrict__ skey, uint32_t V, uint32_t* __restrict__ pos,
                             uint64_t* __restrict__ klow, uint32_t* __restrict__ val, uint64_t* __restrict__ seg,
                             uint32_t* __restrict__ dense_copy) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= V || tied_scan[i + 1] == tied_scan[i]) return;
    const uint32_t j = tied_scan[i];
    const uint32_t d = sorted_dense[i];
    const uint4 k = skey[d];
    pos[j] = i;
    klow[j] = ((uint64_t)k.y << 32) | k.x;
    val[j] = j;
    seg[j] = head_scan[i] + head[i];   /* run ordinal (inclusive count of run heads) */
    dense_copy[j] = d;
}
__global__ void k_pt_apply(const uint32_t* __restrict__ final_idx, uint32_t m, const uint32_t* __restrict__ pos,
                           const uint32_t* __restrict__ dense_copy, uint32_t* __restrict__ sorted_dense) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) sorted_dense[pos[j]] = dense_copy[final_idx[j]];
}

int launch_vocab_prefix_ties(const uint64_t* sorted_hi, uint32_t* sorted_dense, const uint4* skey, uint32_t V,
                             uint32_t low_mask, Arena& ar, hipStream_t s) {
    if (V < 2 || !low_mask) return 0;
    const size_t m0 = ar.mark();
    uint32_t* tied = (uint32_t*)ar.get(((size_t)V + 2) * 4);
    uint32_t* head = (uint32_t*)ar.get(((size_t)V + 2) * 4);
    uint32_t* ts = (uint32_t*)ar.get(((size_t)V + 2) * 4);
    uint32_t* hs = (uint32_t*)ar.get(((size_t)V + 2) * 4);
    if (!tied || !head || !ts || !hs) return -2;
    k_pt_flags<<<grid_for(V), NT, 0, s>>>(sorted_hi, V, tied, head);
    if (scan_excl_u32(tied, ts, V, ar, s)) return -2;
    uint32_t m = 0;
    if (hipMemcpyAsync(&m, ts + V, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    if (m) {
        if (scan_excl_u32(head, hs, V, ar, s)) return -2;
        uint32_t* pos = (uint32_t*)ar.get((size_t)m * 4);
        uint64_t* k0 = (uint64_t*)ar.get((size_t)m * 8);
        uint64_t* k1 = (uint64_t*)ar.get((size_t)m * 8);
        uint32_t* v0 = (uint32_t*)ar.get((size_t)m * 4);
        uint32_t* v1 = (uint32_t*)ar.get((size_t)m * 4);
        uint64_t* sg = (uint64_t*)ar.get((size_t)m * 8);
        uint64_t* s0 = (uint64_t*)ar.get((size_t)m * 8);
        uint64_t* s1 = (uint64_t*)ar.get((size_t)m * 8);
        uint32_t* dc = (uint32_t*)ar.get((size_t)m * 4);
        if (!pos || !k0 || !k1 || !v0 || !v1 || !sg || !s0 || !s1 || !dc) return -2;
        k_pt_collect<<<grid_for(V), NT, 0, s>>>(ts, hs, head, sorted_dense, skey, V, pos, k0, v0, sg, dc);
        const int cur = radix_sort_u64(k0, v0, k1, v1, m, low_mask, ar, s);
        if (cur < 0) return cur;
        uint32_t* vk = cur ? v1 : v0;
        uint32_t* vo = cur ? v0 : v1;
        k_vlf_seg_of<<<grid_for(m), NT, 0, s>>>(vk, sg, m, s0);
        const int cs = radix_sort_u64(s0, vk, s1, vo, m, 0x0Fu, ar, s);   /* stable on the run ordinal */
        if (cs < 0) return cs;
        k_pt_apply<<<grid_for(m), NT, 0, s>>>(cs ? vo : vk, m, pos, dc, sorted_dense);
    }
    ar.release(m0);
    return ok();
}

/* -------------------------------------------------------------- partials -- */

__global__ void k_part_keys(const uint32_t* __restrict__ pdoc, const uint32_t* __restrict__ pslot,
                            const uint32_t* __restrict__ rank_of_slot, uint64_t n, uint64_t* __restrict__ keys,
                            uint32_t* __restrict__ seq) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = ((uint64_t)pdoc[i] << 32) | rank_of_slot[pslot[i]];
    seq[i] = (uint32_t)i;
}
int launch_part_keys(const uint32_t* part_doc, const uint32_t* part_slot, const uint32_t* rank_of_slot, uint64_t n,
                     uint64_t* keys, uint32_t* seq, hipStream_t s) {
    if (!n) return 0;
    k_part_keys<<<grid_for(n), NT, 0, s>>>(part_doc, part_slot, rank_of_slot, n, keys, seq);
    return ok();
}

__global__ void k_part_heads(const uint64_t* __restrict__ keys, uint64_t n, uint32_t* __restrict__ head) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}
int launch_part_heads(const uint64_t* keys, uint64_t n, uint32_t* head, hipStream_t s) {
    if (!n) return 0;
    k_part_heads<<<grid_for(n), NT, 0, s>>>(keys, n, head);
    return ok();
}

/* One merged record per (doc, rank) run of the sorted partial records.  Runs can be
 * thousands of records long (a term of a 100 MB document appears in each of its ~6000
 * chunks), so the counts are not summed by the run's head thread: every record adds its
 * count after a wave-level segmented reduction (runs are contiguous, so lanes of one run
 * are adjacent), one device atomic per run and wave into the zeroed rec_cnt. */
__global__ void k_part_merge(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ seq,
                             const uint32_t* __restrict__ pcnt, const uint32_t* __restrict__ head_pos, uint64_t n,
                             const uint32_t* __restrict__ slot_of_rank, uint64_t rec_base,
                             uint32_t* __restrict__ rec_slot, uint32_t* __restrict__ rec_cnt,
                             uint64_t* __restrict__ doc_recoff, uint8_t* __restrict__ doc_flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool val = i < n;
    const uint64_t k = val ? keys[i] : ~0ull;
    const uint64_t kp = (val && i > 0) ? keys[i - 1] : ~0ull;
    const bool head = val && (i == 0 || kp != k);
    const uint64_t u = val ? rec_base + head_pos[i] - (head ? 0u : 1u) : ~0ull;
    uint32_t v = val ? pcnt[seq[i]] : 0u;
    /* suffix sums within the run: after the step with offset o, v = sum over [lane, lane + 2o) of the run */
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t vo = __shfl_down(v, o);
        const uint64_t uo = __shfl_down(u, o);
        if (lane + o < 64 && uo == u) v += vo;
    }
    const uint64_t up = __shfl_up(u, 1);
    if (val && (lane == 0 || up != u)) atomicAdd(&rec_cnt[u], v);
    if (!head) return;
    rec_slot[u] = (uint32_t)k;   /* the term RANK: merged records are ranked already (DF skips their gather) */
    (void)slot_of_rank;
    uint32_t d = (uint32_t)(k >> 32);
    if (i == 0 || (uint32_t)(kp >> 32) != d) {
        doc_recoff[d] = u;
        doc_flags[d] = DF_PARTIAL | DF_PRESORTED;
    }
}
__global__ void k_part_npairs(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ head_pos, uint64_t n,
                              uint64_t rec_base, const uint64_t* __restrict__ doc_recoff,
                              uint32_t* __restrict__ doc_npairs) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t d = (uint32_t)(keys[i] >> 32);
    if (i + 1 < n && (uint32_t)(keys[i + 1] >> 32) == d) return; /* last record of d */
    /* unique index of record i's run: head_pos is an EXCLUSIVE scan of run heads */
    const bool is_head = (i == 0 || keys[i] != keys[i - 1]);
    const uint64_t u = head_pos[i] - (is_head ? 0u : 1u);
    doc_npairs[d] = (uint32_t)(rec_base + u + 1 - doc_recoff[d]);
}
int launch_part_merge(const uint64_t* keys, const uint32_t* seq, const uint32_t* part_cnt, const uint32_t* head_pos,
                      uint64_t n, const uint32_t* slot_of_rank, uint64_t rec_base, uint32_t* rec_slot,
                      uint32_t* rec_cnt, uint64_t* doc_recoff, uint32_t* doc_npairs, uint8_t* doc_flags,
                      hipStream_t s) {
    if (!n) return 0;
    /* merged counts accumulate atomically: zero the (at most n) merged record slots */
    if (hipMemsetAsync(rec_cnt + rec_base, 0, n * 4, s) != hipSuccess) return -1;
    k_part_merge<<<grid_for(n), NT, 0, s>>>(keys, seq, part_cnt, head_pos, n, slot_of_rank, rec_base, rec_slot,
                                           rec_cnt, doc_recoff, doc_flags);
    k_part_npairs<<<grid_for(n), NT, 0, s>>>(keys, head_pos, n, rec_base, doc_recoff, doc_npairs);
    return ok();
}

/* ------------------------------------------------ dense merge (long documents) --
 * A document of many chunks (longer than DENSE_DOC, listed by K0) leaves one partial
 * record per (chunk, term): c5's four 100 MB documents give 23 M of them.  Instead of
 * radix-sorting those, they are summed into a dense per-document count array over term
 * ranks (u32[nb][V], L2/MALL-resident at V = 5e4), and only the other partial records
 * are sorted and merged; the dense arrays are then emitted in rank order — the same
 * presorted runs the merge writes. */
__global__ void k_set_big_idx(const uint32_t* __restrict__ big_list, uint32_t nb, uint32_t* __restrict__ big_idx) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) big_idx[big_list[b]] = b;
}
int launch_set_big_idx(const uint32_t* big_list, uint32_t nb, uint32_t* big_idx, hipStream_t s) {
    if (!nb) return 0;
    k_set_big_idx<<<grid_for(nb), NT, 0, s>>>(big_list, nb, big_idx);
    return ok();
}

/* Records of listed documents are added into their dense array; the others are written
 * straight out as sort keys (order is irrelevant: they are sorted next), positions by a
 * wave-aggregated atomic on *nkeep. */
__global__ void k_part_dense(const uint32_t* __restrict__ pdoc, const uint32_t* __restrict__ pslot,
                             const uint32_t* __restrict__ pcnt, uint64_t q, const uint32_t* __restrict__ big_idx,
                             const uint32_t* __restrict__ rank_of_slot, uint32_t V, uint32_t* __restrict__ dense,
                             uint64_t* __restrict__ keys, uint32_t* __restrict__ seq, uint32_t* __restrict__ cnt_out,
                             uint32_t* __restrict__ nkeep) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool val = i < q;
    const uint32_t d = val ? pdoc[i] : 0u;
    const uint32_t b = val ? big_idx[d] : 0u;
    const uint32_t r = val ? rank_of_slot[pslot[i]] : 0u;
    const uint32_t c = val ? pcnt[i] : 0u;
    const bool kept = val && b == 0xFFFFFFFFu;
    /* DENSE_REP copies per document, picked by workgroup: a hot term's adds (one per chunk
     * of the document, ~6000) spread over the copies instead of queueing on one address */
    if (val && !kept && r < V) atomicAdd(&dense[((uint64_t)b * DENSE_REP + (blockIdx.x & (DENSE_REP - 1))) * V + r], c);
    const uint64_t km = __ballot(kept);
    if (!km) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t leader = (uint32_t)__builtin_ctzll(km);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(nkeep, (uint32_t)__popcll(km));
    base = (uint32_t)__shfl(base, (int)leader);
    if (kept) {
        const uint32_t p = base + (uint32_t)__popcll(km & ((1ull << lane) - 1ull));
        keys[p] = ((uint64_t)d << 32) | r;
        seq[p] = p;
        cnt_out[p] = c;
    }
}
/* The same split with the listed documents' adds aggregated in LDS first (V <= 65536).
 * Partial records arrive in K1's flush order, so a long run of them belongs to one long
 * document (its chunks are in flight together): a workgroup takes PDL_RECS consecutive
 * records and one slice of PDL_SLICE ranks (blockIdx.y), sums the records of its range's
 * first document ("home") into u32 LDS bins of that slice, and adds only the non-zero
 * bins to the dense array at the end — one device atomic per (range, term) instead of
 * one per record.  Records of other listed documents take the global atomic as before;
 * kept records are written by slice 0 only.  c5 merge: 1.06 ms with per-record atomics,
 * 0.48 / 0.57 / 0.72 ms with 64K / 128K / 256K-record ranges. */
constexpr uint32_t PDL_NT = 1024;
constexpr uint32_t PDL_SLICE = 32768;      /* u32 bins: 128 KB of LDS */
#ifndef PDL_RECS_N
#define PDL_RECS_N 65536u
#endif
constexpr uint32_t PDL_RECS = PDL_RECS_N;    /* records per workgroup */
#ifndef PDL_B_N
#define PDL_B_N 4
#endif
constexpr int PDL_B = PDL_B_N;                 /* records per thread in flight together */
__global__ __launch_bounds__(PDL_NT) void k_part_dense_lds(const uint32_t* __restrict__ pdoc,
                                                           const uint32_t* __restrict__ pslot,
                                                           const uint32_t* __restrict__ pcnt, uint64_t q,
                                                           const uint32_t* __restrict__ big_idx,
                                                           const uint32_t* __restrict__ rank_of_slot, uint32_t V,
                                                           uint32_t* __restrict__ dense, uint64_t* __restrict__ keys,
                                                           uint32_t* __restrict__ seq, uint32_t* __restrict__ cnt_out,
                                                           uint32_t* __restrict__ nkeep) {
    extern __shared__ uint32_t pbins[];
    __shared__ uint32_t home;
    const uint32_t s0 = blockIdx.y * PDL_SLICE;
    const uint32_t sw = V - s0 < PDL_SLICE ? V - s0 : PDL_SLICE;
    const uint64_t r0 = (uint64_t)blockIdx.x * PDL_RECS;
    const uint64_t r1 = r0 + PDL_RECS < q ? r0 + PDL_RECS : q;
    const uint32_t rep = blockIdx.x & (DENSE_REP - 1);
    for (uint32_t k = threadIdx.x; k < sw; k += PDL_NT) pbins[k] = 0;
    if (threadIdx.x == 0) home = big_idx[pdoc[r0]];
    __syncthreads();
    const uint32_t hb = home;
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t i0 = r0 + threadIdx.x; i0 < r1; i0 += (uint64_t)PDL_B * PDL_NT) {
        uint32_t d[PDL_B], b[PDL_B], r[PDL_B], c[PDL_B];
#pragma unroll
        for (int e = 0; e < PDL_B; ++e) {
            const uint64_t i = i0 + (uint64_t)e * PDL_NT;
            const bool val = i < r1;
            d[e] = val ? pdoc[i] : 0u;
            r[e] = val ? pslot[i] : 0u;
            c[e] = val ? pcnt[i] : 0u;
        }
#pragma unroll
        for (int e = 0; e < PDL_B; ++e) {
            const bool val = i0 + (uint64_t)e * PDL_NT < r1;
            b[e] = val ? big_idx[d[e]] : 0u;
            r[e] = val ? rank_of_slot[r[e]] : 0u;
        }
#pragma unroll
        for (int e = 0; e < PDL_B; ++e) {
            const uint64_t i = i0 + (uint64_t)e * PDL_NT;
            const bool val = i < r1;
            const bool kept = val && b[e] == 0xFFFFFFFFu;
            if (val && !kept && r[e] < V && r[e] - s0 < sw) {
                if (b[e] == hb) atomicAdd(&pbins[r[e] - s0], c[e]);
                else atomicAdd(&dense[((uint64_t)b[e] * DENSE_REP + rep) * V + r[e]], c[e]);
            }
            if (blockIdx.y != 0) continue;
            const uint64_t km = __ballot(kept);
            if (!km) continue;
            const uint32_t leader = (uint32_t)__builtin_ctzll(km);
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(nkeep, (uint32_t)__popcll(km));
            base = (uint32_t)__shfl(base, (int)leader);
            if (kept) {
                const uint32_t p = base + (uint32_t)__popcll(km & ((1ull << lane) - 1ull));
                keys[p] = ((uint64_t)d[e] << 32) | r[e];
                seq[p] = p;
                cnt_out[p] = c[e];
            }
        }
    }
    __syncthreads();
    if (hb == 0xFFFFFFFFu) return;
    uint32_t* dst = dense + ((uint64_t)hb * DENSE_REP + rep) * V + s0;
    for (uint32_t k = threadIdx.x; k < sw; k += PDL_NT) {
        const uint32_t v = pbins[k];
        if (v) atomicAdd(&dst[k], v);
    }
}
int launch_part_dense(const uint32_t* part_doc, const uint32_t* part_slot, const uint32_t* part_cnt, uint64_t q,
                      const uint32_t* big_idx, const uint32_t* rank_of_slot, uint32_t V, uint32_t* dense,
                      uint64_t* keys, uint32_t* seq, uint32_t* cnt_out, uint32_t* nkeep, hipStream_t s) {
    if (!q) return 0;
    if (V <= 2u * PDL_SLICE) {
        const dim3 grid((uint32_t)((q + PDL_RECS - 1) / PDL_RECS), (V + PDL_SLICE - 1) / PDL_SLICE);
        const uint32_t lds = (V < PDL_SLICE ? V : PDL_SLICE) * 4u;
        k_part_dense_lds<<<grid, PDL_NT, lds, s>>>(part_doc, part_slot, part_cnt, q, big_idx, rank_of_slot, V, dense,
                                                   keys, seq, cnt_out, nkeep);
        return ok();
    }
    k_part_dense<<<grid_for(q), NT, 0, s>>>(part_doc, part_slot, part_cnt, q, big_idx, rank_of_slot, V, dense, keys,
                                           seq, cnt_out, nkeep);
    return ok();
}

constexpr uint32_t DENSE_TILE = 4 * NT;   /* ranks per emission tile: 4 per thread */
__device__ __forceinline__ uint32_t dense_sum(const uint32_t* __restrict__ dense, uint32_t b, uint32_t V, uint32_t r) {
    uint32_t v = 0;
#pragma unroll
    for (uint32_t k = 0; k < DENSE_REP; ++k) v += dense[((uint64_t)b * DENSE_REP + k) * V + r];
    return v;
}
__global__ void k_dense_count(const uint32_t* __restrict__ dense, uint32_t V, uint32_t nt,
                              uint32_t* __restrict__ tile_cnt) {
    __shared__ uint32_t wsum[NT / 64];
    const uint32_t t = blockIdx.x, b = blockIdx.y;
    const uint32_t r0 = t * DENSE_TILE + threadIdx.x * 4;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) c += (r0 + k < V && dense_sum(dense, b, V, r0 + k) != 0u) ? 1u : 0u;
    uint32_t tot;
    (void)block_excl_scan<NT, false>(c, wsum, &tot);
    if (threadIdx.x == 0) tile_cnt[(uint64_t)b * nt + t] = tot;
}
__global__ void k_dense_write(const uint32_t* __restrict__ dense, uint32_t V, uint32_t nt,
                              const uint32_t* __restrict__ big_list, const uint32_t* __restrict__ slot_of_rank,
                              uint64_t rec_base, const uint32_t* __restrict__ merged_count,
                              const uint32_t* __restrict__ tile_off, uint32_t* __restrict__ rec_slot,
                              uint32_t* __restrict__ rec_cnt, uint64_t* __restrict__ doc_recoff,
                              uint32_t* __restrict__ doc_npairs, uint8_t* __restrict__ doc_flags) {
    __shared__ uint32_t wsum[NT / 64];
    const uint32_t t = blockIdx.x, b = blockIdx.y;
    const uint32_t r0 = t * DENSE_TILE + threadIdx.x * 4;
    uint32_t v[4], c = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = r0 + k < V ? dense_sum(dense, b, V, r0 + k) : 0u;
        c += v[k] ? 1u : 0u;
    }
    uint32_t tot;
    uint32_t o = block_excl_scan<NT, false>(c, wsum, &tot);
    const uint64_t base = rec_base + *merged_count + tile_off[(uint64_t)b * nt + t];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (v[k]) { rec_slot[base + o] = r0 + k; rec_cnt[base + o] = v[k]; ++o; }   /* ranks (see k_part_merge) */
    if (t == 0 && threadIdx.x == 0) {
        const uint32_t d = big_list[b];
        const uint64_t first = tile_off[(uint64_t)b * nt], last = tile_off[(uint64_t)(b + 1) * nt];
        doc_recoff[d] = rec_base + *merged_count + first;
        doc_npairs[d] = (uint32_t)(last - first);
        doc_flags[d] = DF_PARTIAL | DF_PRESORTED;
    }
}
__global__ void k_add_count(uint32_t* __restrict__ merged_count, const uint32_t* __restrict__ add) {
    merged_count[0] += add[0];
}
int launch_dense_emit(const uint32_t* dense, uint32_t nb, uint32_t V, const uint32_t* big_list,
                      const uint32_t* slot_of_rank, uint64_t rec_base, uint32_t* merged_count, uint32_t* tile_cnt,
                      uint32_t* rec_slot, uint32_t* rec_cnt, uint64_t* doc_recoff, uint32_t* doc_npairs,
                      uint8_t* doc_flags, Arena& ar, hipStream_t s) {
    if (!nb || !V) return 0;
    const uint32_t nt = (V + DENSE_TILE - 1) / DENSE_TILE;
    const dim3 grid(nt, nb);
    k_dense_count<<<grid, NT, 0, s>>>(dense, V, nt, tile_cnt);
    if (ok()) return -1;
    if (scan_excl_u32(tile_cnt, tile_cnt, (uint64_t)nt * nb, ar, s)) return -1;
    k_dense_write<<<grid, NT, 0, s>>>(dense, V, nt, big_list, slot_of_rank, rec_base, merged_count, tile_cnt, rec_slot,
                                      rec_cnt, doc_recoff, doc_npairs, doc_flags);
    if (ok()) return -1;
    /* the DF pass and K5 size the merged region from merged_count: add the dense records */
    k_add_count<<<1, 1, 0, s>>>(merged_count, tile_cnt + (uint64_t)nt * nb);
    return ok();
}

/* -------------------------------------------------------------------- DF -- */

constexpr uint32_t DFH_RECS = 65535;      /* records per workgroup up to which no u16 bin can wrap */
constexpr uint32_t DFH_MAXV = 65536;
constexpr uint32_t DFH_ROUNDS = 4;        /* workgroups per resident slot at most: beyond 4 x 65535 records
                                             per slot one workgroup per slot (the wide form) */

/* LDS-privatised DF histogram: 1024 threads (16 waves; at V = 65536 the 128 KB bin array allows one
 * workgroup per CU).  Each thread owns 64 records of the workgroup's range and keeps
 * DFH_B of them in flight at once (slot loads, then rank lookups, then LDS adds): the
 * loop is latency-bound, so the number of dependent round trips is what matters.  The
 * slot -> rank lookups go through a 32 KB direct-mapped LDS cache first (the frequent
 * terms recur in every document of the workgroup's range); only its misses send a
 * random L2 request into the 2-byte map (c2 DF 0.385 -> 0.344 ms, profiles/r04_k1_ab_c2.txt). */
constexpr int DFH_NT = 1024;
#ifndef DFH_B_N
#define DFH_B_N 16
#endif
constexpr int DFH_B = DFH_B_N;
#ifndef DFH_CK_BITS
#define DFH_CK_BITS 12
#endif
constexpr uint32_t DFH_CK = 1u << DFH_CK_BITS;   /* LDS slot -> rank cache entries (4096: 32 KB; with V = 65536 the
                                                    bins + cache fill the 160 KB of LDS exactly) */
__device__ __forceinline__ uint32_t dfh_cslot(uint32_t slot) { return (slot * 0x9E3779B1u) >> (32 - DFH_CK_BITS); }
/* WIDE: a workgroup takes more than DFH_RECS records (large corpora: c3's 2.9e9 records in
 * 256 workgroups instead of 44 K, so 25 MB of partial histograms are written and summed
 * instead of 4.4 GB).  A u16 counter then moves 0x8000 into the global df whenever it
 * reaches 0x8000: the one add that returned 0x7FFF does it, so every crossing is moved once
 * and no counter passes 0x8000 + the adds in flight (< 0xFFFF): no field wraps or carries. */
template <bool WIDE>
__global__ __launch_bounds__(DFH_NT) void k_df_hist_lds(uint32_t* __restrict__ rec_slot, uint64_t nrec,
                                                        const uint32_t* __restrict__ nrec_extra,
                                                        const uint32_t* __restrict__ rank_of_slot,
                                                        const uint16_t* __restrict__ rank16, uint32_t V,
                                                        uint64_t slot_cap, uint64_t ranked_from,
                                                        uint32_t* __restrict__ status, uint64_t per,
                                                        uint32_t* __restrict__ part /* [grid][V/2 words] */,
                                                        uint32_t* __restrict__ df) {
    extern __shared__ __attribute__((aligned(16))) uint32_t bins[]; /* V/2 words of two u16 counters */
    const uint32_t W = (V + 1) / 2;
    for (uint32_t k = threadIdx.x; k < W; k += DFH_NT) bins[k] = 0;
    /* a direct-mapped LDS cache of slot -> rank behind the bins (one 64-bit word per entry:
     * (slot + 1) << 32 | rank, written and read whole): a workgroup's records repeat the
     * corpus's frequent terms in every document, so most rank lookups hit here instead of
     * sending a random L2 request */
    unsigned long long* cache = reinterpret_cast<unsigned long long*>(bins + ((W + 1) & ~1u));
    for (uint32_t k = threadIdx.x; k < DFH_CK; k += DFH_NT) cache[k] = 0ull;
    __syncthreads();
    if (nrec_extra) nrec += *nrec_extra; /* merged partial records, counted on the device */
    const uint64_t r0 = (uint64_t)blockIdx.x * per;
    const uint64_t r1 = r0 + per < nrec ? r0 + per : nrec;
    /* The ranks go back into the records one iteration late, after the next iteration's
     * loads, and every load and store is unconditional (buffer instructions: a record past
     * the range reads as 0 and is replaced, a store with an offset past the range is
     * dropped by the hardware), so the compiler can count them: the first use of a loaded
     * record waits for the loads only (in-order vmcnt), not for the stores behind them.
     * With stores in branches it waited for everything, and with the stores at the end of
     * the iteration the next loads waited for the stores (their data registers) — a third
     * memory round trip per iteration. */
    const uint32_t nr = r1 > r0 ? (uint32_t)(r1 - r0) : 0u;   /* this workgroup's records, relative */
    /* records from rk on hold ranks already (the merged ones) */
    const uint32_t rk = ranked_from <= r0 ? 0u : ranked_from - r0 >= nr ? nr : (uint32_t)(ranked_from - r0);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(rec_slot + r0), 0, (int)(nr * 4u),
                                                                        0x00020000);
    /* the slot -> rank maps through buffer loads too: 32-bit offsets, no 64-bit addresses */
    const __amdgpu_buffer_rsrc_t ms = __builtin_amdgcn_make_buffer_rsrc(
        rank16 ? (void*)rank16 : (void*)rank_of_slot, 0,
        (int)(slot_cap * (rank16 ? 2u : 4u) < 0x7FFFFFF0ull ? slot_cap * (rank16 ? 2u : 4u) : 0x7FFFFFF0ull), 0x00020000);
    uint32_t rp[DFH_B];   /* the previous iteration's ranks to store */
    uint32_t pofs = 0xFFFFFFF0u;   /* their first byte offset (past the range: none) */
    uint32_t pvalid = 0;           /* bit q: record q of the previous iteration is stored */
#pragma unroll
    for (int q = 0; q < DFH_B; ++q) rp[q] = 0u;
    auto store_prev = [&]() {
#pragma unroll
        for (int q = 0; q < DFH_B; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(rp[q], rs,
                                                  ((pvalid >> q) & 1u) ? pofs + (uint32_t)q * DFH_NT * 4u : 0xFFFFFFF0u,
                                                  0, 2 /* nt */);
    };
    for (uint32_t j = threadIdx.x; j < nr; j += (uint32_t)DFH_B * DFH_NT) {
        uint32_t sl[DFH_B], r[DFH_B], g[DFH_B];
        const uint32_t ofs = j * 4u;
#pragma unroll
        for (int q = 0; q < DFH_B; ++q) {
            const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rs, ofs + (uint32_t)q * DFH_NT * 4u, 0, 2 /* nt */);
            sl[q] = j + (uint32_t)q * DFH_NT < nr ? v : 0xFFFFFFFFu;
        }
        store_prev();
        /* classify without branches around loads: every lane reads its cache entry; a
         * miss's rank gather is one unconditional load per record (lanes that need none
         * read entry 0), all DFH_B of them in flight before the first is used (a gather
         * inside the miss branch made the compiler wait for each before the next) */
        uint32_t miss = 0;   /* bit q: record q's rank comes from global memory */
#pragma unroll
        for (int q = 0; q < DFH_B; ++q) {
            const bool ranked = j + (uint32_t)q * DFH_NT >= rk;   /* merged records hold ranks */
            if (sl[q] != 0xFFFFFFFFu && sl[q] >= (ranked ? (uint64_t)V : slot_cap)) {
                atomicOr(status, ST_BOUNDS);
                sl[q] = 0xFFFFFFFFu;
            }
            const unsigned long long e = cache[dfh_cslot(sl[q])];
            const bool hit = (uint32_t)(e >> 32) == sl[q] + 1u;
            const bool need = sl[q] != 0xFFFFFFFFu && !ranked && !hit;
            miss |= need ? 1u << q : 0u;
            r[q] = ranked ? sl[q] : (uint32_t)e;
        }
        if (rank16) {
#pragma unroll
            for (int q = 0; q < DFH_B; ++q)
                g[q] = __builtin_amdgcn_raw_buffer_load_b16(ms, ((miss >> q) & 1u) ? sl[q] * 2u : 0u, 0, 0);
        } else {
#pragma unroll
            for (int q = 0; q < DFH_B; ++q)
                g[q] = __builtin_amdgcn_raw_buffer_load_b32(ms, ((miss >> q) & 1u) ? sl[q] * 4u : 0u, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < DFH_B; ++q) {
            if ((miss >> q) & 1u) {
                r[q] = g[q];
                cache[dfh_cslot(sl[q])] = ((unsigned long long)(sl[q] + 1u) << 32) | r[q];
            }
        }
        pvalid = 0;
#pragma unroll
        for (int q = 0; q < DFH_B; ++q) {
            /* records carry term ranks from here on: K5 reads them without a gather */
            rp[q] = r[q];
            pvalid |= sl[q] != 0xFFFFFFFFu && j + (uint32_t)q * DFH_NT < rk ? 1u << q : 0u;
            if (sl[q] == 0xFFFFFFFFu) continue;
            const uint32_t sh = 16 * (r[q] & 1);
            if (WIDE) {
                const uint32_t old = atomicAdd(&bins[r[q] >> 1], 1u << sh);
                if (((old >> sh) & 0xFFFFu) == 0x7FFFu) {
                    atomicSub(&bins[r[q] >> 1], 0x8000u << sh);
                    atomicAdd(&df[r[q]], 0x8000u);
                }
            } else {
                atomicAdd(&bins[r[q] >> 1], 1u << sh);
            }
        }
        pofs = ofs;
    }
    store_prev();
    __syncthreads();
    uint32_t* out = part + (uint64_t)blockIdx.x * W;
    for (uint32_t k = threadIdx.x; k < W; k += DFH_NT) out[k] = bins[k];
}
/* df[r] += sum over DFC_G partial histograms (blockIdx.y picks the group): all of a
 * thread's column loads are in flight at once, one atomic per (rank, group) */
constexpr uint32_t DFC_G = 32;
__global__ void k_df_colsum(const uint32_t* __restrict__ part, uint32_t nparts, uint32_t V, uint32_t* __restrict__ df) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= V) return;
    const uint32_t W = (V + 1) / 2, sh = 16 * (r & 1);
    const uint32_t p0 = blockIdx.y * DFC_G;
    uint32_t v[DFC_G];
#pragma unroll
    for (uint32_t q = 0; q < DFC_G; ++q)
        v[q] = p0 + q < nparts ? part[(uint64_t)(p0 + q) * W + (r >> 1)] : 0u;
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < DFC_G; ++q) sum += (v[q] >> sh) & 0xFFFFu;
    if (sum) atomicAdd(&df[r], sum);
}
/* V > 65536 (no LDS histogram): global atomics; DFA_B records per thread per pass so that
 * DFA_B rank gathers (random over the slot table: 256 MB at c4) are in flight together
 * instead of one dependent gather per iteration */
constexpr int DFA_B = 8;
__global__ void k_df_hist_atomic(uint32_t* __restrict__ rec_slot, uint64_t nrec, const uint32_t* __restrict__ nrec_extra,
                                 const uint32_t* __restrict__ rank_of_slot, uint64_t slot_cap, uint64_t ranked_from,
                                 uint32_t V, uint32_t* __restrict__ status, uint32_t* __restrict__ df) {
    if (nrec_extra) nrec += *nrec_extra;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < nrec; i0 += stride * DFA_B) {
        uint32_t sl[DFA_B], r[DFA_B];
#pragma unroll
        for (int k = 0; k < DFA_B; ++k) {
            const uint64_t i = i0 + (uint64_t)k * stride;
            sl[k] = i < nrec ? rec_slot[i] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int k = 0; k < DFA_B; ++k) {
            const bool ranked = i0 + (uint64_t)k * stride >= ranked_from;
            r[k] = ranked ? sl[k] : sl[k] < slot_cap ? rank_of_slot[sl[k]] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int k = 0; k < DFA_B; ++k) {
            const uint64_t i = i0 + (uint64_t)k * stride;
            if (i >= nrec) continue;
            if (r[k] >= V) { atomicOr(status, ST_BOUNDS); continue; }
            atomicAdd(&df[r[k]], 1u);
            if (i < ranked_from) rec_slot[i] = r[k];
        }
    }
}
/* V > 65536, partitioned: the 113 M random device atomics of k_df_hist_atomic (c4) miss
 * L2 (df is 40 MB), so instead the records' ranks are partitioned into slices of
 * DFS_SLICE ranks and each slice is counted by one workgroup in LDS.
 *   count    tile t of DFS_TILE records: rank gather, rank written in place (K5 reads
 *            ranks), LDS histogram of slices -> cnt[slice * ntiles + t]
 *   scan     exclusive scan of cnt (slice-major): each (slice, tile) gets its segment
 *   scatter  the same tiles again: LDS positions within the tile's segments, ranks out
 *   count    one workgroup per slice: u32 LDS bins over its ranks, df stored directly */
constexpr uint32_t DFS_NT = 1024;
constexpr uint32_t DFS_PER = 16;
constexpr uint64_t DFS_TILE = (uint64_t)DFS_NT * DFS_PER;
constexpr uint32_t DFS_SLICE = 32768;      /* u32 bins: 128 KB of LDS */
constexpr uint32_t DFS_MAXSL = 4096;       /* slice histogram: 16 KB of LDS (V <= 134 M) */
__global__ __launch_bounds__(DFS_NT) void k_dfs_count(uint32_t* __restrict__ rec_slot, uint64_t nrec,
                                                      const uint32_t* __restrict__ nrec_extra,
                                                      const uint32_t* __restrict__ rank_of_slot, uint64_t slot_cap,
                                                      uint64_t ranked_from, uint32_t V, uint32_t nsl,
                                                      uint32_t* __restrict__ status, uint32_t* __restrict__ cnt) {
    __shared__ uint32_t h[DFS_MAXSL];
    if (nrec_extra) nrec += *nrec_extra;
    for (uint32_t k = threadIdx.x; k < nsl; k += DFS_NT) h[k] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * DFS_TILE + threadIdx.x;
    uint32_t sl[DFS_PER];
#pragma unroll
    for (uint32_t e = 0; e < DFS_PER; ++e) {
        const uint64_t i = t0 + (uint64_t)e * DFS_NT;
        /* the records stream through once: non-temporal, so they do not push the rank map
         * the gathers below hit out of the caches */
        sl[e] = i < nrec ? __builtin_nontemporal_load(&rec_slot[i]) : 0xFFFFFFFFu;
    }
#pragma unroll
    for (uint32_t e = 0; e < DFS_PER; ++e) {
        const uint64_t i = t0 + (uint64_t)e * DFS_NT;
        if (i >= nrec || i >= ranked_from) continue;   /* merged records hold ranks already */
        sl[e] = sl[e] < slot_cap ? rank_of_slot[sl[e]] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (uint32_t e = 0; e < DFS_PER; ++e) {
        const uint64_t i = t0 + (uint64_t)e * DFS_NT;
        if (i >= nrec) continue;
        if (sl[e] >= V) { atomicOr(status, ST_BOUNDS); continue; }   /* never expected */
        if (i < ranked_from) __builtin_nontemporal_store(sl[e], &rec_slot[i]);   /* records carry term ranks from here on */
        atomicAdd(&h[sl[e] / DFS_SLICE], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nsl; k += DFS_NT) cnt[(uint64_t)k * gridDim.x + blockIdx.x] = h[k];
}
__global__ __launch_bounds__(DFS_NT) void k_dfs_scatter(const uint32_t* __restrict__ rec_rank, uint64_t nrec,
                                                        const uint32_t* __restrict__ nrec_extra, uint32_t V,
                                                        uint32_t nsl, const uint32_t* __restrict__ off,
                                                        uint32_t* __restrict__ out) {
    __shared__ uint32_t h[DFS_MAXSL];
    __shared__ uint32_t base[DFS_MAXSL];   /* the tile's segment starts, one gather each */
    if (nrec_extra) nrec += *nrec_extra;
    for (uint32_t k = threadIdx.x; k < nsl; k += DFS_NT) {
        h[k] = 0;
        base[k] = off[(uint64_t)k * gridDim.x + blockIdx.x];
    }
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * DFS_TILE + threadIdx.x;
    uint32_t r[DFS_PER];
#pragma unroll
    for (uint32_t e = 0; e < DFS_PER; ++e) {
        const uint64_t i = t0 + (uint64_t)e * DFS_NT;
        r[e] = i < nrec ? __builtin_nontemporal_load(&rec_rank[i]) : 0xFFFFFFFFu;
    }
#pragma unroll
    for (uint32_t e = 0; e < DFS_PER; ++e) {
        if (r[e] >= V) continue;   /* past the records, or a bad slot (flagged above) */
        const uint32_t k = r[e] / DFS_SLICE;
        const uint32_t p = atomicAdd(&h[k], 1u);
        out[base[k] + p] = r[e];
    }
}
__global__ __launch_bounds__(DFS_NT) void k_dfs_slice(const uint32_t* __restrict__ part, const uint32_t* __restrict__ off,
                                                      uint32_t ntiles, uint32_t V, uint32_t* __restrict__ df,
                                                      bool accumulate) {
    extern __shared__ uint32_t sbins[];
    const uint32_t k = blockIdx.x, s0 = k * DFS_SLICE;
    const uint32_t sw = V - s0 < DFS_SLICE ? V - s0 : DFS_SLICE;
    for (uint32_t j = threadIdx.x; j < sw; j += DFS_NT) sbins[j] = 0;
    __syncthreads();
    const uint32_t b = off[(uint64_t)k * ntiles], e = off[(uint64_t)(k + 1) * ntiles];
    constexpr int B = 8;
    for (uint32_t i0 = b + threadIdx.x; i0 < e; i0 += B * DFS_NT) {
        uint32_t r[B];
#pragma unroll
        for (int q = 0; q < B; ++q) r[q] = i0 + q * DFS_NT < e ? part[i0 + q * DFS_NT] : 0xFFFFFFFFu;
#pragma unroll
        for (int q = 0; q < B; ++q)
            if (r[q] != 0xFFFFFFFFu) atomicAdd(&sbins[r[q] - s0], 1u);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < sw; j += DFS_NT) df[s0 + j] = accumulate ? df[s0 + j] + sbins[j] : sbins[j];
}

/* the LDS histogram's split of nrec_max records: records per workgroup so that the
 * workgroups fill whole waves of the CUs' resident slots (c2: 946 x 65535 records = 3.7
 * waves -> 1024 x 60548, no tail), at most DFH_ROUNDS waves (c3: one per slot, 256 x 11 M
 * records, the wide form).  TFIDF_DF_WGS=<n> fixes the number of workgroups (tests of the wide form on
 * small inputs). */
static void df_lds_plan(uint64_t nrec_max, uint32_t V, uint64_t* per_out, uint32_t* nparts_out) {
    uint64_t nparts = (nrec_max + DFH_RECS - 1) / DFH_RECS;
    const uint32_t W = (V + 1) / 2;
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const uint64_t wg_lds = (uint64_t)((W + 1) & ~1u) * 4 + (uint64_t)DFH_CK * 8;
    const uint64_t per_cu = (uint64_t)163840 / wg_lds >= 2 ? 2 : 1;   /* 1024-thread workgroups */
    const uint64_t slots = (uint64_t)ncu * per_cu;
    uint64_t full = (nparts + slots - 1) / slots * slots;
    /* beyond DFH_ROUNDS waves of 65535-record workgroups: one workgroup per slot (the wide
     * form; c3 DF 11.2 -> 10.2 ms against four per slot, profiles/r06_k1_ab_c2.txt call
     * r06r — the smaller splits keep several rounds, so that the merge stage's kernels beside
     * the main pass find free CUs between them: c5 merge 0.70 vs 0.82 ms) */
    if (full > DFH_ROUNDS * slots) full = slots;
    const char* fe = getenv("TFIDF_DF_WGS");
    const uint64_t forced = fe ? strtoull(fe, nullptr, 0) : 0ull;
    if (forced >= 1 && forced <= (1u << 20)) full = forced;
    uint64_t per = (nrec_max + full - 1) / full;
    if (per < 8192u && !forced) per = 8192u;   /* small inputs: few workgroups (each clears and writes W words) */
    if (per > (1u << 28)) per = 1u << 28;       /* a workgroup's records: 32-bit byte offsets */
    if (per == 0) per = 1;
    *per_out = per;
    *nparts_out = (uint32_t)((nrec_max + per - 1) / per);
}

size_t df_hist_scratch(uint64_t nrec_max, uint32_t V) {
    if (V == 0 || nrec_max == 0) return 256;
    if (V <= DFH_MAXV) {
        uint64_t per = 0;
        uint32_t nparts = 0;
        df_lds_plan(nrec_max, V, &per, &nparts);
        return (size_t)nparts * ((V + 1) / 2) * 4 + 256;
    }
    /* the sliced pass: slice counts per tile (+ their scan's tile sums) and the ranks
     * grouped by slice */
    const uint64_t nsl = ((uint64_t)V + DFS_SLICE - 1) / DFS_SLICE;
    const uint64_t ntiles = (nrec_max + DFS_TILE - 1) / DFS_TILE;
    return (size_t)((ntiles * nsl + 1) * 4 + nrec_max * 4 + (ntiles * nsl) / 16 + 8192 + 1024);
}

int launch_df_hist(uint32_t* rec_slot, uint64_t nrec, const uint32_t* nrec_extra, uint64_t nrec_max,
                   const uint32_t* rank_of_slot, const uint16_t* rank16, uint32_t V, uint64_t slot_cap,
                   uint32_t* status, uint32_t* df, Arena& ar, hipStream_t s, bool accumulate) {
    /* records [0, nrec) hold vocabulary slots (K1), the merged ones after them term ranks */
    const uint64_t ranked_from = nrec;
    if (V == 0) return 0;
    if (nrec_max < nrec) nrec_max = nrec;
    if (nrec_max == 0)
        return accumulate ? 0 : hipMemsetAsync(df, 0, (size_t)V * 4, s) == hipSuccess ? 0 : -1;
    if (V <= DFH_MAXV) {
        uint64_t per = 0;
        uint32_t nparts = 0;
        df_lds_plan(nrec_max, V, &per, &nparts);
        const uint32_t W = (V + 1) / 2;
        size_t m = ar.mark();
        uint32_t* part = (uint32_t*)ar.get((size_t)nparts * W * 4);
        if (!part) return -2;
        if (!accumulate && hipMemsetAsync(df, 0, (size_t)V * 4, s) != hipSuccess) return -1;
        const size_t lds = (size_t)((W + 1) & ~1u) * 4 + (size_t)DFH_CK * 8;
        if (per > DFH_RECS)
            k_df_hist_lds<true><<<nparts, DFH_NT, lds, s>>>(rec_slot, nrec, nrec_extra, rank_of_slot, rank16, V,
                                                            slot_cap, ranked_from, status, per, part, df);
        else
            k_df_hist_lds<false><<<nparts, DFH_NT, lds, s>>>(rec_slot, nrec, nrec_extra, rank_of_slot, rank16, V,
                                                             slot_cap, ranked_from, status, per, part, df);
        k_df_colsum<<<dim3(grid_for(V), (nparts + DFC_G - 1) / DFC_G), NT, 0, s>>>(part, nparts, V, df);
        ar.release(m);
        return ok();
    }
    {
        const uint32_t nsl = (uint32_t)(((uint64_t)V + DFS_SLICE - 1) / DFS_SLICE);
        const uint64_t ntiles = (nrec_max + DFS_TILE - 1) / DFS_TILE;
        if (nsl <= DFS_MAXSL && nrec_max < (1ull << 32) && ntiles * nsl < (1ull << 31)) {
            size_t m = ar.mark();
            uint32_t* cnt = (uint32_t*)ar.get((size_t)(ntiles * nsl + 1) * 4);
            uint32_t* part = (uint32_t*)ar.get((size_t)nrec_max * 4);
            if (!cnt || !part) return -2;   /* arena too small: the run is retried with a larger one */
            {
                k_dfs_count<<<(uint32_t)ntiles, DFS_NT, 0, s>>>(rec_slot, nrec, nrec_extra, rank_of_slot, slot_cap,
                                                               ranked_from, V, nsl, status, cnt);
                if (ok()) return -1;
                if (scan_excl_u32(cnt, cnt, ntiles * nsl, ar, s)) return -1;
                k_dfs_scatter<<<(uint32_t)ntiles, DFS_NT, 0, s>>>(rec_slot, nrec, nrec_extra, V, nsl, cnt, part);
                if (ok()) return -1;
                k_dfs_slice<<<nsl, DFS_NT, (size_t)(V < DFS_SLICE ? V : DFS_SLICE) * 4, s>>>(part, cnt, (uint32_t)ntiles,
                                                                                           V, df, accumulate);
                ar.release(m);
                return ok();
            }
        }
    }
    if (!accumulate && hipMemsetAsync(df, 0, (size_t)V * 4, s) != hipSuccess) return -1;
    k_df_hist_atomic<<<4096, NT, 0, s>>>(rec_slot, nrec, nrec_extra, rank_of_slot, slot_cap, ranked_from, V, status,
                                         df);
    return ok();
}

/* present[df] = 1 for every df value in use (present sized N+2, pre-zeroed) */
__global__ void k_df_mark(const uint32_t* __restrict__ df, uint32_t V, uint32_t* __restrict__ present) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < V) present[df[r]] = 1u;
}
int launch_df_mark(const uint32_t* df, uint32_t V, uint32_t* present, hipStream_t s) {
    if (!V) return 0;
    k_df_mark<<<grid_for(V), NT, 0, s>>>(df, V, present);
    return ok();
}
/* vals[k] = k-th distinct df value; present_scan = exclusive scan of present (nvals+1) */
__global__ void k_df_list(const uint32_t* __restrict__ ps, uint64_t nvals, uint32_t* __restrict__ vals) {
    uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= nvals) return;
    if (ps[x + 1] != ps[x]) vals[ps[x]] = (uint32_t)x;
}
int launch_df_list(const uint32_t* present_scan, uint64_t nvals, uint32_t* vals, hipStream_t s) {
    k_df_list<<<grid_for(nvals), NT, 0, s>>>(present_scan, nvals, vals);
    return ok();
}

/* ------------------------------------------------------- document order -- */

/* "docN@" strcmp order: decimal digits padded on the right with the value 10 ('@' sorts
 * after every digit, TFIDF.c:132,245,273), read as a base-11 number. */
__global__ void k_doc_keys(const uint32_t* __restrict__ ids, uint32_t n, uint64_t* __restrict__ keys,
                           uint32_t* __restrict__ seq) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t id = ids ? ids[i] : i + 1;
    uint32_t dg[10];
    int k = 0;
    do { dg[k++] = id % 10; id /= 10; } while (id);
    uint64_t key = 0;
    for (int p = 0; p < 10; ++p) key = key * 11 + (p < k ? dg[k - 1 - p] : 10u);
    keys[i] = key;
    seq[i] = i;
}
int launch_doc_keys(const uint32_t* doc_ids, uint32_t ndocs, uint64_t* keys, uint32_t* seq, hipStream_t s) {
    if (!ndocs) return 0;
    k_doc_keys<<<grid_for(ndocs), NT, 0, s>>>(doc_ids, ndocs, keys, seq);
    return ok();
}
/* per output position i (document order[i]): its pair count for the offsets scan, and
 * the packed K5 metadata {record offset lo, hi, npairs | flags << 30, docSize} so that
 * K5 reads one coalesced 16-byte word per document instead of a dependent chain */
__global__ void k_gather_meta(const uint32_t* __restrict__ order, const uint32_t* __restrict__ np,
                              const uint64_t* __restrict__ recoff, const uint32_t* __restrict__ dsize,
                              const uint8_t* __restrict__ flags, uint32_t n, uint64_t* __restrict__ out,
                              uint4* __restrict__ meta) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t d = order[i];
    const uint32_t c = np[d];
    const uint64_t rb = c ? recoff[d] : 0ull;
    out[i] = c;
    meta[i] = make_uint4((uint32_t)rb, (uint32_t)(rb >> 32), (c & 0x3FFFFFFFu) | ((uint32_t)(flags[d] & 3u) << 30), dsize[d]);
}
int launch_gather_meta(const uint32_t* order, const uint32_t* doc_npairs, const uint64_t* doc_recoff,
                       const uint32_t* doc_size, const uint8_t* doc_flags, uint32_t ndocs, uint64_t* npairs_ord,
                       uint4* meta, hipStream_t s) {
    if (!ndocs) return 0;
    k_gather_meta<<<grid_for(ndocs), NT, 0, s>>>(order, doc_npairs, doc_recoff, doc_size, doc_flags, ndocs,
                                                npairs_ord, meta);
    return ok();
}

/* ------------------------------------------------------ score + order (K5) */

constexpr int K5_MAX = K5_MAX_PAIRS;
constexpr uint32_t K5_SMALL = 64;     /* one wave, bitonic across the lanes */
constexpr uint32_t K5_SMALL_DOC = 128; /* documents up to this many pairs: k_score_small */
constexpr uint32_t K5_PS_SPLIT = 4096; /* presorted documents over this many pairs: chunk tasks */
constexpr uint32_t K5_WAVE = 1024;    /* one wave, LDS radix sort of packed (rank, index) keys */
constexpr uint32_t K5_IDX_BITS = 11;  /* index bits of a packed key (n <= 2048) */
constexpr int K5_BATCH = 8;           /* gathers per lane in flight together */
#ifndef K5_EB
#define K5_EB 4                       /* wide path: idf gathers per lane in flight together */
#endif
#ifndef K5_EMIT
#define K5_EMIT 2                     /* bucket path's emission: positions per lane whose idf are gathered
                                         before any of their stores (8: 15 VGPRs spilled, slower;
                                         profiles/r06_k1_ab_c2.txt call r06q) */
#endif
#ifndef K5_WPS
#define K5_WPS 4                      /* waves per SIMD the wave kernel is compiled for */
#endif
#ifndef K5_WPS_WIDE
#define K5_WPS_WIDE 4                 /* ... its wide-rank instance */
#endif
constexpr uint32_t K5_NB_BITS = 9;    /* bucket sort: 512 buckets by the rank's top bits */
constexpr uint32_t K5_NB = 1u << K5_NB_BITS;
constexpr uint32_t K5_GROUP_MAX = 48; /* larger buckets (skewed ranks): the radix path */
constexpr uint32_t K5L_GROUP_MAX = 32; /* k_score_large: larger buckets (skewed ranks) take the radix path */
#ifndef K5L_EB
#define K5L_EB 8                      /* k_score_large: elements per thread in flight together */
#endif

/* idf of every term rank: one gather per pair in K5 instead of three dependent ones */
__global__ void k_idf_of_rank(const uint32_t* __restrict__ df_of_rank, const uint32_t* __restrict__ idf_idx,
                              const double* __restrict__ idf, uint32_t V, double* __restrict__ out) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < V) out[r] = idf_idx ? idf[idf_idx[df_of_rank[r]]] : idf[df_of_rank[r]];   /* null: table over all df */
}

/* idf of term rank r: the per-rank table, or (BYDF: a.idf_by_df) the idf table over df
 * values indexed by the term's df.  A compile-time choice (every score kernel is
 * instantiated for both): as a run-time branch, the join after it made the compiler wait
 * with vmcnt(0) before every idf gather of the by-rank case (the other branch's df load
 * might still be in flight), so a batch's gathers ran one after another and each also
 * waited for every store before it. */
template <bool BYDF>
__device__ __forceinline__ double k5_idf(const K5Args& a, uint32_t r) {
    if constexpr (BYDF) return G(a.idf)[G(a.df_of_rank)[r]];
    else return G(a.idf_rank)[r];
}

/* The output is 16 bytes per pair (term rank, count, score): the document, docSize and
 * df of a pair are per-document / per-term values the fetch expands on the host. */
template <bool BYDF>
__device__ __forceinline__ void k5_emit(const K5Args& a, uint64_t o, double ds, uint32_t rank, uint32_t cnt) {
    const double tf = (double)cnt / ds;   /* TFIDF.c:202 */
    sto(&a.out_term[o], (uint32_t)(rank));
    sto(&a.out_cnt[o], (uint32_t)(cnt));
    sto(&a.out_score[o], (double)(tf * k5_idf<BYDF>(a, rank))); /* TFIDF.c:243-244 (idf from the host-libm LUT) */
}

/* records hold term ranks once the DF pass has run (k_df_hist_* rewrite them in place) */
__device__ __forceinline__ uint32_t k5_rank(const K5Args& a, uint32_t r) {
    if (r >= a.nterms) { atomicOr(a.status, ST_BOUNDS); r = 0; }
    return r;
}

/* ranks up to 32 - K5_IDX_BITS bits pack (rank, index) keys; up to K5_WIDE_BITS the wave
 * kernel's bucket sort packs only the rank bits below the bucket (wide mode) */
constexpr uint32_t K5_WIDE_BITS = 32 - K5_IDX_BITS + K5_NB_BITS;
/* which kernel sorts a document of n pairs */
__device__ __forceinline__ bool k5_by_wave(const K5Args& a, uint32_t n, bool presorted) {
    if (presorted) return n <= K5_WAVE;
    return n <= K5_SMALL || (n <= K5_WAVE && a.rank_bits <= K5_WIDE_BITS);
}

/* Skewed documents (a bucket of the bucket sort above K5_GROUP_MAX keys): LSD radix sort
 * by rank, 8-bit digits, of the packed keys in buf0 — a wave-private histogram, a DPP scan
 * of the 256 bins and a stable multisplit scatter (8 ballots) per round of 64 keys. */
/* (the fields it uses are passed as values: a reference to the kernel's argument struct
 * would put the struct on the stack, and every field the caller reads would become a
 * scratch load — one in-order vmcnt wait behind its prefetch loads) */
__device__ __noinline__ void k5_radix(uint32_t rank_bits, const uint32_t* rec_cnt, const double* idf_rank,
                                      uint32_t* out_term, uint32_t* out_cnt, double* out_score, uint32_t* buf0,
                                      uint32_t* buf1, uint32_t* h, uint32_t n, uint64_t rb, uint64_t ob, double ds) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t cur = 0;
    for (uint32_t sh = K5_IDX_BITS; sh < K5_IDX_BITS + rank_bits; sh += 8) {
        const uint32_t* src = cur ? buf1 : buf0;
        uint32_t* dst = cur ? buf0 : buf1;
        h[4 * lane] = 0; h[4 * lane + 1] = 0; h[4 * lane + 2] = 0; h[4 * lane + 3] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t j = lane; j < n; j += 64) atomicAdd(&h[(src[j] >> sh) & 0xFFu], 1u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        {
            const uint32_t v0 = h[4 * lane], v1 = h[4 * lane + 1], v2 = h[4 * lane + 2], v3 = h[4 * lane + 3];
            const uint32_t tot = v0 + v1 + v2 + v3;
            const uint32_t ex = wave_incl_scan(tot) - tot;
            h[4 * lane] = ex; h[4 * lane + 1] = ex + v0; h[4 * lane + 2] = ex + v0 + v1; h[4 * lane + 3] = ex + v0 + v1 + v2;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t r0 = 0; r0 < n; r0 += 64) {
            const uint32_t j = r0 + lane;
            const bool valid = j < n;
            const uint32_t key = valid ? src[j] : 0u;
            const uint32_t dg = (key >> sh) & 0xFFu;
            uint64_t m = __ballot(valid);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const bool bit = (dg >> b) & 1u;
                const uint64_t bb = __ballot(valid && bit);
                m &= bit ? bb : ~bb;
            }
            const uint32_t lrank = (uint32_t)__popcll(m & below);
            const uint32_t cnt = (uint32_t)__popcll(m);
            const uint32_t base = valid ? h[dg] : 0u;   /* every lane reads before any lane writes */
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (valid) {
                dst[base + lrank] = key;
                if (lrank == cnt - 1u) h[dg] = base + cnt;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        cur ^= 1u;
    }
    const uint32_t* fin = cur ? buf1 : buf0;
    for (uint32_t j0 = 0; j0 < n; j0 += 64 * K5_BATCH) {
        uint32_t key[K5_BATCH], cnt[K5_BATCH];
        double idf[K5_BATCH];
#pragma unroll
        for (int q = 0; q < K5_BATCH; ++q) {
            const uint32_t j = j0 + 64 * q + lane;
            key[q] = j < n ? fin[j] : 0u;
        }
#pragma unroll
        for (int q = 0; q < K5_BATCH; ++q) {
            cnt[q] = rec_cnt[rb + (key[q] & ((1u << K5_IDX_BITS) - 1u))];
            idf[q] = G(idf_rank)[key[q] >> K5_IDX_BITS];
        }
#pragma unroll
        for (int q = 0; q < K5_BATCH; ++q) {
            const uint32_t j = j0 + 64 * q + lane;
            if (j < n) {
                sto(&out_term[ob + j], (uint32_t)(key[q] >> K5_IDX_BITS));
                sto(&out_cnt[ob + j], (uint32_t)(cnt[q]));
                sto(&out_score[ob + j], (double)(((double)cnt[q] / ds) * idf[q])); /* TFIDF.c:202,243-244 */
            }
        }
    }
}

/* One wave per document, four documents per workgroup, no block barriers.  The wave's
 * next document is prefetched while the current one is sorted: its metadata two documents
 * ahead, its output offset, and up to K5_PF x 64 (slot, count) records one document
 * ahead, so a document costs two dependent global round trips (rank gathers, idf
 * gathers) instead of five.
 *   n <= 64      bitonic sort of (rank, count) across the lanes (__shfl_xor);
 *   n <= 1024    bucket sort of packed (rank << 11 | index) keys by the rank's top 9 bits
 *                (counts kept in LDS by index), k5_radix for skewed documents;
 *   presorted    merged runs (finalize's partial merge) are emitted as they are. */
constexpr int K5_PF = 8;                 /* records prefetched per lane: documents up to 512 pairs */
constexpr int K5_RQ = K5_WAVE / 64;      /* rank registers per lane: documents up to K5_WAVE pairs */
__device__ __forceinline__ void k5_prefetch(const K5Args& a, const uint4& m, uint32_t lane, uint32_t (&s)[K5_PF],
                                            uint32_t (&c)[K5_PF]) {
    const uint32_t n = m.z & 0x3FFFFFFFu;
    const uint64_t rb = ((uint64_t)m.y << 32) | m.x;
    const bool ok = n != 0u && n <= K5_WAVE && rb + n <= a.rec_total;
#pragma unroll
    for (int q = 0; q < K5_PF; ++q) {
        const uint32_t j = 64u * q + lane;
        const bool v = ok && j < n;
        s[q] = v ? a.rec_slot[rb + j] : 0u;
        c[q] = v ? a.rec_cnt[rb + j] : 0u;
    }
}

__device__ __forceinline__ uint32_t lane_id_fresh() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

/* WIDE: the instance launched when ranks exceed 32 - K5_IDX_BITS bits (its extra path
 * costs registers the common instance must not pay: c2 score 0.88 -> 1.16 ms with it) */
template <bool WIDE, bool BYDF>
__global__ __launch_bounds__(NT, WIDE ? K5_WPS_WIDE : K5_WPS) void k_score_wave(K5Args a) {
    static_assert(WIDE || !BYDF, "idf by df only with wide ranks (V > 2^21; k5_radix reads idf by rank)");
    __shared__ __attribute__((aligned(16))) uint32_t kb[NT / 64][2][K5_WAVE];
    __shared__ uint32_t hist[NT / 64][K5_NB];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * (NT / 64);
    uint32_t* buf0 = kb[w][0];
    uint32_t* buf1 = kb[w][1];
    uint32_t* h = hist[w];
    /* the positions this kernel scores: its segment of the class list (k_k5_classify), or
     * every position */
    const uint32_t* L = nullptr;
    uint32_t lcount = a.ndocs;
    if (a.cls_list) {
        const uint32_t lo = G(a.cls_off)[a.cls_nblk];
        L = a.cls_list + lo;
        lcount = G(a.cls_off)[2 * a.cls_nblk] - lo;
    }
    auto pos_of = [&](uint32_t li) -> uint32_t { return L ? G(L)[li] : li; };
    uint32_t li = blockIdx.x * (NT / 64) + w;
    uint32_t i_cur = li < lcount ? pos_of(li) : 0u;
    uint32_t i_nxt = li + stride < lcount ? pos_of(li + stride) : 0u;
    uint4 m_cur = li < lcount ? gload(a.meta + (i_cur)) : make_uint4(0, 0, 0, 0);
    uint4 m_nxt = li + stride < lcount ? gload(a.meta + (i_nxt)) : make_uint4(0, 0, 0, 0);
    uint64_t ob_cur = li < lcount ? G(a.out_off)[i_cur] : 0ull;
    uint32_t s_cur[K5_PF], c_cur[K5_PF];
    k5_prefetch(a, m_cur, lane, s_cur, c_cur);
    for (; li < lcount; li += stride) {
        /* the lane index recomputed per document (an asm the compiler cannot hoist): held
         * across the loop it and the LDS addresses derived from it were spilled, and each
         * reload's vmcnt wait also waited for the next document's prefetch loads */
        const uint32_t lane = lane_id_fresh();
        const uint32_t i = i_cur;
        const uint4 mc = m_cur;
        const uint64_t ob = ob_cur;
        const uint32_t n = mc.z & 0x3FFFFFFFu;
        const bool presorted = ((mc.z >> 30) & DF_PRESORTED) != 0;
        const uint64_t rb = ((uint64_t)mc.y << 32) | mc.x;
        const double ds = (double)mc.w;
        const bool small_doc = n != 0u && k5_by_wave(a, n, presorted) && rb + n <= a.rec_total;
        /* this document's rank gathers first, then the next document's prefetch: the
         * waits for the ranks leave the prefetch loads in flight */
        uint32_t r[K5_RQ];
#pragma unroll
        for (int q = 0; q < K5_PF; ++q) {
            const uint32_t j = 64u * q + lane;
            r[q] = (small_doc && j < n) ? k5_rank(a, s_cur[q]) : 0xFFFFFFFFu;
            if (small_doc && j < n) buf0[j] = c_cur[q]; /* counts by record index */
        }
        if (small_doc && n > 64u * K5_PF) { /* beyond the prefetch: loaded here */
            uint32_t sx[K5_RQ - K5_PF];
#pragma unroll
            for (int q = K5_PF; q < K5_RQ; ++q) {
                const uint32_t j = 64u * q + lane;
                sx[q - K5_PF] = j < n ? a.rec_slot[rb + j] : 0u;
                if (j < n) buf0[j] = a.rec_cnt[rb + j];
            }
#pragma unroll
            for (int q = K5_PF; q < K5_RQ; ++q) {
                const uint32_t j = 64u * q + lane;
                r[q] = j < n ? k5_rank(a, sx[q - K5_PF]) : 0xFFFFFFFFu;
            }
        } else {
#pragma unroll
            for (int q = K5_PF; q < K5_RQ; ++q) r[q] = 0xFFFFFFFFu;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        {
            const uint32_t inx = li + stride;
            m_cur = m_nxt;
            i_cur = i_nxt;
            ob_cur = inx < lcount ? G(a.out_off)[i_cur] : 0ull;
            i_nxt = inx + stride < lcount ? pos_of(inx + stride) : 0u;
            m_nxt = inx + stride < lcount ? gload(a.meta + (i_nxt)) : make_uint4(0, 0, 0, 0);
            k5_prefetch(a, m_cur, lane, s_cur, c_cur);
        }
        if (n == 0) continue;
        if (!k5_by_wave(a, n, presorted)) { /* k_score_large's document */
            if (WIDE && lane == 0) G(a.large_list)[atomicAdd(a.large_count, 1u)] = i; /* else listed up front */
            continue;
        }
        if (rb + n > a.rec_total) { if (lane == 0) atomicOr(a.status, ST_BOUNDS); continue; }
        if (presorted) {
#pragma unroll
            for (int q = 0; q < K5_RQ; ++q) {
                const uint32_t j = 64u * q + lane;
                if (j < n) k5_emit<BYDF>(a, ob + j, ds, r[q], buf0[j]);
            }
            continue;
        }
#ifndef K5_CNT
#define K5_CNT 128
#endif
        if (n <= (uint32_t)K5_CNT) {
            /* rank by counting: ranks are distinct within a document, so an element's
             * output position is the number of smaller ranks in the document; every lane
             * scans the document's ranks with broadcast 16-byte LDS reads (no atomics, one
             * fence), then gathers its idf values together and stores */
            constexpr int QC = K5_CNT / 64;
#pragma unroll
            for (int q = 0; q < QC; ++q) {
                const uint32_t j = 64u * q + lane;
                if (j < n) buf1[j] = r[q];
            }
            const uint32_t n4 = (n + 3u) & ~3u;
            if (lane < 4u && n + lane < n4) buf1[n + lane] = 0xFFFFFFFFu;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t pos[QC];
#pragma unroll
            for (int q = 0; q < QC; ++q) pos[q] = 0u;
            const uint4* k4p = reinterpret_cast<const uint4*>(buf1);
            for (uint32_t i4 = 0; i4 < n4 / 4u; ++i4) {
                const uint4 k4 = k4p[i4];
#pragma unroll
                for (int q = 0; q < QC; ++q)
                    pos[q] += (k4.x < r[q] ? 1u : 0u) + (k4.y < r[q] ? 1u : 0u) + (k4.z < r[q] ? 1u : 0u) +
                              (k4.w < r[q] ? 1u : 0u);
            }
            double idf[QC];
#pragma unroll
            for (int q = 0; q < QC; ++q) idf[q] = (64u * q + lane < n) ? k5_idf<BYDF>(a, r[q]) : 0.0;
#pragma unroll
            for (int q = 0; q < QC; ++q) {
                const uint32_t j = 64u * q + lane;
                if (j < n) {
                    const uint64_t o = ob + pos[q];
                    const uint32_t cnt = buf0[j];
                    sto(&a.out_term[o], (uint32_t)(r[q]));
                    sto(&a.out_cnt[o], (uint32_t)(cnt));
                    sto(&a.out_score[o], (double)(((double)cnt / ds) * idf[q]));   /* TFIDF.c:202,243-244 */
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            continue;
        }
        if (n <= K5_SMALL) {
            uint32_t key = r[0], val = lane < n ? buf0[lane] : 0u;
#pragma unroll
            for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
                for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                    uint32_t pk = __shfl_xor(key, j, 64), pv = __shfl_xor(val, j, 64);
                    bool take_min = ((lane & k) == 0) == ((lane & j) == 0);
                    if (take_min ? (pk < key) : (pk > key)) { key = pk; val = pv; }
                }
            }
            if (lane < n) k5_emit<BYDF>(a, ob + lane, ds, key, val);
            continue;
        }
        /* ---- bucket sort: ranks are distinct within a document, so an element's position
         * is its bucket's start plus the number of smaller keys in its bucket.  Buckets by
         * the rank's top K5_NB_BITS bits hold ~n/512 keys each. ---- */
        const uint32_t hsh = a.rank_bits > K5_NB_BITS ? a.rank_bits - K5_NB_BITS : 0u;
#pragma unroll
        for (uint32_t q = 0; q < K5_NB / 64; ++q) h[q * 64 + lane] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int q = 0; q < K5_RQ; ++q)
            if (64u * q + lane < n) atomicAdd(&h[r[q] >> hsh], 1u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t gmax;
        {
            constexpr uint32_t PER = K5_NB / 64;
            uint32_t v[PER], tot = 0, mx = 0;
#pragma unroll
            for (uint32_t q = 0; q < PER; ++q) { v[q] = h[lane * PER + q]; tot += v[q]; mx = v[q] > mx ? v[q] : mx; }
            uint32_t run = wave_incl_scan(tot) - tot;
#pragma unroll
            for (uint32_t q = 0; q < PER; ++q) { h[lane * PER + q] = run; run += v[q]; }
            gmax = wave_max(mx);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const bool wide = WIDE;   /* launched only for ranks over 32 - K5_IDX_BITS bits */
        if (gmax > K5_GROUP_MAX && wide) { /* skewed and too wide for packed keys: k_score_large */
            if (lane == 0) G(a.large_list)[atomicAdd(a.large_count, 1u)] = i;
            continue;
        }
        if constexpr (WIDE) if (wide) {
            /* wide ranks (V > 2^21): keys hold the rank bits below the bucket and the index;
             * each lane counts its own elements' smaller bucket mates and stores its pairs
             * at their output positions directly (as the counting path does) */
            const uint32_t lm = (1u << hsh) - 1u;
#pragma unroll
            for (int q = 0; q < K5_RQ; ++q) {
                const uint32_t j = 64u * q + lane;
                if (j < n) buf1[atomicAdd(&h[r[q] >> hsh], 1u)] = ((r[q] & lm) << K5_IDX_BITS) | j;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            constexpr int EB = K5_EB;
#pragma unroll
            for (int q0 = 0; q0 < K5_RQ; q0 += EB) {
                if (64u * q0 >= n) continue;
                uint32_t pos[EB], cnt[EB];
                double idf[EB];
#pragma unroll
                for (int e = 0; e < EB; ++e) {
                    const uint32_t j = 64u * (q0 + e) + lane;
                    const uint32_t rk = r[q0 + e];
                    pos[e] = 0u;
                    cnt[e] = 0u;
                    if (j < n) {
                        const uint32_t d = rk >> hsh, k = ((rk & lm) << K5_IDX_BITS) | j;
                        const uint32_t gs = d ? h[d - 1] : 0u, ge = h[d];
                        uint32_t less = 0;
                        for (uint32_t f = gs; f < ge; ++f) less += buf1[f] < k ? 1u : 0u;
                        pos[e] = gs + less;
                        cnt[e] = buf0[j];
                    }
                    idf[e] = j < n ? k5_idf<BYDF>(a, rk) : 0.0;
                }
#pragma unroll
                for (int e = 0; e < EB; ++e) {
                    if (64u * (q0 + e) + lane < n) {
                        const uint64_t o = ob + pos[e];
                        sto(&a.out_term[o], (uint32_t)(r[q0 + e]));
                        sto(&a.out_cnt[o], (uint32_t)(cnt[e]));
                        sto(&a.out_score[o], (double)(((double)cnt[e] / ds) * idf[e]));   /* TFIDF.c:202,243-244 */
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            continue;
        }
        if (gmax > K5_GROUP_MAX) { /* skewed ranks: stable radix passes over buf0 */
#pragma unroll
            for (int q = 0; q < K5_RQ; ++q) {
                const uint32_t j = 64u * q + lane;
                if (j < n) buf0[j] = (r[q] << K5_IDX_BITS) | j;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if constexpr (!WIDE)   /* the wide instance runs only for wide ranks: handed off above */
                k5_radix(a.rank_bits, a.rec_cnt, a.idf_rank, a.out_term, a.out_cnt, a.out_score, buf0, buf1, h, n,
                         rb, ob, ds);
            continue;
        }
#pragma unroll
        for (int q = 0; q < K5_RQ; ++q) {
            const uint32_t j = 64u * q + lane;
            if (j < n) buf1[atomicAdd(&h[r[q] >> hsh], 1u)] = (r[q] << K5_IDX_BITS) | j;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        /* h[d] is now bucket d's end (= bucket d+1's start).  Every position is computed
         * before any key moves (buf1 is read by the in-bucket counts), then the keys are
         * placed in order and emitted with coalesced stores.  Positions are computed per
         * element (q, lane), whose key is (r[q], its index): only the positions are held
         * (round 5 held each bucketed slot's key as well, 16 more VGPRs: 9 spilled) */
        uint32_t pp[K5_RQ];
#pragma unroll
        for (int q = 0; q < K5_RQ; ++q) {
            const uint32_t j = 64u * q + lane;
            pp[q] = 0u;
            if (j < n) {
                const uint32_t k = (r[q] << K5_IDX_BITS) | j, d = r[q] >> hsh;
                const uint32_t gs = d ? h[d - 1] : 0u, ge = h[d];
                uint32_t less = 0;
                for (uint32_t f = gs; f < ge; ++f) less += buf1[f] < k ? 1u : 0u;
                pp[q] = gs + less;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int q = 0; q < K5_RQ; ++q)
            if (64u * q + lane < n) buf1[pp[q]] = (r[q] << K5_IDX_BITS) | (64u * q + lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        /* Emission: every idf of a batch is gathered before any of its stores, and a batch
         * covers up to K5_EMIT positions per lane.  gfx950's vmcnt counts stores as well as
         * loads, in order, so a gather issued after a store cannot be waited for without
         * waiting for the store: round 5's 4-position batches made each later batch (and the
         * next document's first load) wait for the earlier batches' store acknowledgements.
         * Only the idf values are held across the gathers; keys and counts are re-read from
         * LDS at the store. */
        constexpr int EB = K5_EMIT;
        for (uint32_t j0 = 0; j0 < n; j0 += 64 * EB) {
            double idf[EB];
#pragma unroll
            for (int q = 0; q < EB; ++q) {
                const uint32_t j = j0 + 64 * q + lane;
                idf[q] = k5_idf<BYDF>(a, (j < n ? buf1[j] : 0u) >> K5_IDX_BITS);
            }
#pragma unroll
            for (int q = 0; q < EB; ++q) {
                const uint32_t j = j0 + 64 * q + lane;
                if (j < n) {
                    const uint32_t key = buf1[j], cnt = buf0[key & ((1u << K5_IDX_BITS) - 1u)];
                    sto(&a.out_term[ob + j], (uint32_t)(key >> K5_IDX_BITS));
                    sto(&a.out_cnt[ob + j], (uint32_t)(cnt));
                    sto(&a.out_score[ob + j], (double)(((double)cnt / ds) * idf[q])); /* TFIDF.c:202,243-244 */
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }  /* persistent loop */
}

/* Documents the wave kernel leaves: one workgroup each.  Presorted (merged) runs are
 * scored straight through; others are LSD radix-sorted by rank in LDS, 8-bit digits, with a
 * stable wave64 multisplit (8 ballots) per round of 256 elements. */
/* Two instances share the list: MAXN = K5_MAX / 2 with 1024 buckets (38 KB of LDS: four
 * workgroups per CU) takes presorted documents and those of <= K5_MAX / 2 pairs; MAXN =
 * K5_MAX (72 KB: two per CU) the rest.  The bucket counters alias the radix scratch. */
template <uint32_t MAXN, uint32_t NBB, bool BYDF>
__global__ __launch_bounds__(NT) void k_score_large(K5Args a) {
    constexpr uint32_t NB = 1u << NBB;
    __shared__ uint32_t kbuf[2][MAXN];
    __shared__ uint32_t vbuf[2][MAXN];
    union Scratch {
        struct {
            uint32_t hist[256], run[256];
            uint32_t wcnt[NT / 64][256];
        } r;                              /* radix passes */
        uint32_t bh[NB];                  /* bucket sort */
    };
    __shared__ Scratch U;
    uint32_t (&hist)[256] = U.r.hist;
    uint32_t (&run)[256] = U.r.run;
    uint32_t (&wcnt)[NT / 64][256] = U.r.wcnt;
    uint32_t (&bh)[NB] = U.bh;
    __shared__ uint32_t wsum[NT / 64];
    __shared__ uint32_t bmax;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t* LL = a.large_list;
    uint32_t nlarge;
    if (a.cls_list) {   /* its segment of the class list */
        const uint32_t lo = G(a.cls_off)[2 * a.cls_nblk];
        LL = a.cls_list + lo;
        nlarge = G(a.cls_off)[3 * a.cls_nblk] - lo;
    } else {   /* handed off by the wide wave kernel */
        nlarge = *a.large_count;
    }
    for (uint32_t li = blockIdx.x; li < nlarge; li += gridDim.x) {
    const uint32_t i = G(LL)[li];
    const uint32_t d = G(a.order)[i];
    const uint32_t n = G(a.doc_npairs)[d];
    const bool presorted = (G(a.doc_flags)[d] & DF_PRESORTED) != 0;
    if (MAXN < (uint32_t)K5_MAX ? (!presorted && n > MAXN) : (presorted || n <= (uint32_t)K5_MAX / 2)) continue;
    const uint64_t ob = G(a.out_off)[i], rb = G(a.doc_recoff)[d];
    const double ds = (double)G(a.doc_size)[d];
    if (rb + n > a.rec_total) { /* never expected: report instead of reading past the records */
        if (tid == 0) atomicOr(a.status, ST_BOUNDS);
        continue;
    }
    if (presorted || n > (uint32_t)K5_MAX) {
        if (n > (uint32_t)K5_MAX && !presorted) { if (tid == 0) atomicOr(a.status, ST_BOUNDS); continue; }
        /* K5L_EB elements per thread in flight: the loads, then the idf gathers, then the
         * stores (a per-element loop is one dependent chain of round trips) */
        for (uint32_t j0 = 0; j0 < n; j0 += NT * K5L_EB) {
            uint32_t rk[K5L_EB], cn[K5L_EB];
            double f[K5L_EB];
#pragma unroll
            for (int e = 0; e < K5L_EB; ++e) {
                const uint32_t j = j0 + NT * e + tid;
                rk[e] = j < n ? a.rec_slot[rb + j] : 0u;
                cn[e] = j < n ? a.rec_cnt[rb + j] : 0u;
            }
#pragma unroll
            for (int e = 0; e < K5L_EB; ++e) {
                const uint32_t j = j0 + NT * e + tid;
                if (j < n) rk[e] = k5_rank(a, rk[e]);
                f[e] = j < n ? k5_idf<BYDF>(a, rk[e]) : 0.0;
            }
#pragma unroll
            for (int e = 0; e < K5L_EB; ++e) {
                const uint32_t j = j0 + NT * e + tid;
                if (j < n) {
                    sto(&a.out_term[ob + j], (uint32_t)(rk[e]));
                    sto(&a.out_cnt[ob + j], (uint32_t)(cn[e]));
                    sto(&a.out_score[ob + j], (double)(((double)cn[e] / ds) * f[e]));   /* TFIDF.c:202,243-244 */
                }
            }
        }
        continue;
    }
    for (uint32_t j0 = 0; j0 < n; j0 += NT * K5L_EB) {   /* loads in flight together */
        uint32_t sl[K5L_EB], cn[K5L_EB];
#pragma unroll
        for (int e = 0; e < K5L_EB; ++e) {
            const uint32_t j = j0 + NT * e + tid;
            sl[e] = j < n ? a.rec_slot[rb + j] : 0u;
            cn[e] = j < n ? a.rec_cnt[rb + j] : 0u;
        }
#pragma unroll
        for (int e = 0; e < K5L_EB; ++e) {
            const uint32_t j = j0 + NT * e + tid;
            if (j < n) {
                kbuf[0][j] = k5_rank(a, sl[e]);
                vbuf[0][j] = cn[e];
            }
        }
    }
    {
        /* bucket sort (ranks are distinct within a document): K5L_NB buckets by the rank's
         * top bits, an element's position = its bucket's start + the smaller keys in its
         * bucket.  One histogram, one scan, one scatter instead of rank_bits/8 stable radix
         * passes; skewed documents (a bucket over K5L_GROUP_MAX) keep the radix passes. */
        const uint32_t hsh = a.rank_bits > NBB ? a.rank_bits - NBB : 0u;
        for (uint32_t q = tid; q < NB; q += NT) bh[q] = 0u;
        if (tid == 0) bmax = 0u;
        __syncthreads();
        for (uint32_t j = tid; j < n; j += NT) atomicAdd(&bh[kbuf[0][j] >> hsh], 1u);
        __syncthreads();
        constexpr uint32_t PER = NB / NT;
        uint32_t v[PER], tot = 0, mx = 0;
#pragma unroll
        for (uint32_t q = 0; q < PER; ++q) { v[q] = bh[tid * PER + q]; tot += v[q]; mx = v[q] > mx ? v[q] : mx; }
        uint32_t all;
        uint32_t run = block_excl_scan<NT>(tot, wsum, &all);
#pragma unroll
        for (uint32_t q = 0; q < PER; ++q) { bh[tid * PER + q] = run; run += v[q]; }
        mx = wave_max(mx);
        if (lane == 0) atomicMax(&bmax, mx);
        __syncthreads();
        if (bmax <= K5L_GROUP_MAX) {
            for (uint32_t j = tid; j < n; j += NT) {
                const uint32_t k = kbuf[0][j];
                const uint32_t q = atomicAdd(&bh[k >> hsh], 1u);
                kbuf[1][q] = k;
                vbuf[1][q] = j;
            }
            __syncthreads();   /* bh[d] = bucket d's end = bucket d+1's start */
            for (uint32_t p0 = 0; p0 < n; p0 += NT * K5L_EB) {
                uint32_t kk[K5L_EB], ps[K5L_EB], cn[K5L_EB];
                double f[K5L_EB];
#pragma unroll
                for (int e = 0; e < K5L_EB; ++e) {
                    const uint32_t p = p0 + NT * e + tid;
                    kk[e] = 0u; ps[e] = 0u; cn[e] = 0u;
                    if (p < n) {
                        const uint32_t k = kbuf[1][p], d = k >> hsh;
                        const uint32_t gs = d ? bh[d - 1] : 0u, ge = bh[d];
                        uint32_t less = 0;
                        for (uint32_t g = gs; g < ge; ++g) less += kbuf[1][g] < k ? 1u : 0u;
                        kk[e] = k;
                        ps[e] = gs + less;
                        cn[e] = vbuf[0][vbuf[1][p]];
                    }
                    f[e] = p < n ? k5_idf<BYDF>(a, kk[e]) : 0.0;
                }
#pragma unroll
                for (int e = 0; e < K5L_EB; ++e) {
                    if (p0 + NT * e + tid < n) {
                        const uint64_t o = ob + ps[e];
                        sto(&a.out_term[o], (uint32_t)(kk[e]));
                        sto(&a.out_cnt[o], (uint32_t)(cn[e]));
                        sto(&a.out_score[o], (double)(((double)cn[e] / ds) * f[e]));   /* TFIDF.c:202,243-244 */
                    }
                }
            }
            __syncthreads();   /* the next document reuses the LDS buffers */
            continue;
        }
    }
    const uint64_t lt = (1ull << lane) - 1ull;
    int cur = 0;
    for (uint32_t sh = 0; sh < a.rank_bits; sh += 8) {
        hist[tid] = 0;
        run[tid] = 0;
#pragma unroll
        for (int q = 0; q < NT / 64; ++q) wcnt[q][tid] = 0;
        __syncthreads();
        for (uint32_t j = tid; j < n; j += NT) atomicAdd(&hist[(kbuf[cur][j] >> sh) & 0xFFu], 1u);
        __syncthreads();
        uint32_t tot;
        const uint32_t base = block_excl_scan<NT>(hist[tid], wsum, &tot);
        hist[tid] = base; /* hist now holds each digit's first output slot */
        __syncthreads();
        for (uint32_t r0 = 0; r0 < n; r0 += NT) {
            const uint32_t j = r0 + tid;
            const bool valid = j < n;
            uint32_t key = 0, val = 0, dg = 0;
            if (valid) { key = kbuf[cur][j]; val = vbuf[cur][j]; dg = (key >> sh) & 0xFFu; }
            uint64_t m = __ballot(valid);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                bool bit = (dg >> b) & 1u;
                uint64_t bb = __ballot(valid && bit);
                m &= bit ? bb : ~bb;
            }
            const uint32_t lrank = (uint32_t)__popcll(m & lt);
            if (valid && lrank == 0) wcnt[w][dg] = (uint32_t)__popcll(m);
            __syncthreads();
            if (valid) {
                uint32_t pos = hist[dg] + run[dg] + lrank;
                for (uint32_t q = 0; q < w; ++q) pos += wcnt[q][dg];
                kbuf[cur ^ 1][pos] = key;
                vbuf[cur ^ 1][pos] = val;
            }
            __syncthreads();
            uint32_t add = 0;
#pragma unroll
            for (int q = 0; q < NT / 64; ++q) { add += wcnt[q][tid]; wcnt[q][tid] = 0; }
            run[tid] += add;
            __syncthreads();
        }
        cur ^= 1;
    }
    for (uint32_t j = tid; j < n; j += NT) k5_emit<BYDF>(a, ob + j, ds, kbuf[cur][j], vbuf[cur][j]);
    __syncthreads(); /* the next document reuses the LDS buffers */
    }
}
/* The document classes of K5 (non-wide ranks): 1 small (<= K5_SMALL_DOC pairs:
 * k_score_small), 2 the wave kernel's, 3 k_score_large's; 0 none (no pairs, or a presorted
 * run emitted by k_emit_split's chunk tasks, which k_k5_classify lists).  A per-block count,
 * a scan and a scatter give class-contiguous lists without a device-wide counter (c5: 1e6
 * small documents appended through one atomic counter took 0.18 ms), listed before any
 * scoring kernel runs so that k_score_large can start beside the wave kernel. */
__device__ __forceinline__ uint32_t k5_class(const K5Args& a, uint32_t i) {
    if (i >= a.ndocs) return 0u;
    const uint4 m = gload(a.meta + (i));
    const uint32_t n = m.z & 0x3FFFFFFFu;
    const bool presorted = ((m.z >> 30) & DF_PRESORTED) != 0;
    if (n == 0u) return 0u;
    if (n <= K5_SMALL_DOC) return 1u;
    if (k5_by_wave(a, n, presorted)) return 2u;
    if (presorted && n > K5_PS_SPLIT && a.split_count) return 4u;
    return 3u;
}
__global__ __launch_bounds__(256) void k_k5_classify(K5Args a) {
    __shared__ uint32_t c3[3];
    if (threadIdx.x < 3) c3[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint32_t c = k5_class(a, i);
    if (c >= 1u && c <= 3u) atomicAdd(&c3[c - 1u], 1u);
    if (c == 4u) {
        /* a presorted run (a merged long document: c5's 100 MB ones) needs no sort: its
         * emission is split into 4096-pair tasks every workgroup can take (few: atomics) */
        const uint32_t n = gload(a.meta + (i)).z & 0x3FFFFFFFu;
        const uint32_t nt = (n + K5_PS_SPLIT - 1) / K5_PS_SPLIT;
        const uint32_t b = atomicAdd(a.split_count, nt);
        for (uint32_t k = 0; k < nt; ++k) {
            if (b + k < a.split_cap) a.split_tasks[b + k] = make_uint2(i, k);
            else atomicOr(a.status, ST_BOUNDS);
        }
    }
    __syncthreads();
    if (threadIdx.x < 3) a.cls_off[threadIdx.x * a.cls_nblk + blockIdx.x] = c3[threadIdx.x];
    if (blockIdx.x == 0 && threadIdx.x == 3) a.cls_off[3 * a.cls_nblk] = 0u;   /* the scan's total */
}
__global__ __launch_bounds__(256) void k_k5_scatter(K5Args a) {
    __shared__ uint32_t wc[4][3];
    const uint32_t i = blockIdx.x * 256u + threadIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t c = k5_class(a, i);
    uint32_t rk = 0;
#pragma unroll
    for (uint32_t k = 1; k <= 3; ++k) {
        const uint64_t m = __ballot(c == k);
        if (lane == 0) wc[w][k - 1] = (uint32_t)__popcll(m);
        if (c == k) rk = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    }
    __syncthreads();
    if (c >= 1u && c <= 3u) {
        uint32_t base = G(a.cls_off)[(c - 1) * a.cls_nblk + blockIdx.x];
        for (uint32_t q = 0; q < w; ++q) base += wc[q][c - 1];
        a.cls_list[base + rk] = i;
    }
}

/* Documents of <= K5_SMALL_DOC pairs (c5: 1e6 documents of ~50 pairs), listed by
 * k_k5_classify.  One wave per document, each wave over a contiguous run of the small
 * list: the run's metadata is loaded 64 documents at a time (lane j: document j of the
 * batch) and read out with readlane, and the per-document chain (records -> idf -> output)
 * is software-pipelined: while document k is positioned and written, the idf of k+1 and
 * the records of k+2 are in flight, so a document costs about one memory round trip
 * instead of five.  Position of a pair = the number of smaller ranks in its document
 * (ranks are distinct within a document; presorted runs keep their order).
 * TFIDF.c:202,243-245,273. */
constexpr int K5S_WG = 4;   /* waves per workgroup */
#ifndef K5S_OCC
#define K5S_OCC 6           /* workgroups per CU it is compiled for */
#endif
struct K5SDoc {
    uint64_t rb, ob;
    uint32_t n;
    bool presorted;
    double ds;
};
__device__ __forceinline__ void k5s_batch(const K5Args& a, const uint32_t* L, uint32_t d, uint32_t d1, uint4& m,
                                          uint64_t& ob) {
    m = make_uint4(0, 0, 0, 0);
    ob = 0;
    if (d < d1) {
        const uint32_t i = G(L)[d];
        m = gload(a.meta + i);
        ob = G(a.out_off)[i];
    }
}
template <bool BYDF>
__global__ __launch_bounds__(256, K5S_OCC) void k_score_small(K5Args a) {
    __shared__ __attribute__((aligned(16))) uint32_t kb[K5S_WG][K5_SMALL_DOC + 4];
    __shared__ uint4 bm[K5S_WG][64];      /* the current batch's metadata (the next one: registers) */
    __shared__ uint64_t bo[K5S_WG][64];
    constexpr int Q = K5_SMALL_DOC / 64;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* buf = kb[w];
    const uint32_t nsmall = G(a.cls_off)[a.cls_nblk];   /* the small segment starts the class list */
    const uint32_t nw = gridDim.x * K5S_WG, wid = blockIdx.x * K5S_WG + w;
    const uint32_t per = (nsmall + nw - 1) / nw;
    const uint32_t d0 = wid * per;
    const uint32_t d1 = d0 + per < nsmall ? d0 + per : nsmall;
    if (d0 >= d1) return;
    const uint32_t cnt = d1 - d0;
    const uint32_t* L = a.cls_list;
    uint4 mnxt;
    uint64_t onxt;
    k5s_batch(a, L, d0 + lane, d1, mnxt, onxt);
    bm[w][lane] = mnxt;
    bo[w][lane] = onxt;
    k5s_batch(a, L, d0 + 64 + lane, d1, mnxt, onxt);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t curb = 0;   /* batch in bm / bo */
    auto doc_at = [&](uint32_t k) -> K5SDoc {
        K5SDoc d;
        if (k >= cnt) { d.rb = 0; d.ob = 0; d.n = 0; d.presorted = true; d.ds = 1.0; return d; }
        const int l = (int)(k & 63u);
        uint32_t mx, my, mz, mw, olo, ohi;
        if ((k >> 6) == curb) {
            const uint4 m = bm[w][l];
            const uint64_t o = bo[w][l];
            mx = __builtin_amdgcn_readfirstlane(m.x); my = __builtin_amdgcn_readfirstlane(m.y);
            mz = __builtin_amdgcn_readfirstlane(m.z); mw = __builtin_amdgcn_readfirstlane(m.w);
            olo = __builtin_amdgcn_readfirstlane((uint32_t)o);
            ohi = __builtin_amdgcn_readfirstlane((uint32_t)(o >> 32));
        } else {
            mx = __builtin_amdgcn_readlane(mnxt.x, l); my = __builtin_amdgcn_readlane(mnxt.y, l);
            mz = __builtin_amdgcn_readlane(mnxt.z, l); mw = __builtin_amdgcn_readlane(mnxt.w, l);
            olo = __builtin_amdgcn_readlane((uint32_t)onxt, l);
            ohi = __builtin_amdgcn_readlane((uint32_t)(onxt >> 32), l);
        }
        d.rb = ((uint64_t)my << 32) | mx;
        d.ob = ((uint64_t)ohi << 32) | olo;
        d.n = mz & 0x3FFFFFFFu;
        d.presorted = ((mz >> 30) & DF_PRESORTED) != 0;
        d.ds = (double)mw;
        if (d.n > K5_SMALL_DOC || d.rb + d.n > a.rec_total) {
            if (lane == 0) atomicOr(a.status, ST_BOUNDS);
            d.n = 0;
        }
        return d;
    };
    auto load_rec = [&](const K5SDoc& d, uint32_t (&r)[Q], uint32_t (&c)[Q]) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t j = 64u * q + lane;
            const bool v = j < d.n;
            r[q] = v ? a.rec_slot[d.rb + j] : 0xFFFFFFFFu;
            c[q] = v ? a.rec_cnt[d.rb + j] : 0u;
        }
    };
    auto load_idf = [&](const K5SDoc& d, uint32_t (&r)[Q], double (&f)[Q]) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const bool v = 64u * q + lane < d.n;
            if (v) r[q] = k5_rank(a, r[q]);
            f[q] = v ? k5_idf<BYDF>(a, r[q]) : 0.0;
        }
    };
    K5SDoc D0 = doc_at(0), D1 = doc_at(1);
    uint32_t r0[Q], c0[Q], r1[Q], c1[Q];
    double f0[Q];
    load_rec(D0, r0, c0);
    load_rec(D1, r1, c1);
    load_idf(D0, r0, f0);
    for (uint32_t k = 0; k < cnt; ++k) {
        if (k && (k & 63u) == 0u) {   /* doc k starts batch curb + 1 */
            bm[w][lane] = mnxt;
            bo[w][lane] = onxt;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            ++curb;
            k5s_batch(a, L, d0 + 64u * (curb + 1) + lane, d1, mnxt, onxt);
        }
        const K5SDoc D2 = doc_at(k + 2);
        uint32_t r2[Q], c2[Q];
        double f1[Q];
        load_rec(D2, r2, c2);
        load_idf(D1, r1, f1);
        /* document k: positions, then the output */
        const uint32_t n = D0.n;
        uint32_t pos[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) pos[q] = 64u * q + lane;
        if (!D0.presorted && n > 1u) {
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const uint32_t j = 64u * q + lane;
                if (j < n) buf[j] = r0[q];
            }
            const uint32_t n4 = (n + 3u) & ~3u;
            if (lane < 4u && n + lane < n4) buf[n + lane] = 0xFFFFFFFFu;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int q = 0; q < Q; ++q) pos[q] = 0u;
            const uint4* k4p = reinterpret_cast<const uint4*>(buf);
            for (uint32_t i4 = 0; i4 < n4 / 4u; ++i4) {
                const uint4 k4 = k4p[i4];
#pragma unroll
                for (int q = 0; q < Q; ++q)
                    pos[q] += (k4.x < r0[q] ? 1u : 0u) + (k4.y < r0[q] ? 1u : 0u) + (k4.z < r0[q] ? 1u : 0u) +
                              (k4.w < r0[q] ? 1u : 0u);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            if (64u * q + lane < n) {
                const uint64_t o = D0.ob + pos[q];
                sto(&a.out_term[o], (uint32_t)(r0[q]));
                sto(&a.out_cnt[o], (uint32_t)(c0[q]));
                sto(&a.out_score[o], (double)(((double)c0[q] / D0.ds) * f0[q]));   /* TFIDF.c:202,243-244 */
            }
        }
        D0 = D1;
        D1 = D2;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            r0[q] = r1[q]; c0[q] = c1[q]; f0[q] = f1[q];
            r1[q] = r2[q]; c1[q] = c2[q];
        }
    }
}
/* the chunk tasks of long presorted documents: one workgroup per 4096-pair chunk */
template <bool BYDF>
__global__ __launch_bounds__(256) void k_emit_split(K5Args a) {
    const uint32_t nt = *a.split_count < a.split_cap ? *a.split_count : a.split_cap;
    for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
        const uint2 tk = a.split_tasks[t];
        const uint4 m = gload(a.meta + tk.x);
        const uint32_t n = m.z & 0x3FFFFFFFu;
        const uint64_t rb = ((uint64_t)m.y << 32) | m.x;
        const uint64_t ob = G(a.out_off)[tk.x];
        const double ds = (double)m.w;
        if (rb + n > a.rec_total) { if (threadIdx.x == 0) atomicOr(a.status, ST_BOUNDS); continue; }
        const uint32_t j1 = (tk.y + 1) * K5_PS_SPLIT < n ? (tk.y + 1) * K5_PS_SPLIT : n;
        for (uint32_t j0 = tk.y * K5_PS_SPLIT; j0 < j1; j0 += 256 * K5L_EB) {   /* K5L_EB in flight */
            uint32_t rk[K5L_EB], cn[K5L_EB];
            double f[K5L_EB];
#pragma unroll
            for (int e = 0; e < K5L_EB; ++e) {
                const uint32_t j = j0 + 256u * e + threadIdx.x;
                rk[e] = j < j1 ? a.rec_slot[rb + j] : 0u;
                cn[e] = j < j1 ? a.rec_cnt[rb + j] : 0u;
            }
#pragma unroll
            for (int e = 0; e < K5L_EB; ++e) {
                const uint32_t j = j0 + 256u * e + threadIdx.x;
                if (j < j1) rk[e] = k5_rank(a, rk[e]);
                f[e] = j < j1 ? k5_idf<BYDF>(a, rk[e]) : 0.0;
            }
#pragma unroll
            for (int e = 0; e < K5L_EB; ++e) {
                const uint32_t j = j0 + 256u * e + threadIdx.x;
                if (j < j1) {
                    sto(&a.out_term[ob + j], (uint32_t)(rk[e]));
                    sto(&a.out_cnt[ob + j], (uint32_t)(cn[e]));
                    sto(&a.out_score[ob + j], (double)(((double)cn[e] / ds) * f[e]));   /* TFIDF.c:202,243-244 */
                }
            }
        }
    }
}
static void launch_score_wave(const K5Args& a, bool wide, uint32_t wg, hipStream_t s) {
    if (!wide) k_score_wave<false, false><<<wg, NT, 0, s>>>(a);
    else if (a.idf_by_df) k_score_wave<true, true><<<wg, NT, 0, s>>>(a);
    else k_score_wave<true, false><<<wg, NT, 0, s>>>(a);
}
static void launch_emit_split(const K5Args& a, int ncu, hipStream_t s) {
    if (a.idf_by_df) k_emit_split<true><<<(unsigned)ncu * 4u, 256, 0, s>>>(a);
    else k_emit_split<false><<<(unsigned)ncu * 4u, 256, 0, s>>>(a);
}
static void launch_score_large(const K5Args& a, uint32_t grid, hipStream_t s) {
    static_assert(K5_MAX % 2 == 0 && K5_MAX / 2 >= 1024, "k_score_large instances");
    if (a.idf_by_df) {
        k_score_large<(uint32_t)K5_MAX / 2, 10, true><<<grid, NT, 0, s>>>(a);
        k_score_large<(uint32_t)K5_MAX, 11, true><<<grid, NT, 0, s>>>(a);
    } else {
        k_score_large<(uint32_t)K5_MAX / 2, 10, false><<<grid, NT, 0, s>>>(a);
        k_score_large<(uint32_t)K5_MAX, 11, false><<<grid, NT, 0, s>>>(a);
    }
}
int launch_score_order(const K5Args& a, Arena& ar, hipStream_t s, hipStream_t s2, hipEvent_t ev_fork,
                       hipEvent_t ev_join) {
    if (!a.ndocs) return 0;
    {   /* the handed-off list's and the chunk tasks' counters, one launch */
        FillList fl{};
        fl.p[0] = a.large_count;
        fl.bytes[0] = 4;
        fl.n = 1;
        if (a.split_count) {
            fl.p[1] = a.split_count;
            fl.bytes[1] = 4;
            fl.n = 2;
        }
        if (launch_fill_multi(fl, s)) return -1;
    }
    if (!a.idf_by_df)
        k_idf_of_rank<<<grid_for(a.nterms ? a.nterms : 1), NT, 0, s>>>(a.df_of_rank, a.idf_idx, a.idf, a.nterms,
                                                                      a.idf_rank);
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const uint32_t wg_need = (a.ndocs + NT / 64 - 1) / (NT / 64);
    const bool wide = a.rank_bits + K5_IDX_BITS > 32;
    const uint32_t wg_cu = wide ? (uint32_t)K5_WPS_WIDE : 4u;   /* 40 KB LDS: 4 per CU; wide: its registers */
    const uint32_t wg = wg_need < (uint32_t)ncu * wg_cu ? wg_need : (uint32_t)ncu * wg_cu;
    const uint32_t grid = a.ndocs < 2048u ? a.ndocs : 2048u; /* persistent over the handed-off list */
    /* wide ranks (> 32 - K5_IDX_BITS bits): the wave kernel's instance that hands skewed
     * documents to k_score_large during the run, scored after it by a second k_score_large
     * over that list */
    K5Args hand = a;
    hand.cls_list = nullptr;
    if (!a.cls_list || !a.cls_off) return -1;
    k_k5_classify<<<a.cls_nblk, 256, 0, s>>>(a);
    if (scan_excl_u32(a.cls_off, a.cls_off, 3ull * a.cls_nblk + 1, ar, s)) return -1;
    k_k5_scatter<<<a.cls_nblk, 256, 0, s>>>(a);
    if (a.idf_by_df && !wide) return -1;   /* the engine sets idf_by_df only with wide ranks */
    if (a.idf_by_df) k_score_small<true><<<(unsigned)ncu * (unsigned)K5S_OCC, 256, 0, s>>>(a);
    else k_score_small<false><<<(unsigned)ncu * (unsigned)K5S_OCC, 256, 0, s>>>(a);
    /* k_score_large after the wave kernel on the same stream (beside it on the side stream,
     * round 5's A/B: c2 score 0.74 vs 0.76 ms but c4 3.18-3.29 vs 3.04-3.11 and c5 0.83 vs
     * 0.81) */
    launch_score_wave(a, wide, wg, s);
    if (a.split_count) launch_emit_split(a, ncu, s);
    launch_score_large(a, grid, s);
    if (wide) launch_score_large(hand, grid, s);
    return ok();
}

/* ------------------------------------------------------ multi-GPU union -- */

__global__ void k_keys_by_rank(const uint4* __restrict__ vkeys, const uint32_t* __restrict__ slot_of_rank, uint32_t V,
                               uint4* __restrict__ out) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < V) out[r] = vkeys[slot_of_rank[r]];
}
int launch_keys_by_rank(const uint4* vkeys, const uint32_t* slot_of_rank, uint32_t V, uint4* out, hipStream_t s) {
    if (!V) return 0;
    k_keys_by_rank<<<grid_for(V), NT, 0, s>>>(vkeys, slot_of_rank, V, out);
    return ok();
}
/* ---- the hash-owner DF exchange (engine.cpp exchange_collective) ----
 * Every term has one owner rank, picked by a hash of its identity key independent of the
 * vocabulary slot hash.  A rank sends (key, local df) of each of its terms to the term's
 * owner; the owner sums the df of equal keys in a hash table and answers every received
 * entry with the global df, in the order received.  Per rank that moves and aggregates
 * ~V_local entries, where the all-gather union it replaces sorted max V x nranks keys on
 * every rank. */
__device__ __forceinline__ uint32_t owner_of(const uint4 k, uint32_t R) {
    const uint64_t lo = ((uint64_t)k.y << 32) | k.x, hi = ((uint64_t)k.w << 32) | k.z;
    const uint64_t h = mix64(lo ^ (hi * 0x9E3779B97F4A7C15ull) ^ 0x5851F42D4C957F2Dull);
    return (uint32_t)(((h >> 32) * (uint64_t)R) >> 32);
}
constexpr uint32_t XO_MAXR = 1024;   /* ranks (tfidf_group_open's limit) */
/* term rank i's identity key from the vocabulary sort's keys (OwnerKeySrc): round 5 gathered
 * every key through the slot table (k_keys_by_rank: a random 16-byte read per term from a
 * table of ~3x the terms' size, 0.33-0.43 ms per rank at c4 / 8 shards).  Byte 15 of
 * a short identity key is 0x00 or 0x09 (dev_common.h); a long term's sort key holds its 16th
 * byte there, which is neither NUL nor whitespace. */
__device__ __forceinline__ uint4 owner_key(const OwnerKeySrc& ks, uint32_t i) {
    const uint4 s = gload(ks.skey + i);
    const uint32_t b15 = s.x & 0xFFu;
    if (b15 == 0x00u || b15 == 0x09u)
        return make_uint4(__builtin_bswap32(s.w), __builtin_bswap32(s.z), __builtin_bswap32(s.y), __builtin_bswap32(s.x));
    return gload(ks.vkeys + G(ks.slot_of_rank)[i]);
}
/* per-owner counts of this rank's terms (LDS histogram, one device atomic per block and owner) */
__global__ void k_owner_count(const OwnerKeySrc ks, uint32_t V, uint32_t R, uint32_t* __restrict__ cnt) {
    __shared__ uint32_t h[XO_MAXR];
    for (uint32_t o = threadIdx.x; o < R; o += blockDim.x) h[o] = 0;
    __syncthreads();
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < V; r += gridDim.x * blockDim.x)
        atomicAdd(&h[owner_of(owner_key(ks, r), R)], 1u);
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < R; o += blockDim.x)
        if (h[o]) atomicAdd(&cnt[o], h[o]);
}
/* The send buffer grouped by owner as 20-byte records (the 16-byte key and the local df:
 * one all-to-all instead of two); order inside an owner's segment is free (the replies come
 * back in send order, sidx maps them to term ranks).  cur[o] starts at 0. */
__global__ void k_owner_scatter(const OwnerKeySrc ks, const uint32_t* __restrict__ df, uint32_t V, uint32_t R,
                                const uint32_t* __restrict__ cnt, uint32_t* __restrict__ cur, uint32_t* __restrict__ srec,
                                uint32_t* __restrict__ sidx) {
    __shared__ uint32_t h[XO_MAXR], base[XO_MAXR], seg[XO_MAXR];
    /* segment starts: an exclusive scan of cnt (R <= 1024, serial per 256 entries is cheap) */
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t o = 0; o < R; ++o) { seg[o] = acc; acc += cnt[o]; }
    }
    for (uint32_t o = threadIdx.x; o < R; o += blockDim.x) h[o] = 0;
    __syncthreads();
    const uint32_t r0 = blockIdx.x * blockDim.x * 8;
    uint32_t own[8], pos[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const uint32_t r = r0 + q * blockDim.x + threadIdx.x;
        own[q] = r < V ? owner_of(owner_key(ks, r), R) : 0xFFFFFFFFu;
        pos[q] = own[q] != 0xFFFFFFFFu ? atomicAdd(&h[own[q]], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < R; o += blockDim.x) base[o] = h[o] ? seg[o] + atomicAdd(&cur[o], h[o]) : 0u;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const uint32_t r = r0 + q * blockDim.x + threadIdx.x;
        if (own[q] == 0xFFFFFFFFu) continue;
        const uint32_t p = base[own[q]] + pos[q];
        const uint4 k = owner_key(ks, r);
        uint32_t* d = srec + 5ull * p;
        d[0] = k.x; d[1] = k.y; d[2] = k.z; d[3] = k.w; d[4] = df[r];
        sidx[p] = r;
    }
}
/* owner side: find-or-insert of a received key into the owner's table (the claim protocol
 * of the vocabulary's vocab_insert_s: EMPTY -> PENDING by CAS, low word, then the high word
 * published); *claimed when this call inserted it.  The table holds >= 1.5x the received
 * entries, so a probe run ends.  One loop body for every case: a lane that finds a slot
 * PENDING re-reads it (at the memory side) in its next iteration, so a claiming lane of the
 * same wave publishes in the same pass of the body instead of waiting behind the spin; the
 * wait is bounded anyway (ST_VOCAB_SPIN, INVALID_SLOT). */
__device__ uint32_t owner_insert(uint4* __restrict__ keys, uint64_t mask, uint64_t klo, uint64_t khi, bool* claimed,
                                 uint32_t* status) {
    uint64_t h = key_hash(klo, khi) & mask;
    uint32_t spins = 0;
    bool reread = false;
    for (uint64_t probe = 0; probe <= mask;) {
        unsigned long long* slot = reinterpret_cast<unsigned long long*>(&keys[h]);
        uint64_t lo, hi;
        if (reread) {
            hi = atomicOr(&slot[1], 0ull);
            lo = atomicOr(&slot[0], 0ull);
        } else {
            const uint4 s = keys[h];
            lo = ((uint64_t)s.y << 32) | s.x;
            hi = ((uint64_t)s.w << 32) | s.z;
        }
        reread = false;
        if (hi == KEY_EMPTY_HI) {
            const unsigned long long old = atomicCAS(&slot[1], (unsigned long long)KEY_EMPTY_HI,
                                                     (unsigned long long)KEY_PENDING_HI);
            if (old == KEY_EMPTY_HI) {
                atomicExch(&slot[0], (unsigned long long)klo);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                atomicExch(&slot[1], (unsigned long long)khi);
                *claimed = true;
                return (uint32_t)h;
            }
            reread = true;                 /* another lane claimed it: look again */
            continue;
        }
        if (hi == KEY_PENDING_HI) {
            if (++spins > (1u << 22)) { atomicOr(status, ST_VOCAB_SPIN); return INVALID_SLOT; }
            __builtin_amdgcn_s_sleep(2);
            reread = true;
            continue;
        }
        /* a published hi carries its lo (lo is written first, both in one line) */
        if (hi == khi && lo == klo) return (uint32_t)h;
        h = (h + 1) & mask;
        ++probe;
    }
    return INVALID_SLOT;
}
/* find-only probe of a table filled by owner_insert (every key looked up is in it) */
__device__ uint32_t owner_find(const uint4* __restrict__ keys, uint64_t mask, uint64_t klo, uint64_t khi) {
    uint64_t h = key_hash(klo, khi) & mask;
    for (uint64_t probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
        const uint4 s = keys[h];
        const uint64_t lo = ((uint64_t)s.y << 32) | s.x, hi = ((uint64_t)s.w << 32) | s.z;
        if (hi == khi && lo == klo) return (uint32_t)h;
        if (hi == KEY_EMPTY_HI) break;
    }
    return INVALID_SLOT;
}
/* the segment of a position: last p with off[p] <= i (off: R + 1 prefix offsets) */
__device__ __forceinline__ uint32_t seg_of(const uint32_t* __restrict__ off, uint32_t R, uint64_t i) {
    uint32_t lo = 0, hi = R;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}
/* every received record into the owner's table, its df added; rslot[i] = the record's slot,
 * *used += distinct keys (one claim each) */
__global__ void k_owner_insert(const uint32_t* __restrict__ rrec, uint64_t n, uint4* __restrict__ tkey, uint64_t tmask,
                               uint32_t* __restrict__ tdf, uint32_t* __restrict__ rslot,
                               unsigned long long* __restrict__ used, uint32_t* __restrict__ status) {
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = i0 + threadIdx.x;
        bool claimed = false;
        if (i < n) {
            const uint32_t* r = rrec + 5 * i;
            const uint32_t sl = owner_insert(tkey, tmask, ((uint64_t)r[1] << 32) | r[0], ((uint64_t)r[3] << 32) | r[2],
                                             &claimed, status);
            if (sl == INVALID_SLOT) {   /* not reachable at the table's load (or a bounded wait gave up) */
                atomicOr(status, ST_BOUNDS);
                rslot[i] = 0u;
            } else {
                atomicAdd(&tdf[sl], r[4]);
                rslot[i] = sl;
            }
        }
        const uint32_t c = (uint32_t)__popcll(__ballot(claimed));
        if ((threadIdx.x & 63) == 0 && c) atomicAdd(used, (unsigned long long)c);
    }
}
/* The replies, one segment per sender p: the summed df of each of its records in the order
 * received, then one trailer word = this owner's distinct keys (its share of the global V),
 * so every sender learns global V from the same all-to-all (reply[roff[p] + p + i]). */
__global__ void k_owner_reply(const uint32_t* __restrict__ rslot, uint64_t n, const uint32_t* __restrict__ roff, uint32_t R,
                              const uint32_t* __restrict__ tdf, const unsigned long long* __restrict__ used,
                              uint32_t* __restrict__ reply) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) reply[i + seg_of(roff, R, i)] = tdf[rslot[i]];
    if (i < R) reply[(uint64_t)roff[i + 1] + i] = (uint32_t)*used;
}
/* sender side: the global df of each sent term back at its rank; global V = the owners'
 * trailers summed (back[soff[p] + p + i], trailer of owner p at soff[p + 1] + p) */
__global__ void k_owner_back(const uint32_t* __restrict__ back, const uint32_t* __restrict__ soff, uint32_t R,
                             const uint32_t* __restrict__ sidx, uint32_t V, uint32_t* __restrict__ df_global,
                             uint32_t* __restrict__ vg) {
    /* the segment search over an LDS copy of soff (a search in memory is a chain of dependent
     * loads per thread); segments are long, so most blocks lie in one and search nothing */
    __shared__ uint32_t so[XO_MAXR + 1];
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (R <= XO_MAXR) {
        for (uint32_t p = threadIdx.x; p <= R; p += blockDim.x) so[p] = soff[p];
        __syncthreads();
        if (j < V) {
            uint32_t lo = 0, hi = R;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (so[mid] <= j) lo = mid; else hi = mid;
            }
            df_global[sidx[j]] = back[j + lo];
        }
    } else if (j < V) {
        df_global[sidx[j]] = back[j + seg_of(soff, R, j)];
    }
    if (blockIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t p = threadIdx.x; p < R; p += blockDim.x) t += back[(uint64_t)soff[p + 1] + p];
        t = wave_sum(t);
        __shared__ uint32_t ws[NT / 64];
        if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = t;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t a = 0;
            for (int w = 0; w < NT / 64; ++w) a += ws[w];
            *vg = a;
        }
    }
}
/* prefix offsets of this rank's send (soff: its row of the all-gathered count matrix) and
 * receive (roff: its column) segments; m holds R rows of R counts + 1 status word */
__global__ void k_owner_offsets(const uint32_t* __restrict__ m, uint32_t R, uint32_t me, uint32_t* __restrict__ soff,
                                uint32_t* __restrict__ roff) {
    if (threadIdx.x == 0) {
        uint32_t a = 0, b = 0;
        for (uint32_t p = 0; p < R; ++p) {
            soff[p] = a;
            roff[p] = b;
            a += m[(uint64_t)me * (R + 1) + p];
            b += m[(uint64_t)p * (R + 1) + me];
        }
        soff[R] = a;
        roff[R] = b;
    }
}
int launch_owner_partition(const OwnerKeySrc& ks, const uint32_t* df, uint32_t V, uint32_t R, uint32_t* cnt, uint32_t* cur,
                           uint32_t* srec, uint32_t* sidx, hipStream_t s) {
    if (R < 1 || R > XO_MAXR) return -3;
    if (hipMemsetAsync(cnt, 0, (size_t)R * 4, s) != hipSuccess || hipMemsetAsync(cur, 0, (size_t)R * 4, s) != hipSuccess)
        return -1;
    if (!V) return 0;
    const uint32_t nb = (V + NT * 8 - 1) / (NT * 8);
    k_owner_count<<<nb < 1024 ? nb : 1024, NT, 0, s>>>(ks, V, R, cnt);
    k_owner_scatter<<<nb, NT, 0, s>>>(ks, df, V, R, cnt, cur, srec, sidx);
    return ok();
}
int launch_owner_offsets(const uint32_t* m, uint32_t R, uint32_t me, uint32_t* soff, uint32_t* roff, hipStream_t s) {
    k_owner_offsets<<<1, 64, 0, s>>>(m, R, me, soff, roff);
    return ok();
}
int launch_owner_aggregate(const uint32_t* rrec, uint64_t n, const uint32_t* roff, uint32_t R, uint4* tkey, uint64_t tcap,
                           uint32_t* tdf, uint32_t* rslot, uint32_t* reply, unsigned long long* used, uint32_t* status,
                           hipStream_t s) {
    if (hipMemsetAsync(tkey, 0xEE, tcap * 16, s) != hipSuccess || hipMemsetAsync(tdf, 0, tcap * 4, s) != hipSuccess ||
        hipMemsetAsync(used, 0, 8, s) != hipSuccess)
        return -1;
    if (n) {
        const uint64_t nb = (n + NT - 1) / NT;
        k_owner_insert<<<(unsigned)(nb < 8192 ? nb : 8192), NT, 0, s>>>(rrec, n, tkey, tcap - 1, tdf, rslot, used, status);
    }
    const uint64_t m = n > R ? n : R;
    k_owner_reply<<<grid_for(m), NT, 0, s>>>(rslot, n, roff, R, tdf, used, reply);
    return ok();
}
/* ---- the owner's aggregation, bucketed: the received records are grouped by the top bits
 * of their key hash into buckets of ~XB_MEAN records (every copy of a key in one bucket), then
 * one workgroup per bucket sums the df of equal keys in an LDS table and answers each record.
 * The grouping is an LSD radix sort of (bucket, record index) pairs (prims.hip: LDS-staged,
 * each tile's runs stored contiguously; 2 digit passes up to 2^16 buckets), not a scatter of
 * the records: round 4's per-record returning atomic for the bucket rank and its scattered
 * 24-byte stores (c4 at 8 shards: 1.2 ms of the owner's 2.1 ms) are gone, and the bucket
 * workgroups read the records in place through the sorted indices. */
constexpr uint32_t XB_MEAN = 512;    /* mean records per bucket (at most; 256 measured no faster at c4 /
                                        8 shards, profiles/r06_k1_ab_c2.txt call r06ad) */
constexpr uint32_t XB_T = 2048;      /* LDS slots of the largest table (4x the mean; a bucket's table is
                                        the power of two >= 2x its records, cleared per bucket) */
/* bucket = the top bits of a 64-bit mix (key_hash is 32-bit; its low bits pick the LDS slot),
 * independent of owner_of's mix */
__device__ __forceinline__ uint64_t xb_hash(const uint32_t* r) {
    const uint64_t lo = ((uint64_t)r[1] << 32) | r[0], hi = ((uint64_t)r[3] << 32) | r[2];
    return mix64(hi ^ (lo * 0xD6E8FEB86659FD93ull) ^ 0x2545F4914F6CDD1Dull);
}
/* (bucket, record index) pairs, the radix sort's input */
__global__ void k_xb_keys(const uint32_t* __restrict__ rrec, uint64_t n, uint32_t shift, uint64_t* __restrict__ key,
                          uint32_t* __restrict__ idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    key[i] = xb_hash(rrec + 5 * i) >> shift;
    idx[i] = (uint32_t)i;
}
/* off[b] = the first sorted position of bucket b (off[nb] = n) from the sorted bucket ids */
__global__ void k_xb_bounds(const uint64_t* __restrict__ key, uint64_t n, uint32_t nb, uint32_t* __restrict__ off) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t b = (uint32_t)key[p];
    const uint32_t prev = p ? (uint32_t)key[p - 1] : 0xFFFFFFFFu;
    for (uint32_t q = prev + 1; q <= b; ++q) off[q] = (uint32_t)p;   /* prev + 1 wraps to 0 at p = 0 */
    if (p == n - 1)
        for (uint32_t q = b + 1; q <= nb; ++q) off[q] = (uint32_t)n;
}
__device__ __forceinline__ uint4 xb_key_at(const uint32_t* __restrict__ rrec, uint32_t i) {
    const uint32_t* r = rrec + 5ull * i;
    return make_uint4(r[0], r[1], r[2], r[3]);
}
/* one workgroup per bucket (grid-stride over buckets).  Each thread loads its records (up to
 * XB_PER: index, key, df) once, in independent loads, and keeps them in registers; the keys
 * are also staged in LDS, so the find-or-claim probes compare keys without waiting on
 * memory: LDS slot -> the bucket-local index of the key's first copy + the summed df, and
 * each record is answered from the slot it found (reply[i + sender]).  A bucket of more
 * than XB_MAXREC records (not expected: the mean is <= XB_MEAN) takes the same steps with
 * the keys compared in memory. */
constexpr uint32_t XB_NT = 256;
constexpr uint32_t XB_MAXREC = 1024;
constexpr uint32_t XB_PER = XB_MAXREC / XB_NT;
__device__ __forceinline__ uint32_t xb_seg(const uint32_t* sroff, const uint32_t* __restrict__ roff, uint32_t R,
                                           uint32_t i) {
    uint32_t lo = 0, hi = R;
    if (R <= XO_MAXR) {
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sroff[mid] <= i) lo = mid; else hi = mid;
        }
        return lo;
    }
    return seg_of(roff, R, i);
}
__device__ __forceinline__ bool xb_eq(const uint4& a, const uint4& b) {
    return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
}
__device__ __forceinline__ uint32_t xb_home(const uint4& k, uint32_t tm) {
    return (uint32_t)key_hash(((uint64_t)k.y << 32) | k.x, ((uint64_t)k.w << 32) | k.z) & tm;
}
__global__ void __launch_bounds__(XB_NT) k_xb_bucket(const uint32_t* __restrict__ rrec, const uint32_t* __restrict__ sidx,
                                                     const uint32_t* __restrict__ off, uint32_t nb,
                                                     const uint32_t* __restrict__ roff, uint32_t R,
                                                     uint32_t* __restrict__ reply, unsigned long long* __restrict__ used,
                                                     uint32_t* __restrict__ status, uint32_t stage_max) {
    __shared__ uint4 skey[XB_MAXREC];
    __shared__ uint32_t tix[XB_T], tdf[XB_T];
    __shared__ uint32_t sroff[XO_MAXR + 1];
    for (uint32_t p = threadIdx.x; p <= R && p <= XO_MAXR; p += XB_NT) sroff[p] = roff[p];
    uint32_t claims = 0;
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t b0 = off[b], nrec = off[b + 1] - b0;
        uint32_t T = 256;
        while (T < 2 * nrec && T < XB_T) T *= 2;
        const uint32_t tm = T - 1;
        for (uint32_t t = threadIdx.x; t < T; t += XB_NT) { tix[t] = 0xFFFFFFFFu; tdf[t] = 0; }
        if (nrec <= stage_max) {
            uint32_t ii[XB_PER], dd[XB_PER], hh[XB_PER];
            uint4 kk[XB_PER];
#pragma unroll
            for (uint32_t q = 0; q < XB_PER; ++q) {
                const uint32_t j = threadIdx.x + q * XB_NT;
                ii[q] = j < nrec ? sidx[b0 + j] : 0u;
            }
#pragma unroll
            for (uint32_t q = 0; q < XB_PER; ++q) {
                const uint32_t j = threadIdx.x + q * XB_NT;
                if (j < nrec) {
                    kk[q] = xb_key_at(rrec, ii[q]);
                    dd[q] = rrec[5ull * ii[q] + 4];
                    skey[j] = kk[q];
                }
            }
            __syncthreads();
#pragma unroll
            for (uint32_t q = 0; q < XB_PER; ++q) {   /* find-or-claim, df added */
                const uint32_t j = threadIdx.x + q * XB_NT;
                hh[q] = 0xFFFFFFFFu;
                if (j >= nrec) continue;
                uint32_t h = xb_home(kk[q], tm);
                for (uint32_t probe = 0; probe < T; ++probe, h = (h + 1) & tm) {
                    uint32_t x = tix[h];
                    if (x == 0xFFFFFFFFu) {
                        x = atomicCAS(&tix[h], 0xFFFFFFFFu, j);
                        if (x == 0xFFFFFFFFu) { ++claims; hh[q] = h; break; }
                    }
                    if (xb_eq(skey[x], kk[q])) { hh[q] = h; break; }
                }
                if (hh[q] != 0xFFFFFFFFu) atomicAdd(&tdf[hh[q]], dd[q]);
                else atomicOr(status, ST_BOUNDS);   /* more distinct keys than slots in one bucket */
            }
            __syncthreads();
#pragma unroll
            for (uint32_t q = 0; q < XB_PER; ++q) {   /* the answers */
                const uint32_t j = threadIdx.x + q * XB_NT;
                if (j < nrec) reply[ii[q] + xb_seg(sroff, roff, R, ii[q])] = hh[q] != 0xFFFFFFFFu ? tdf[hh[q]] : 0u;
            }
        } else {
            __syncthreads();
            for (uint32_t j0 = 0; j0 < nrec; j0 += XB_NT) {   /* find-or-claim, df added */
                const uint32_t j = j0 + threadIdx.x;
                if (j >= nrec) continue;
                const uint32_t i = sidx[b0 + j];
                const uint4 k = xb_key_at(rrec, i);
                uint32_t h = xb_home(k, tm), probe = 0;
                for (; probe < T; ++probe, h = (h + 1) & tm) {
                    uint32_t x = tix[h];
                    if (x == 0xFFFFFFFFu) {
                        x = atomicCAS(&tix[h], 0xFFFFFFFFu, j);
                        if (x == 0xFFFFFFFFu) { ++claims; break; }
                    }
                    if (xb_eq(xb_key_at(rrec, sidx[b0 + x]), k)) break;
                }
                if (probe < T) atomicAdd(&tdf[h], rrec[5ull * i + 4]);
                else atomicOr(status, ST_BOUNDS);
            }
            __syncthreads();
            for (uint32_t j0 = 0; j0 < nrec; j0 += XB_NT) {   /* the answers */
                const uint32_t j = j0 + threadIdx.x;
                if (j >= nrec) continue;
                const uint32_t i = sidx[b0 + j];
                const uint4 k = xb_key_at(rrec, i);
                uint32_t h = xb_home(k, tm), d = 0;
                for (uint32_t probe = 0; probe < T; ++probe, h = (h + 1) & tm) {
                    const uint32_t x = tix[h];
                    if (x == 0xFFFFFFFFu) break;
                    if (xb_eq(xb_key_at(rrec, sidx[b0 + x]), k)) { d = tdf[h]; break; }
                }
                reply[i + xb_seg(sroff, roff, R, i)] = d;
            }
        }
        __syncthreads();   /* the table is cleared for the next bucket only after every lookup */
    }
    const uint32_t c = wave_sum(claims);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(used, (unsigned long long)c);
}
__global__ void k_xb_trailer(const uint32_t* __restrict__ roff, uint32_t R, const unsigned long long* __restrict__ used,
                             uint32_t* __restrict__ reply) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < R) reply[(uint64_t)roff[p + 1] + p] = (uint32_t)*used;
}
static uint32_t owner_buckets(uint64_t n) {   /* >= 2: the bucket is hash >> (64 - lg), lg >= 1 */
    uint32_t nb = 2;
    while ((uint64_t)nb * XB_MEAN < n && nb < (1u << 24)) nb *= 2;
    return nb;
}
static size_t xb_al(size_t b) { return (b + 255) & ~(size_t)255; }
size_t owner_bucket_scratch(uint64_t n) {
    /* sort keys 2 x 8n, indices 2 x 4n, bucket offsets, the sort's histograms + scan scratch */
    return 2 * xb_al(n * 8 + 8) + 2 * xb_al(n * 4 + 4) + xb_al(((size_t)owner_buckets(n) + 1) * 4) + n / 2 + (2u << 20);
}
int launch_owner_aggregate_buckets(const uint32_t* rrec, uint64_t n, const uint32_t* roff, uint32_t R, void* scratch,
                                   size_t scratch_bytes, uint32_t* reply, unsigned long long* used, uint32_t* status,
                                   uint32_t stage_max, hipStream_t s) {
    /* stage_max: buckets of up to this many records (<= XB_MAXREC) are staged in LDS; the
     * tests set 0 so that every bucket takes the path that compares keys in memory */
    if (stage_max > XB_MAXREC) stage_max = XB_MAXREC;
    const uint32_t nb = owner_buckets(n);
    uint32_t lg = 0;
    while ((1u << lg) < nb) ++lg;
    const uint32_t shift = 64 - lg;
    if (hipMemsetAsync(used, 0, 8, s) != hipSuccess) return -1;
    if (n) {
        if (n >= 0xFFFFFFFFull) return -2;
        if (scratch_bytes < owner_bucket_scratch(n)) return -2;
        uint8_t* p = (uint8_t*)scratch;
        uint64_t* k0 = (uint64_t*)p;  p += xb_al(n * 8 + 8);
        uint64_t* k1 = (uint64_t*)p;  p += xb_al(n * 8 + 8);
        uint32_t* v0 = (uint32_t*)p;  p += xb_al(n * 4 + 4);
        uint32_t* v1 = (uint32_t*)p;  p += xb_al(n * 4 + 4);
        uint32_t* off = (uint32_t*)p; p += xb_al(((size_t)nb + 1) * 4);
        Arena ar;
        ar.base = p;
        ar.cap = scratch_bytes - (size_t)(p - (uint8_t*)scratch);
        const unsigned g = (unsigned)((n + NT - 1) / NT);
        k_xb_keys<<<g, NT, 0, s>>>(rrec, n, shift, k0, v0);
        const uint32_t mask = lg <= 8 ? 0x1u : lg <= 16 ? 0x3u : 0x7u;
        const int cur = radix_sort_u64(k0, v0, k1, v1, n, mask, ar, s);
        if (cur < 0) return cur == -2 ? -2 : -1;
        const uint64_t* ks = cur ? k1 : k0;
        const uint32_t* vs = cur ? v1 : v0;
        k_xb_bounds<<<g, NT, 0, s>>>(ks, n, nb, off);
        k_xb_bucket<<<nb < 8192 ? nb : 8192, XB_NT, 0, s>>>(rrec, vs, off, nb, roff, R, reply, used, status, stage_max);
    }
    k_xb_trailer<<<(R + NT - 1) / NT, NT, 0, s>>>(roff, R, used, reply);
    return ok();
}
int launch_owner_back(const uint32_t* back, const uint32_t* soff, uint32_t R, const uint32_t* sidx, uint32_t V,
                      uint32_t* df_global, uint32_t* vg, hipStream_t s) {
    k_owner_back<<<grid_for(V > 1 ? V : 1), NT, 0, s>>>(back, soff, R, sidx, V, df_global, vg);
    return ok();
}

/* ---- the dense DF exchange (north_star's form: per-rank DF vectors over one shared
 * vocabulary, summed by an all-reduce).  Every rank all-gathers the ranks' term keys
 * (each rank's list padded to the largest V with EMPTY keys), inserts them all into a table
 * and numbers each distinct key by the smallest position it has in the gathered list: the
 * same numbering on every rank with no further exchange.  Each rank scatters its local df
 * into a dense vector over those positions, the vectors are all-reduced (sum), and each rank
 * reads back its terms' global df; global V = the table's distinct keys. */
__global__ void k_dense_insert(const uint4* __restrict__ gkeys, uint64_t n, uint4* __restrict__ tkey, uint64_t tmask,
                               uint32_t* __restrict__ tpos, unsigned long long* __restrict__ used,
                               uint32_t* __restrict__ status) {
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = i0 + threadIdx.x;
        bool claimed = false;
        if (i < n) {
            const uint4 k = gkeys[i];
            const uint64_t hi = ((uint64_t)k.w << 32) | k.z;
            if (hi != KEY_EMPTY_HI) {   /* padding */
                const uint32_t sl = owner_insert(tkey, tmask, ((uint64_t)k.y << 32) | k.x, hi, &claimed, status);
                if (sl == INVALID_SLOT) atomicOr(status, ST_BOUNDS);
                else atomicMin(&tpos[sl], (uint32_t)i);
            }
        }
        const uint32_t c = (uint32_t)__popcll(__ballot(claimed));
        if ((threadIdx.x & 63) == 0 && c) atomicAdd(used, (unsigned long long)c);
    }
}
__global__ void k_dense_scatter(const uint4* __restrict__ mine, const uint32_t* __restrict__ df, uint32_t V,
                                const uint4* __restrict__ tkey, uint64_t tmask, const uint32_t* __restrict__ tpos,
                                uint32_t* __restrict__ pos, uint32_t* __restrict__ dense, uint32_t* __restrict__ status) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= V) return;
    const uint4 k = mine[r];
    const uint32_t sl = owner_find(tkey, tmask, ((uint64_t)k.y << 32) | k.x, ((uint64_t)k.w << 32) | k.z);
    if (sl == INVALID_SLOT) { atomicOr(status, ST_BOUNDS); pos[r] = 0; return; }
    const uint32_t p = tpos[sl];
    pos[r] = p;
    dense[p] = df[r];   /* one term per position: the keys of a rank are distinct */
}
__global__ void k_dense_gather(const uint32_t* __restrict__ dense, const uint32_t* __restrict__ pos, uint32_t V,
                               uint32_t* __restrict__ df_global) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < V) df_global[r] = dense[pos[r]];
}
__global__ void k_sum_rows_u32(const uint32_t* __restrict__ rows, uint32_t nrows, uint64_t n, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t t = 0;
    for (uint32_t r = 0; r < nrows; ++r) t += rows[(uint64_t)r * n + i];
    out[i] = t;
}
int launch_sum_rows_u32(const uint32_t* rows, uint32_t nrows, uint64_t n, uint32_t* out, hipStream_t s) {
    if (!n) return 0;
    k_sum_rows_u32<<<grid_for(n), NT, 0, s>>>(rows, nrows, n, out);
    return ok();
}
/* every word of every segment, in tiles of XC_TILE words (grid-stride over tiles).  A tile
 * inside one segment (nearly all: segments are long) finds it by one block-uniform search and
 * moves its words with XC_PER independent coalesced loads per thread, then the stores; a
 * tile across a boundary searches per word.  (Round 5 searched the kernel-argument offsets
 * per word — a chain of dependent loads for every 4 bytes: 8 concurrent 98 MB copies at
 * c4 / 8 shards took ~1 ms.) */
constexpr uint32_t XC_PER = 4;
constexpr uint32_t XC_TILE = NT * XC_PER;
__global__ __launch_bounds__(NT) void k_xcopy(const XCopyList l) {
    const uint64_t total = l.off[l.n];
    for (uint64_t t0 = (uint64_t)blockIdx.x * XC_TILE; t0 < total; t0 += (uint64_t)gridDim.x * XC_TILE) {
        uint32_t lo = 0, hi = l.n;   /* last segment with off <= t0 (uniform) */
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (l.off[mid] <= t0) lo = mid; else hi = mid;
        }
        if (t0 + XC_TILE <= l.off[lo + 1]) {
            const uint32_t* src = l.src[lo] + (t0 - l.off[lo]);
            uint32_t* dst = l.dst[lo] + (t0 - l.off[lo]);
            uint32_t v[XC_PER];
#pragma unroll
            for (uint32_t q = 0; q < XC_PER; ++q) v[q] = __builtin_nontemporal_load(src + q * NT + threadIdx.x);
#pragma unroll
            for (uint32_t q = 0; q < XC_PER; ++q) dst[q * NT + threadIdx.x] = v[q];   /* read next by the receiver */
            continue;
        }
        for (uint32_t q = 0; q < XC_PER; ++q) {
            const uint64_t i = t0 + q * NT + threadIdx.x;
            if (i >= total) break;
            uint32_t a = lo, b = l.n;
            while (b - a > 1) {
                const uint32_t mid = (a + b) >> 1;
                if (l.off[mid] <= i) a = mid; else b = mid;
            }
            l.dst[a][i - l.off[a]] = l.src[a][i - l.off[a]];
        }
    }
}
__global__ void k_xsum_slice(const XCopyList l, uint64_t lo, uint64_t len, uint32_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t t = 0;
        for (uint32_t r = 0; r < l.n; ++r) t += l.src[r][lo + i];
        out[i] = t;
    }
}
static unsigned xgrid(uint64_t n) {
    const uint64_t b = (n + NT - 1) / NT;
    return (unsigned)(b < 4096 ? (b ? b : 1) : 4096);
}
int launch_xcopy(const XCopyList& l, hipStream_t s) {
    if (l.n < 1 || l.n > XCOPY_MAX) return -3;
    if (!l.off[l.n]) return 0;
    k_xcopy<<<xgrid((l.off[l.n] + XC_PER - 1) / XC_PER), NT, 0, s>>>(l);
    return ok();
}
int launch_xsum_slice(const XCopyList& l, uint64_t lo, uint64_t len, uint32_t* out, hipStream_t s) {
    if (l.n < 1 || l.n > XCOPY_MAX) return -3;
    if (!len) return 0;
    k_xsum_slice<<<xgrid(len), NT, 0, s>>>(l, lo, len, out);
    return ok();
}
int launch_dense_ids(const uint4* gkeys, uint64_t n, uint4* tkey, uint32_t* tpos, uint64_t tcap,
                     unsigned long long* used, uint32_t* status, hipStream_t s) {
    if (hipMemsetAsync(tkey, 0xEE, tcap * 16, s) != hipSuccess || hipMemsetAsync(tpos, 0xFF, tcap * 4, s) != hipSuccess ||
        hipMemsetAsync(used, 0, 8, s) != hipSuccess)
        return -1;
    if (n) {
        const uint64_t nb = (n + NT - 1) / NT;
        k_dense_insert<<<(unsigned)(nb < 8192 ? nb : 8192), NT, 0, s>>>(gkeys, n, tkey, tcap - 1, tpos, used, status);
    }
    return ok();
}
int launch_dense_scatter(const uint4* mine, const uint32_t* df, uint32_t V, const uint4* tkey, uint64_t tcap,
                         const uint32_t* tpos, uint32_t* pos, uint32_t* dense, uint32_t* status, hipStream_t s) {
    if (!V) return 0;
    k_dense_scatter<<<grid_for(V), NT, 0, s>>>(mine, df, V, tkey, tcap - 1, tpos, pos, dense, status);
    return ok();
}
int launch_dense_gather(const uint32_t* dense, const uint32_t* pos, uint32_t V, uint32_t* df_global, hipStream_t s) {
    if (!V) return 0;
    k_dense_gather<<<grid_for(V), NT, 0, s>>>(dense, pos, V, df_global);
    return ok();
}

/* ---- cross-rank identity of long terms (kernels.h LongEnt).  Within a rank a long term's
 * key match is verified against the incumbent's bytes (dev_vocab.h); across ranks the DF
 * exchange matches keys only, so every key that two ranks share is checked here against the
 * terms' bytes, as TFIDF.c:229's strcmp would compare them. */
__global__ void k_long_list(const uint4* __restrict__ vkeys, const uint64_t* __restrict__ vrep,
                            const uint32_t* __restrict__ slot_of_rank, uint32_t V, LongEnt* __restrict__ ents,
                            uint64_t* __restrict__ src, unsigned long long* __restrict__ cnt) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= V) return;
    const uint32_t sl = slot_of_rank[r];
    const uint4 k = vkeys[sl];
    if ((k.w >> 24) != 0xFFu) return;   /* short term: its key is its bytes */
    const uint64_t rep = vrep[sl];      /* (length << 40) | corpus offset of one occurrence */
    const uint32_t len = (uint32_t)(rep >> 40);
    const unsigned long long e = atomicAdd(&cnt[0], 1ull);
    const unsigned long long b = atomicAdd(&cnt[1], (unsigned long long)len);
    LongEnt x;
    x.key = k;
    x.len = len;
    x.pad = 0;
    x.boff = b;
    ents[e] = x;
    src[e] = rep & ((1ull << 40) - 1ull);
}
/* one wave per entry: its bytes from the corpus into the rank's blob */
__global__ void k_long_bytes(const LongEnt* __restrict__ ents, const uint64_t* __restrict__ src, uint32_t n,
                             const uint8_t* __restrict__ bytes, uint8_t* __restrict__ blob) {
    const uint32_t e = blockIdx.x * (NT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (e >= n) return;
    const uint64_t s0 = src[e], d0 = ents[e].boff;
    const uint32_t len = ents[e].len;
    for (uint32_t i = lane; i < len; i += 64) blob[d0 + i] = bytes[s0 + i];
}
__global__ void k_long_insert(const LongEnt* __restrict__ g, uint64_t n, uint4* __restrict__ tkey, uint64_t tmask,
                              uint32_t* __restrict__ tpos, uint32_t* __restrict__ status) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 k = g[i].key;
        const uint64_t hi = ((uint64_t)k.w << 32) | k.z;
        if (hi == KEY_EMPTY_HI) continue;   /* padding */
        bool claimed = false;
        const uint32_t sl = owner_insert(tkey, tmask, ((uint64_t)k.y << 32) | k.x, hi, &claimed, status);
        if (sl == INVALID_SLOT) atomicOr(status, ST_BOUNDS);
        else atomicMin(&tpos[sl], (uint32_t)i);
    }
}
/* one wave per gathered entry: against the first entry of its key (the smallest gathered
 * index), length and bytes */
__global__ void k_long_verify(const LongEnt* __restrict__ g, uint64_t n, uint64_t lcap, const uint8_t* __restrict__ gblob,
                              uint64_t bcap, const uint4* __restrict__ tkey, uint64_t tmask,
                              const uint32_t* __restrict__ tpos, uint32_t* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (i >= n) return;
    const LongEnt a = g[i];
    const uint64_t hi = ((uint64_t)a.key.w << 32) | a.key.z;
    if (hi == KEY_EMPTY_HI) return;
    const uint32_t sl = owner_find(tkey, tmask, ((uint64_t)a.key.y << 32) | a.key.x, hi);
    if (sl == INVALID_SLOT) { if (lane == 0) atomicOr(status, ST_BOUNDS); return; }
    const uint64_t j = tpos[sl];
    if (j == i) return;   /* the key's first entry */
    const LongEnt b = g[j];
    bool diff = a.len != b.len;
    if (!diff) {
        const uint8_t* pa = gblob + (i / lcap) * bcap + a.boff;
        const uint8_t* pb = gblob + (j / lcap) * bcap + b.boff;
        for (uint32_t k = lane; k < a.len && !diff; k += 64) diff = pa[k] != pb[k];
    }
    if (__ballot(diff) != 0ull && lane == 0) atomicOr(status, ST_LONG_COLLIDE);
}
int launch_long_list(const uint4* vkeys, const uint64_t* vrep, const uint32_t* slot_of_rank, uint32_t V, LongEnt* ents,
                     uint64_t* src, unsigned long long* cnt, hipStream_t s) {
    if (hipMemsetAsync(cnt, 0, 16, s) != hipSuccess) return -1;
    if (!V) return 0;
    k_long_list<<<grid_for(V), NT, 0, s>>>(vkeys, vrep, slot_of_rank, V, ents, src, cnt);
    return ok();
}
int launch_long_bytes(const LongEnt* ents, const uint64_t* src, uint32_t n, const uint8_t* bytes, uint8_t* blob,
                      hipStream_t s) {
    if (!n) return 0;
    k_long_bytes<<<(n + NT / 64 - 1) / (NT / 64), NT, 0, s>>>(ents, src, n, bytes, blob);
    return ok();
}
int launch_long_verify(const LongEnt* g, uint64_t n, uint64_t lcap, const uint8_t* gblob, uint64_t bcap, uint4* tkey,
                       uint32_t* tpos, uint64_t tcap, uint32_t* status, hipStream_t s) {
    if (hipMemsetAsync(tkey, 0xEE, tcap * 16, s) != hipSuccess || hipMemsetAsync(tpos, 0xFF, tcap * 4, s) != hipSuccess)
        return -1;
    if (!n) return 0;
    const uint64_t nb = (n + NT - 1) / NT;
    k_long_insert<<<(unsigned)(nb < 8192 ? nb : 8192), NT, 0, s>>>(g, n, tkey, tcap - 1, tpos, status);
    if (hipGetLastError() != hipSuccess) return -1;
    const uint64_t wb = (n + NT / 64 - 1) / (NT / 64);
    if (wb > 0x7FFFFFFFull) return -3;
    k_long_verify<<<(unsigned)wb, NT, 0, s>>>(g, n, lcap, gblob, bcap, tkey, tcap - 1, tpos, status);
    return ok();
}

/* ---- the dense exchange's merge numbering (no rank holds terms of >= 16 bytes).  Then
 * every rank's key list is in term order (its rank order = the big-endian byte order of
 * the identity keys, k_vocab_compact), so a term's number can be its position in the merged
 * lists: pos(k) = sum over ranks q of lb_q(k), the keys of list q below k.  Equal keys get
 * equal numbers, distinct keys distinct ones (for a < b, lb_q(a) <= lb_q(b) on every list
 * and < on the list holding a), all in [0, sum V).  A key is counted for global V by the
 * first rank holding it (no list q < me holds it).  No table, no clears: R binary searches
 * per term over the gathered lists (each padded to maxv with all-ones keys, above every
 * short key since those hold a TAB). */
__device__ __forceinline__ void term_order(const uint4 k, uint64_t& a, uint64_t& b) {
    a = bswap64(((uint64_t)k.y << 32) | k.x);
    b = bswap64(((uint64_t)k.w << 32) | k.z);
}
/* lbm[q V + i] = lb_q(key i) | 2^31 if q < me holds it */
__global__ void k_dense_lb(const uint4* __restrict__ gkeys, uint64_t maxv, uint32_t me, uint32_t V,
                           uint32_t* __restrict__ lbm) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t q = blockIdx.y;
    if (i >= V) return;
    uint32_t lb = i;   /* own list: key i is at position i */
    bool held = false;
    if (q != me) {
        const uint4* L = gkeys + (uint64_t)q * maxv;
        uint64_t ka, kb;
        term_order(gkeys[(uint64_t)me * maxv + i], ka, kb);
        uint32_t lo = 0, n = (uint32_t)maxv;
        while (n) {   /* first position whose key is >= key i */
            const uint32_t h = n >> 1;
            uint64_t a, b;
            term_order(L[lo + h], a, b);
            if (a < ka || (a == ka && b < kb)) { lo += h + 1; n -= h + 1; }
            else n = h;
        }
        lb = lo;
        if (q < me && lo < maxv) {
            uint64_t a, b;
            term_order(L[lo], a, b);
            held = a == ka && b == kb;
        }
    }
    lbm[(uint64_t)q * V + i] = lb | (held ? 0x80000000u : 0u);
}
/* pos[i] = sum of the lb's; dense[pos] = df; dense[sumv] += keys first held here */
__global__ void k_dense_merge_scatter(const uint32_t* __restrict__ lbm, uint32_t R, uint32_t V,
                                      const uint32_t* __restrict__ df, uint64_t sumv, uint32_t* __restrict__ pos,
                                      uint32_t* __restrict__ dense) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t p = 0, held = 0;
    if (i < V) {
        for (uint32_t q = 0; q < R; ++q) {
            const uint32_t x = lbm[(uint64_t)q * V + i];
            p += x & 0x7FFFFFFFu;
            held |= x >> 31;
        }
        pos[i] = p;
        dense[p] = df[i];
    }
    const uint32_t first = (uint32_t)__popcll(__ballot(i < V && !held));
    if ((threadIdx.x & 63) == 0 && first) atomicAdd(&dense[sumv], first);
}
int launch_dense_merge_ids(const uint4* gkeys, uint64_t maxv, uint32_t R, uint32_t me, uint32_t V, uint32_t* lbm,
                           const uint32_t* df, uint64_t sumv, uint32_t* pos, uint32_t* dense, hipStream_t s) {
    if (!V) return 0;
    if (maxv >= 0x80000000ull || sumv >= 0x80000000ull || R > 65535u) return -2;
    k_dense_lb<<<dim3((V + NT - 1) / NT, R), NT, 0, s>>>(gkeys, maxv, me, V, lbm);
    k_dense_merge_scatter<<<grid_for(V), NT, 0, s>>>(lbm, R, V, df, sumv, pos, dense);
    return ok();
}

/* ------------------------------------------------------------- synthetic -- */

__device__ __forceinline__ uint32_t blk_doc(const uint64_t* blk_first, uint32_t ndocs, uint64_t b) {
    uint32_t lo = 0, hi = ndocs + 1; /* last i with blk_first[i] <= b */
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (blk_first[mid] <= b) lo = mid + 1; else hi = mid;
    }
    return lo - 1;
}
__global__ void k_synth_bytes(syn_spec sp, const uint32_t* __restrict__ ids, const uint64_t* __restrict__ ntok,
                              const uint64_t* __restrict__ blk_first, uint64_t nblocks, uint32_t ndocs,
                              uint64_t* __restrict__ out) {
    uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    uint32_t i = blk_doc(blk_first, ndocs, b);
    uint64_t id = ids ? ids[i] : (uint64_t)i + 1;
    out[b] = syn_block_bytes(&sp, id, ntok[i], b - blk_first[i]);
}
__global__ void k_synth_fill(syn_spec sp, const uint32_t* __restrict__ ids, const uint64_t* __restrict__ ntok,
                             const uint64_t* __restrict__ blk_first, uint64_t nblocks, uint32_t ndocs,
                             const uint64_t* __restrict__ blk_off, uint8_t* __restrict__ bytes) {
    uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    uint32_t i = blk_doc(blk_first, ndocs, b);
    uint64_t id = ids ? ids[i] : (uint64_t)i + 1;
    syn_block_fill(&sp, id, ntok[i], b - blk_first[i], bytes + blk_off[b]);
}
__global__ void k_synth_docoff(const uint64_t* __restrict__ blk_first, uint32_t ndocs,
                               const uint64_t* __restrict__ blk_off, uint64_t* __restrict__ doc_off) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= ndocs) doc_off[i] = blk_off[blk_first[i]];
}
int launch_synth_bytes(const void* spec, const uint32_t* doc_ids, const uint64_t* ntok, const uint64_t* blk_first,
                       uint64_t nblocks, uint32_t ndocs, uint64_t* blk_bytes, hipStream_t s) {
    if (!nblocks) return 0;
    k_synth_bytes<<<grid_for(nblocks, 64), 64, 0, s>>>(*(const syn_spec*)spec, doc_ids, ntok, blk_first, nblocks,
                                                      ndocs, blk_bytes);
    return ok();
}
int launch_synth_fill(const void* spec, const uint32_t* doc_ids, const uint64_t* ntok, const uint64_t* blk_first,
                      uint64_t nblocks, uint32_t ndocs, const uint64_t* blk_off, uint8_t* bytes, uint64_t* doc_off,
                      hipStream_t s) {
    if (nblocks)
        k_synth_fill<<<grid_for(nblocks, 64), 64, 0, s>>>(*(const syn_spec*)spec, doc_ids, ntok, blk_first, nblocks,
                                                         ndocs, blk_off, bytes);
    k_synth_docoff<<<grid_for((uint64_t)ndocs + 1), NT, 0, s>>>(blk_first, ndocs, blk_off, doc_off);
    return ok();
}
