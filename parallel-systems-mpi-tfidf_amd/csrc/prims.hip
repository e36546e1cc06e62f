/*
 * prims.hip — device-wide primitives for the TF-IDF path (gfx950, wave64):
 *   exclusive scan (u32/u64), LSD radix sort of (u64|u128 key, u32 value) pairs with
 *   8-bit digits and a stable wave64 multisplit (8 ballots per digit), and the
 *   varying-byte probe that lets callers skip constant digit passes.
 */
#include "prims.h"
#include "dev_common.h"

namespace {

constexpr int SC_NT = 256;
constexpr int SC_IT = 8;
constexpr int SC_TILE = SC_NT * SC_IT;

template <typename T>
__device__ __forceinline__ T wave_incl_scan_t(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T block_excl_scan_t(T v, T* wsum, T* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    T inc = wave_incl_scan_t(v);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    T base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < SC_NT / 64; ++k) {
        T s = wsum[k];
        base += (k < w) ? s : (T)0;
        tot += s;
    }
    *total = tot;
    __syncthreads();
    return base + inc - v;
}

template <typename T>
__global__ __launch_bounds__(SC_NT) void k_scan_reduce(const T* __restrict__ in, uint64_t n, T* __restrict__ bsum) {
    __shared__ T wsum[SC_NT / 64];
    uint64_t base = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_IT;
    T s = 0;
#pragma unroll
    for (int j = 0; j < SC_IT; ++j)
        if (base + j < n) s += in[base + j];
    T tot;
    (void)block_excl_scan_t<T>(s, wsum, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

template <typename T>
__global__ __launch_bounds__(SC_NT) void k_scan_apply(const T* in, T* out, uint64_t n, const T* __restrict__ boff) {
    __shared__ T wsum[SC_NT / 64];
    uint64_t base = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_IT;
    T v[SC_IT];
    T s = 0;
#pragma unroll
    for (int j = 0; j < SC_IT; ++j) {
        v[j] = (base + j < n) ? in[base + j] : (T)0;
        s += v[j];
    }
    T tot;
    T run = block_excl_scan_t<T>(s, wsum, &tot) + (boff ? boff[blockIdx.x] : (T)0);
#pragma unroll
    for (int j = 0; j < SC_IT; ++j) {
        if (base + j < n) out[base + j] = run;
        run += v[j];
        if (base + j + 1 == n) out[n] = run;
    }
}

/* the apply pass that sums the block totals before it itself (up to SC_FUSED_MAXNB blocks:
 * each block reads at most that many words), instead of a separate scan launch over them */
constexpr uint64_t SC_FUSED_MAXNB = 1024;
template <typename T>
__global__ __launch_bounds__(SC_NT) void k_scan_apply_fused(const T* in, T* out, uint64_t n, const T* __restrict__ bsum) {
    __shared__ T wsum[SC_NT / 64];
    T pre = 0;
    for (uint32_t k = threadIdx.x; k < blockIdx.x; k += SC_NT) pre += bsum[k];
    T boff;
    (void)block_excl_scan_t<T>(pre, wsum, &boff);
    const uint64_t base = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_IT;
    T v[SC_IT];
    T s = 0;
#pragma unroll
    for (int j = 0; j < SC_IT; ++j) {
        v[j] = (base + j < n) ? in[base + j] : (T)0;
        s += v[j];
    }
    T tot;
    T run = block_excl_scan_t<T>(s, wsum, &tot) + boff;
#pragma unroll
    for (int j = 0; j < SC_IT; ++j) {
        if (base + j < n) out[base + j] = run;
        run += v[j];
        if (base + j + 1 == n) out[n] = run;
    }
}

template <typename T>
int scan_excl_t(const T* in, T* out, uint64_t n, Arena& ar, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(out, 0, sizeof(T), s) == hipSuccess ? 0 : -1;
    uint64_t nb = (n + SC_TILE - 1) / SC_TILE;
    if (nb == 1) {
        k_scan_apply<T><<<1, SC_NT, 0, s>>>(in, out, n, nullptr);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    size_t m = ar.mark();
    T* bsum = (T*)ar.get((nb + 1) * sizeof(T));
    if (!bsum) return -2;
    k_scan_reduce<T><<<(unsigned)nb, SC_NT, 0, s>>>(in, n, bsum);
    if (nb <= SC_FUSED_MAXNB) {   /* two launches instead of three */
        k_scan_apply_fused<T><<<(unsigned)nb, SC_NT, 0, s>>>(in, out, n, bsum);
        ar.release(m);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    int rc = scan_excl_t<T>(bsum, bsum, nb, ar, s);
    if (rc) return rc;
    k_scan_apply<T><<<(unsigned)nb, SC_NT, 0, s>>>(in, out, n, bsum);
    ar.release(m);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* ------------------------------------------------------------ radix sort ---- */

constexpr int RS_NT = 256;
constexpr int RS_IT = 8;
constexpr int RS_TILE = RS_NT * RS_IT;
constexpr uint32_t RS_FUSED_MAXNB = 1024; /* up to 2M keys: each scatter block reads nb histogram words per digit */

__device__ __forceinline__ uint32_t digit_of(uint64_t k, int p) { return (uint32_t)(k >> (8 * p)) & 0xFFu; }
__device__ __forceinline__ uint32_t digit_of(uint4 k, int p) {
    uint32_t w = (p < 4) ? k.x : (p < 8) ? k.y : (p < 12) ? k.z : k.w;
    return (w >> (8 * (p & 3))) & 0xFFu;
}

template <typename K>
__global__ __launch_bounds__(RS_NT) void k_rs_hist(const K* __restrict__ keys, uint64_t n, int p,
                                                  uint32_t* __restrict__ hist, uint32_t nblocks) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    uint64_t base = (uint64_t)blockIdx.x * RS_TILE + threadIdx.x;
#pragma unroll
    for (int j = 0; j < RS_IT; ++j) {
        uint64_t idx = base + (uint64_t)j * RS_NT;
        if (idx < n) atomicAdd(&h[digit_of(keys[idx], p)], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

/* One digit pass of the LSD sort over a tile of RS_TILE keys: a stable local counting
 * sort in LDS, then coalesced stores.  Wave w owns the tile's items [w * 512, w * 512 + 512)
 * in eight rounds of 64; each round's lanes find the lanes with the same digit by eight
 * ballots (a wave64 multisplit) and take their rank from the wave's running per-digit
 * counter (wave-private: no barrier per round).  The per-digit counts of the four waves
 * then give every item its position in the tile's digit-sorted order, the keys are staged
 * there in LDS, and each thread writes staged items tid, tid + 256, ...: consecutive
 * threads store consecutive positions of one digit's run (the previous scatter stored
 * every key straight from its lane, one scattered 16-byte store per key, with three
 * block barriers per 256 keys).  Global position = the tile's base for the digit (the
 * digit-major scan of the per-tile histograms) + the offset inside the run. */
template <typename K, bool FUSED>
__global__ __launch_bounds__(RS_NT) void k_rs_scatter(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                     K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                     uint64_t n, int p, const uint32_t* __restrict__ offs,
                                                     uint32_t nblocks) {
    __shared__ K sk[RS_TILE];
    __shared__ uint32_t sv[RS_TILE];
    __shared__ uint32_t wc[RS_NT / 64][256];   /* per-wave running counts, then per-wave prefixes */
    __shared__ uint32_t dstart[256];           /* tile-local start of each digit's run */
    __shared__ uint32_t gbase[256];            /* global position of the run */
    __shared__ uint32_t wsum[RS_NT / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int q = 0; q < RS_NT / 64; ++q) wc[q][tid] = 0;
    if (FUSED) {
        /* offs is the raw digit-major histogram: this block's base for digit tid is the
         * count of smaller digits everywhere plus digit tid in earlier blocks */
        const uint32_t* row = offs + (uint64_t)tid * nblocks;
        uint32_t pre = 0, tot = 0;
        uint32_t b = 0;
        for (; b + 16 <= nblocks; b += 16) { /* 16 loads in flight per step */
            uint32_t c[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) c[q] = row[b + q];
#pragma unroll
            for (int q = 0; q < 16; ++q) { pre += b + q < blockIdx.x ? c[q] : 0u; tot += c[q]; }
        }
        for (; b < nblocks; ++b) {
            const uint32_t c = row[b];
            pre += b < blockIdx.x ? c : 0u;
            tot += c;
        }
        uint32_t all;
        gbase[tid] = block_excl_scan<RS_NT>(tot, wsum, &all) + pre;
    } else {
        gbase[tid] = offs[(uint64_t)tid * nblocks + blockIdx.x];
        __syncthreads();
    }
    const uint64_t t0 = (uint64_t)blockIdx.x * RS_TILE;
    const uint64_t wb = t0 + (uint64_t)w * (RS_IT * 64);
    const uint64_t lt = (1ull << lane) - 1ull;
    K k[RS_IT];
    uint32_t v[RS_IT], d[RS_IT], r[RS_IT];
#pragma unroll
    for (int j = 0; j < RS_IT; ++j) {
        const uint64_t idx = wb + (uint64_t)j * 64 + lane;
        const bool valid = idx < n;
        k[j] = valid ? kin[idx] : K{};
        v[j] = valid ? vin[idx] : 0u;
        d[j] = valid ? digit_of(k[j], p) : 0u;
    }
#pragma unroll
    for (int j = 0; j < RS_IT; ++j) {
        const bool valid = wb + (uint64_t)j * 64 + lane < n;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d[j] >> b) & 1u;
            const uint64_t bb = __ballot(valid && bit);
            m &= bit ? bb : ~bb;
        }
        const uint32_t lrank = (uint32_t)__popcll(m & lt);
        /* the wave's LDS operations run in order: every lane reads the counter before the
         * group leader adds the group's size */
        r[j] = valid ? wc[w][d[j]] + lrank : 0u;
        if (valid && lrank == 0) wc[w][d[j]] += (uint32_t)__popcll(m);
    }
    __syncthreads();
    {   /* thread tid = digit tid: wave prefixes and the tile-local run start */
        uint32_t c[RS_NT / 64], tot = 0;
#pragma unroll
        for (int q = 0; q < RS_NT / 64; ++q) { c[q] = wc[q][tid]; wc[q][tid] = tot; tot += c[q]; }
        uint32_t all;
        dstart[tid] = block_excl_scan<RS_NT>(tot, wsum, &all);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RS_IT; ++j) {
        if (wb + (uint64_t)j * 64 + lane >= n) continue;
        const uint32_t pos = dstart[d[j]] + wc[w][d[j]] + r[j];
        sk[pos] = k[j];
        sv[pos] = v[j];
    }
    __syncthreads();
    const uint32_t tn = n - t0 < (uint64_t)RS_TILE ? (uint32_t)(n - t0) : (uint32_t)RS_TILE;
#pragma unroll
    for (int q = 0; q < RS_IT; ++q) {
        const uint32_t i = (uint32_t)tid + (uint32_t)q * RS_NT;
        if (i >= tn) continue;
        const K kk = sk[i];
        const uint32_t dd = digit_of(kk, p);
        const uint64_t o = (uint64_t)gbase[dd] + (i - dstart[dd]);
        kout[o] = kk;
        vout[o] = sv[i];
    }
}

template <typename K>
int radix_sort_t(K* k0, uint32_t* v0, K* k1, uint32_t* v1, uint64_t n, uint32_t byte_mask, int nbytes,
                 Arena& ar, hipStream_t s) {
    if (n <= 1 || byte_mask == 0) return 0;
    if (n > 0xFFFFFFFFull) return -3;
    uint32_t nb = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    size_t m = ar.mark();
    uint32_t* hist = (uint32_t*)ar.get(((uint64_t)256 * nb + 1) * sizeof(uint32_t));
    if (!hist) return -2;
    int cur = 0;
    for (int p = 0; p < nbytes; ++p) {
        if (!((byte_mask >> p) & 1u)) continue;
        K* ki = cur ? k1 : k0;
        uint32_t* vi = cur ? v1 : v0;
        K* ko = cur ? k0 : k1;
        uint32_t* vo = cur ? v0 : v1;
        k_rs_hist<K><<<nb, RS_NT, 0, s>>>(ki, n, p, hist, nb);
        if (nb <= RS_FUSED_MAXNB) { /* two launches per digit: the scatter scans the histogram itself */
            k_rs_scatter<K, true><<<nb, RS_NT, 0, s>>>(ki, vi, ko, vo, n, p, hist, nb);
        } else {
            int rc = scan_excl_t<uint32_t>(hist, hist, (uint64_t)256 * nb, ar, s);
            if (rc) return rc;
            k_rs_scatter<K, false><<<nb, RS_NT, 0, s>>>(ki, vi, ko, vo, n, p, hist, nb);
        }
        cur ^= 1;
    }
    ar.release(m);
    return hipGetLastError() == hipSuccess ? cur : -1;
}

/* ------------------------------------------------- small sorts (n <= SORT_TILE_MAXN) ----
 * Two launches, no digit passes: (1) each 1024-thread block bitonic-sorts a tile of 2048
 * (key, input index) pairs in LDS; (2) every element's output position is its index in
 * its own tile plus, for every other tile, the number of that tile's elements ordered
 * before it (a binary search) — its global rank, since (key, input index) pairs are
 * distinct.  Ties on the key keep input order, so the result equals the stable LSD radix
 * sort's.  Replaces 4-5 launches per 8-bit digit for the vocabulary, document-order and
 * partial-record sorts, which are all a few 10^5 elements. */
constexpr int TS_NT = 1024;
constexpr uint32_t TS_T = 2048;

__device__ __forceinline__ bool key_lt(uint64_t a, uint64_t b) { return a < b; }
__device__ __forceinline__ bool key_eq(uint64_t a, uint64_t b) { return a == b; }
__device__ __forceinline__ bool key_lt(uint4 a, uint4 b) {
    if (a.w != b.w) return a.w < b.w;
    if (a.z != b.z) return a.z < b.z;
    if (a.y != b.y) return a.y < b.y;
    return a.x < b.x;
}
__device__ __forceinline__ bool key_eq(uint4 a, uint4 b) { return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w; }
__device__ __forceinline__ void key_max(uint64_t& k) { k = ~0ull; }
__device__ __forceinline__ void key_max(uint4& k) { k = make_uint4(~0u, ~0u, ~0u, ~0u); }

template <typename K>
__global__ __launch_bounds__(TS_NT) void k_tile_sort(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                    uint64_t n, K* __restrict__ tk, uint32_t* __restrict__ tv,
                                                    uint32_t* __restrict__ ti) {
    __shared__ K sk[TS_T];
    __shared__ uint32_t sv[TS_T], si[TS_T];
    const uint32_t tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * TS_T;
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
        const uint32_t e = tid + h * TS_NT;
        const uint64_t g = t0 + e;
        if (g < n) { sk[e] = kin[g]; sv[e] = vin[g]; si[e] = (uint32_t)g; }
        else { K m; key_max(m); sk[e] = m; sv[e] = 0u; si[e] = 0xFFFFFFFFu; }
    }
    __syncthreads();
    for (uint32_t k = 2; k <= TS_T; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            const uint32_t i = 2u * tid - (tid & (j - 1u)), l = i + j;
            const bool asc = (i & k) == 0u;
            const K a = sk[i], b = sk[l];
            const uint32_t ia = si[i], ib = si[l];
            const bool b_first = key_lt(b, a) || (key_eq(a, b) && ib < ia);
            if (b_first == asc) {
                sk[i] = b; sk[l] = a;
                si[i] = ib; si[l] = ia;
                const uint32_t x = sv[i]; sv[i] = sv[l]; sv[l] = x;
            }
            __syncthreads();
        }
    }
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
        const uint32_t e = tid + h * TS_NT;
        const uint64_t g = t0 + e;
        if (g < n) { tk[g] = sk[e]; tv[g] = sv[e]; ti[g] = si[e]; }
    }
}

/* An element's rank, split over blockIdx.y groups of TS_LB tiles so the grid has
 * enough waves to hide the searches' latency: each thread advances its group's TS_LB
 * searches in lockstep (TS_LB independent loads in flight per step) and adds the count
 * to pos[element] (group 0 also adds the element's index in its own tile). */
constexpr uint32_t TS_LB = 8;
template <typename K>
__global__ __launch_bounds__(256) void k_tile_rank(const K* __restrict__ tk, const uint32_t* __restrict__ ti,
                                                  uint64_t n, uint32_t* __restrict__ pos) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const uint32_t t = (uint32_t)(g / TS_T), nt = (uint32_t)((n + TS_T - 1) / TS_T);
    const uint32_t b0 = blockIdx.y * TS_LB;
    const K key = tk[g];
    const uint32_t idx = ti[g];
    uint32_t lo[TS_LB], len[TS_LB];
#pragma unroll
    for (uint32_t q = 0; q < TS_LB; ++q) {
        const uint32_t b = b0 + q;
        const uint64_t st = (uint64_t)b * TS_T;
        lo[q] = 0;
        len[q] = (b < nt && b != t) ? (uint32_t)((n - st) < TS_T ? (n - st) : TS_T) : 0u;
    }
    for (uint32_t it = 0; it < 12; ++it) {  /* ceil(log2(TS_T + 1)) steps */
#pragma unroll
        for (uint32_t q = 0; q < TS_LB; ++q) {
            if (len[q] == 0u) continue;
            const uint32_t half = len[q] >> 1, mid = lo[q] + half;
            const uint64_t e = (uint64_t)(b0 + q) * TS_T + mid;
            const K m = tk[e];
            const bool before = key_lt(m, key) || (key_eq(m, key) && ti[e] < idx);
            if (before) { lo[q] = mid + 1u; len[q] -= half + 1u; }
            else len[q] = half;
        }
    }
    uint32_t c = blockIdx.y == 0 ? (uint32_t)(g - (uint64_t)t * TS_T) : 0u;
#pragma unroll
    for (uint32_t q = 0; q < TS_LB; ++q) c += lo[q];
    if (c) atomicAdd(&pos[g], c);
}
template <typename K>
__global__ void k_tile_place(const K* __restrict__ tk, const uint32_t* __restrict__ tv,
                             const uint32_t* __restrict__ pos, uint64_t n, K* __restrict__ kout,
                             uint32_t* __restrict__ vout) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const uint32_t p = pos[g];
    kout[p] = tk[g];
    vout[p] = tv[g];
}

template <typename K>
int tile_sort_t(const K* k0, const uint32_t* v0, K* k1, uint32_t* v1, uint64_t n, Arena& ar, hipStream_t s) {
    if (n == 0) return 1;   /* nothing to sort: the (empty) result is in (k1, v1) */
    const uint32_t nt = (uint32_t)((n + TS_T - 1) / TS_T);
    size_t m = ar.mark();
    K* tk = (K*)ar.get(n * sizeof(K));
    uint32_t* tv = (uint32_t*)ar.get(n * 4);
    uint32_t* ti = (uint32_t*)ar.get(n * 4);
    if (!tk || !tv || !ti) return -2;
    uint32_t* pos = (uint32_t*)ar.get(n * 4);
    if (!pos) return -2;
    if (hipMemsetAsync(pos, 0, n * 4, s) != hipSuccess) return -1;
    k_tile_sort<K><<<nt, TS_NT, 0, s>>>(k0, v0, n, tk, tv, ti);
    k_tile_rank<K><<<dim3((unsigned)((n + 255) / 256), (nt + TS_LB - 1) / TS_LB), 256, 0, s>>>(tk, ti, n, pos);
    k_tile_place<K><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(tk, tv, pos, n, k1, v1);
    ar.release(m);
    return hipGetLastError() == hipSuccess ? 1 : -1;
}

/* AND / OR of all keys (which bytes vary): wave reduce, then one LDS combine per block and
 * one global atomic per block and word (thousands of same-address atomics serialise). */
__global__ __launch_bounds__(256) void k_orand_u64(const uint64_t* __restrict__ k, uint64_t n, unsigned long long* acc) {
    __shared__ unsigned long long sa[4], so[4];
    uint64_t a = ~0ull, o = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        a &= k[i];
        o |= k[i];
    }
    for (int off = 32; off > 0; off >>= 1) {
        a &= __shfl_xor(a, off, 64);
        o |= __shfl_xor(o, off, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sa[w] = a; so[w] = o; }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAnd(&acc[0], sa[0] & sa[1] & sa[2] & sa[3]);
        atomicOr(&acc[1], so[0] | so[1] | so[2] | so[3]);
    }
}

__global__ __launch_bounds__(256) void k_orand_u128(const uint4* __restrict__ k, uint64_t n, unsigned long long* acc) {
    __shared__ unsigned long long s4[4][4];
    uint64_t a0 = ~0ull, a1 = ~0ull, o0 = 0, o1 = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = k[i];
        uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
        a0 &= lo; a1 &= hi; o0 |= lo; o1 |= hi;
    }
    for (int off = 32; off > 0; off >>= 1) {
        a0 &= __shfl_xor(a0, off, 64); a1 &= __shfl_xor(a1, off, 64);
        o0 |= __shfl_xor(o0, off, 64); o1 |= __shfl_xor(o1, off, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s4[w][0] = a0; s4[w][1] = a1; s4[w][2] = o0; s4[w][3] = o1; }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAnd(&acc[0], s4[0][0] & s4[1][0] & s4[2][0] & s4[3][0]);
        atomicAnd(&acc[1], s4[0][1] & s4[1][1] & s4[2][1] & s4[3][1]);
        atomicOr(&acc[2], s4[0][2] | s4[1][2] | s4[2][2] | s4[3][2]);
        atomicOr(&acc[3], s4[0][3] | s4[1][3] | s4[2][3] | s4[3][3]);
    }
}

}  // namespace

int scan_excl_u32(const uint32_t* in, uint32_t* out, uint64_t n, Arena& ar, hipStream_t s) {
    return scan_excl_t<uint32_t>(in, out, n, ar, s);
}
int scan_excl_u64(const uint64_t* in, uint64_t* out, uint64_t n, Arena& ar, hipStream_t s) {
    return scan_excl_t<uint64_t>(in, out, n, ar, s);
}
int tile_sort_u64(const uint64_t* k0, const uint32_t* v0, uint64_t* k1, uint32_t* v1, uint64_t n, Arena& ar,
                  hipStream_t s) {
    if (n > SORT_TILE_MAXN) return -3;
    if (n <= 1) {
        if (n == 1 && (hipMemcpyAsync(k1, k0, 8, hipMemcpyDeviceToDevice, s) != hipSuccess ||
                       hipMemcpyAsync(v1, v0, 4, hipMemcpyDeviceToDevice, s) != hipSuccess)) return -1;
        return 1;
    }
    return tile_sort_t<uint64_t>(k0, v0, k1, v1, n, ar, s);
}
int tile_sort_u128(const uint4* k0, const uint32_t* v0, uint4* k1, uint32_t* v1, uint64_t n, Arena& ar,
                   hipStream_t s) {
    if (n > SORT_TILE_MAXN) return -3;
    if (n <= 1) {
        if (n == 1 && (hipMemcpyAsync(k1, k0, 16, hipMemcpyDeviceToDevice, s) != hipSuccess ||
                       hipMemcpyAsync(v1, v0, 4, hipMemcpyDeviceToDevice, s) != hipSuccess)) return -1;
        return 1;
    }
    return tile_sort_t<uint4>(k0, v0, k1, v1, n, ar, s);
}
int radix_sort_u64(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, uint64_t n, uint32_t byte_mask,
                   Arena& ar, hipStream_t s) {
    return radix_sort_t<uint64_t>(k0, v0, k1, v1, n, byte_mask, 8, ar, s);
}
int radix_sort_u128(uint4* k0, uint32_t* v0, uint4* k1, uint32_t* v1, uint64_t n, uint32_t byte_mask,
                    Arena& ar, hipStream_t s) {
    return radix_sort_t<uint4>(k0, v0, k1, v1, n, byte_mask, 16, ar, s);
}

static int varying_common(int words, const void* k, uint64_t n, uint32_t* mask, Arena& ar, hipStream_t s) {
    size_t m = ar.mark();
    unsigned long long* acc = (unsigned long long*)ar.get(4 * sizeof(unsigned long long));
    if (!acc) return -2;
    unsigned long long init[4] = {~0ull, ~0ull, 0ull, 0ull};
    if (words == 1) { init[1] = 0ull; }
    if (hipMemcpyAsync(acc, init, sizeof init, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
    unsigned grid = (unsigned)((n + 255) / 256);
    if (grid > 512) grid = 512;
    if (grid == 0) grid = 1;
    if (words == 1) k_orand_u64<<<grid, 256, 0, s>>>((const uint64_t*)k, n, acc);
    else k_orand_u128<<<grid, 256, 0, s>>>((const uint4*)k, n, acc);
    unsigned long long h[4];
    if (hipMemcpyAsync(h, acc, sizeof h, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    ar.release(m);
    uint32_t msk = 0;
    if (words == 1) {
        uint64_t x = h[0] ^ h[1];
        for (int p = 0; p < 8; ++p) if ((x >> (8 * p)) & 0xFF) msk |= 1u << p;
    } else {
        uint64_t x0 = h[0] ^ h[2], x1 = h[1] ^ h[3];
        for (int p = 0; p < 8; ++p) {
            if ((x0 >> (8 * p)) & 0xFF) msk |= 1u << p;
            if ((x1 >> (8 * p)) & 0xFF) msk |= 1u << (p + 8);
        }
    }
    *mask = msk;
    return 0;
}

int key_varying_bytes_u64(const uint64_t* k, uint64_t n, uint32_t* mask, Arena& ar, hipStream_t s) {
    if (n == 0) { *mask = 0; return 0; }
    return varying_common(1, k, n, mask, ar, s);
}
int key_varying_bytes_u128(const uint4* k, uint64_t n, uint32_t* mask, Arena& ar, hipStream_t s) {
    if (n == 0) { *mask = 0; return 0; }
    return varying_common(2, k, n, mask, ar, s);
}

/* ------------------------------------------------------------ HBM probes --
 * Measured streaming peaks for the roofline ("also report the fraction of a
 * measured copy-kernel peak"): a read-only stream (16-byte non-temporal loads, 4 in
 * flight per lane, XOR-folded so nothing is elided) and a copy.  Diagnostics only. */
typedef unsigned int probe_u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream_read(const probe_u32x4* __restrict__ p, uint64_t n16,
                                                     uint32_t* __restrict__ sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    probe_u32x4 acc = {0u, 0u, 0u, 0u};
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const probe_u32x4 a = __builtin_nontemporal_load(p + i), b = __builtin_nontemporal_load(p + i + stride);
        const probe_u32x4 c = __builtin_nontemporal_load(p + i + 2 * stride), d = __builtin_nontemporal_load(p + i + 3 * stride);
        acc ^= a ^ b ^ c ^ d;
    }
    for (; i < n16; i += stride) acc ^= __builtin_nontemporal_load(p + i);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[0] = 1u;   /* never for the probe's zero fill */
}
__global__ __launch_bounds__(256) void k_stream_copy(const probe_u32x4* __restrict__ src, probe_u32x4* __restrict__ dst,
                                                     uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + stride < n16; i += 2 * stride) {
        const probe_u32x4 a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride);
        __builtin_nontemporal_store(a, dst + i);
        __builtin_nontemporal_store(b, dst + i + stride);
    }
    for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}
int launch_stream_read(const void* p, uint64_t nbytes, uint32_t* sink, unsigned grid, hipStream_t s) {
    k_stream_read<<<grid, 256, 0, s>>>((const probe_u32x4*)p, nbytes / 16, sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_stream_copy(const void* src, void* dst, uint64_t nbytes, unsigned grid, hipStream_t s) {
    k_stream_copy<<<grid, 256, 0, s>>>((const probe_u32x4*)src, (probe_u32x4*)dst, nbytes / 16);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
