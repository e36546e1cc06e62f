/*
 * dev_common.h — device helpers shared by the gfx950 kernels.
 *
 * Term identity (TFIDF.c:152,161,172,184 compare and copy words with strcmp/strcpy,
 * so a term is the token's bytes up to its first NUL).  Terms are 128-bit keys:
 *
 *   short term (<= 15 bytes): little-endian bytes w[0..n), byte n = 0x09 (TAB), rest 0.
 *       Exact and injective.  Byte-swapped, the same 16 bytes are the big-endian sort
 *       key "w \t 0...", whose unsigned order is the strcmp order of the reference's
 *       "docN@w\t..." lines for a fixed document.
 *   long term (>= 16 bytes): bytes 0..14 = 120-bit hash of the term, byte 15 = 0xFF.
 *       Its ordering key is the word's first 16 bytes; equal prefixes are resolved by a
 *       full byte compare (vocab_long_fixup).
 * Byte 15 of a short key is 0x00 or 0x09 and of a long key 0xFF, so the sentinels
 * below (byte 15 = 0xEE / 0xDD / 0xFE) never collide with a real key.
 */
#ifndef TFIDF_DEV_COMMON_H
#define TFIDF_DEV_COMMON_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define KEY_EMPTY_HI   0xEEEEEEEEEEEEEEEEull   /* empty hash-table slot */
#define KEY_PENDING_HI 0xDDDDDDDDDDDDDDDDull   /* claimed, key being published */
#define KEY_GSLOT_TAG  0xFE00000000000000ull   /* LDS key already resolved to a global slot */
#define KEY_LONG_TAG   0xFF00000000000000ull
#define DOC_NONE       0xFFFFFFFFu

/* Explicitly global (address space 1) loads and stores.  A pointer that reaches a load
 * through a struct or a lambda capture can lose its address space, and the compiler then
 * emits a flat_ instruction: flat loads count in lgkmcnt as well as vmcnt, so every later
 * LDS wait (lgkmcnt(0)) also waits for the gather in flight. */
#define GLOBAL_AS __attribute__((address_space(1)))
template <class T> __device__ __forceinline__ T gload(const T* p) { return *(const GLOBAL_AS T*)p; }
template <class T> __device__ __forceinline__ void gstore(T* p, T v) { *(GLOBAL_AS T*)p = v; }
/* uint4 is a class type whose copy goes through a generic pointer: load a native vector */
typedef unsigned int g_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gload(const uint4* p) {
    const g_u32x4 r = *(const GLOBAL_AS g_u32x4*)p;
    return make_uint4(r.x, r.y, r.z, r.w);
}

/* C-locale isspace(): the byte set fscanf("%s") stops at (TFIDF.c:142,147) */
__device__ __forceinline__ bool is_ws(uint32_t c) { return c == 0x20u || (c - 0x09u) <= 4u; }

/* 4-bit mask of the C-locale whitespace bytes {0x20, 0x09..0x0D} of a 32-bit word,
 * SWAR: every per-byte sum below stays inside its byte, so the tests are exact. */
__device__ __forceinline__ uint32_t ws_mask4(uint32_t x) {
    const uint32_t lo7 = x & 0x7F7F7F7Fu;
    const uint32_t t = x ^ 0x20202020u;
    const uint32_t ne20 = ((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t;   /* bit 7: byte != 0x20 */
    const uint32_t ge9 = lo7 + 0x77777777u;                         /* bit 7: low7 >= 0x09 */
    const uint32_t ge14 = lo7 + 0x72727272u;                        /* bit 7: low7 >= 0x0E */
    uint32_t m = (~ne20 | (ge9 & ~ge14)) & ~x & 0x80808080u;        /* bit 7 of each ws byte */
    m >>= 7;                                                        /* bits 0, 8, 16, 24 */
    m |= m >> 7;                                                    /* bits 0-1, 16-17 */
    m |= m >> 14;                                                   /* bits 0-3 */
    return m & 0xFu;
}
__device__ __forceinline__ uint32_t ws_mask16_swar(uint4 v) {
    return ws_mask4(v.x) | (ws_mask4(v.y) << 4) | (ws_mask4(v.z) << 8) | (ws_mask4(v.w) << 12);
}

/* 16-bit mask of whitespace bytes in a 16-byte group (bit i = byte i) */
__device__ __forceinline__ uint32_t ws_mask16(uint4 v) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            uint32_t c = (w[k] >> (8 * b)) & 0xFFu;
            m |= (is_ws(c) ? 1u : 0u) << (4 * k + b);
        }
    }
    return m;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Vocabulary hash of a 128-bit term key: two 32-bit multiplies and an xor-shift that brings
 * the products' high bits into the low bits the table mask keeps (on gfx950 v_mul_lo_u32
 * issues like a shift or a v_perm, ~4.8 cycles per wave-instruction per SIMD:
 * scripts/micro/valu_rates.hip).  On c2's 5e4 terms it probes like the four-multiply murmur
 * finaliser it replaced: at a 1M-slot table 2.7 % of the keys leave their home slot (2.5 %
 * before), 0.15 % go past the next one (24-bit-multiply forms that issue as cheaply placed
 * 5-8 % past the pair: not used).  Tables are < 2^32 slots. */
__device__ __forceinline__ uint64_t key_hash(uint64_t lo, uint64_t hi) {
    const uint32_t a = (uint32_t)lo, b = (uint32_t)(lo >> 32), c = (uint32_t)hi, d = (uint32_t)(hi >> 32);
    uint32_t h = ((a ^ __builtin_rotateleft32(c, 16)) * 0x9E3779B1u) ^ ((b ^ __builtin_rotateleft32(d, 8)) * 0x85EBCA77u);
    h ^= h >> 16;
    return h;
}

/* first zero byte index in a u64 (8 if none) */
__device__ __forceinline__ uint32_t first_zero_byte(uint64_t x) {
    uint64_t t = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
    return t ? (uint32_t)(__builtin_ctzll(t) >> 3) : 8u;
}

/* Builds the short key from 16 raw bytes (lo = bytes 0..7, hi = 8..15) of a token of
 * length len (bytes beyond len are ignored).  Returns the term length after NUL
 * truncation; the key is valid only when that length is <= 15. */
__device__ __forceinline__ uint32_t make_short_key(uint64_t lo, uint64_t hi, uint32_t len,
                                                   uint64_t* klo, uint64_t* khi) {
    uint32_t n = len < 16u ? len : 16u;
    /* NUL truncation (strcmp semantics) */
    uint32_t z0 = first_zero_byte(lo);
    uint32_t z = z0 < 8u ? z0 : 8u + first_zero_byte(hi);
    if (z < n) n = z;
    if (n >= 16u) return 16u;
    /* keep bytes < n, put TAB at n, zero the rest */
    uint64_t mlo = n >= 8u ? ~0ull : ((1ull << (8u * n)) - 1ull);
    uint64_t mhi = n <= 8u ? 0ull : ((1ull << (8u * (n - 8u))) - 1ull);
    lo &= mlo;
    hi &= mhi;
    if (n < 8u) lo |= 0x09ull << (8u * n);
    else hi |= 0x09ull << (8u * (n - 8u));
    *klo = lo;
    *khi = hi;
    return n;
}

/* Long-term key: 120-bit hash over the term bytes, byte 15 = 0xFF. */
__device__ __forceinline__ void make_long_key(const uint8_t* p, uint64_t n, uint64_t* klo, uint64_t* khi) {
    uint64_t h1 = 0x243F6A8885A308D3ull ^ n, h2 = 0x13198A2E03707344ull + n * 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t c = p[i];
        h1 = (h1 ^ c) * 0x100000001B3ull;
        h2 = (h2 + c + 1) * 0xC2B2AE3D27D4EB4Full;
        h2 ^= h2 >> 29;
    }
    *klo = mix64(h1 ^ (h2 << 1));
    *khi = (mix64(h2 + 0x7F4A7C15ull * h1) & 0x00FFFFFFFFFFFFFFull) | KEY_LONG_TAG;
#ifdef TFIDF_LONG_KEY_BITS   /* test build only: a truncated tag that forces collisions (dev_vocab.h detects them) */
    *klo &= (1ull << TFIDF_LONG_KEY_BITS) - 1ull;
    *khi = KEY_LONG_TAG;
#endif
}

__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

/* ---- wave64 cross-lane primitives on DPP (GFX9-family data-parallel primitives:
 * no LDS traffic and no lane-index registers, unlike ds_bpermute-based shuffles) ---- */
#define DPP_ROW_SHR(n)   (0x110 + (n))
#define DPP_WAVE_SHL1    0x130   /* lane i reads lane i+1 */
#define DPP_WAVE_SHR1    0x138   /* lane i reads lane i-1 */
#define DPP_ROW_BCAST15  0x142
#define DPP_ROW_BCAST31  0x143

/* value of lane+1 (lane 63 gets its own value) */
__device__ __forceinline__ uint32_t lane_next(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, DPP_WAVE_SHL1, 0xF, 0xF, false);
}
/* value of lane-1 (lane 0 gets its own value) */
__device__ __forceinline__ uint32_t lane_prev(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, DPP_WAVE_SHR1, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(1), 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(2), 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(4), 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_SHR(8), 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_BCAST15, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_ROW_BCAST31, 0xC, 0xF, false);
    return v;
}

/* max over the wave, uniform (scalar) result */
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t t = (uint32_t)__shfl_xor((int)v, o, 64);
        v = t > v ? t : v;
    }
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

/* sum over the wave, uniform (scalar) result */
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v), 63);
}

/* Workgroup barrier that orders LDS only.  __syncthreads() is a release/acquire fence over
 * all address spaces, so it also waits for every outstanding global store of the wave
 * (vmcnt(0)); kernels whose barriers only publish LDS data use this one. */
/* A generic pointer known to address device memory, as a global-address-space pointer:
 * stores through it compile to global_store (counted in vmcnt only) instead of flat_store,
 * which also counts in lgkmcnt, so that every later LDS wait would wait for the store too
 * (pointers loaded from memory, e.g. a K1Out block, are generic to the compiler). */
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gmem(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}

/* device-scope atomic add on device memory through a global-address-space pointer
 * (global_atomic: a returning flat atomic would hold lgkmcnt until it returns) */
__device__ __forceinline__ unsigned long long gatomic_add(unsigned long long* p, unsigned long long v) {
    return __hip_atomic_fetch_add(gmem(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

/* exclusive scan over the block (blockDim = NT, multiple of 64); wsum: NT/64 words LDS.
 * Returns exclusive prefix; *total = block sum.  Contains two barriers. */
template <int NT, bool LDS_ONLY = false>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(v);
    if (lane == 63) wsum[w] = inc;
    if (LDS_ONLY) lds_barrier(); else __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
        uint32_t s = wsum[k];
        base += (k < w) ? s : 0u;
        tot += s;
    }
    *total = tot;
    if (LDS_ONLY) lds_barrier(); else __syncthreads();
    return base + inc - v;
}

#endif
