/* prims.h — host launchers for the device-wide primitives in prims.hip. */
#ifndef TFIDF_PRIMS_H
#define TFIDF_PRIMS_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

/* Bump allocator over one device buffer; reset per run. */
struct Arena {
    uint8_t* base = nullptr;
    size_t cap = 0;
    size_t used = 0;
    size_t peak = 0;
    void* get(size_t bytes) {
        size_t off = (used + 255) & ~(size_t)255;
        if (off + bytes > cap) { peak = off + bytes > peak ? off + bytes : peak; return nullptr; }
        used = off + bytes;
        if (used > peak) peak = used;
        return base + off;
    }
    size_t mark() const { return used; }
    void release(size_t m) { used = m; }
};

/* exclusive scan of n elements; out has n+1 entries, out[n] = total.  in may alias out. */
int scan_excl_u32(const uint32_t* in, uint32_t* out, uint64_t n, Arena& ar, hipStream_t s);
int scan_excl_u64(const uint64_t* in, uint64_t* out, uint64_t n, Arena& ar, hipStream_t s);

/* LSD radix sort of (key, u32 value) pairs, keys of KB bytes (8 or 16), ascending
 * unsigned.  Only digit bytes set in byte_mask are sorted (the caller proves the others
 * constant).  Ping-pongs between (k0,v0) and (k1,v1): returns 0 when the result is in
 * (k0,v0), 1 when in (k1,v1), <0 on error. */
int radix_sort_u64(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, uint64_t n,
                   uint32_t byte_mask, Arena& ar, hipStream_t s);
int radix_sort_u128(uint4* k0, uint32_t* v0, uint4* k1, uint32_t* v1, uint64_t n,
                    uint32_t byte_mask, Arena& ar, hipStream_t s);

/* Stable sort of (key, u32 value) pairs for n <= SORT_TILE_MAXN in two launches (tile
 * bitonic sort + rank by binary search); same result as the radix sort over all bytes.
 * The result is always in (k1, v1): returns 1, or <0 on error. */
constexpr uint64_t SORT_TILE_MAXN = 64ull * 2048ull;
int tile_sort_u64(const uint64_t* k0, const uint32_t* v0, uint64_t* k1, uint32_t* v1, uint64_t n, Arena& ar,
                  hipStream_t s);
int tile_sort_u128(const uint4* k0, const uint32_t* v0, uint4* k1, uint32_t* v1, uint64_t n, Arena& ar,
                   hipStream_t s);

/* Bitwise AND and OR over n keys of KB bytes -> varying-byte mask (synchronises). */
int key_varying_bytes_u64(const uint64_t* k, uint64_t n, uint32_t* mask, Arena& ar, hipStream_t s);
int key_varying_bytes_u128(const uint4* k, uint64_t n, uint32_t* mask, Arena& ar, hipStream_t s);

/* HBM probes (diagnostics for the roofline's measured peak) */
int launch_stream_read(const void* p, uint64_t nbytes, uint32_t* sink, unsigned grid, hipStream_t s);
int launch_stream_copy(const void* src, void* dst, uint64_t nbytes, unsigned grid, hipStream_t s);

#endif
