/*
 * emit.hip — output emission on the GPU: the reference's
 * "docN@word\t%.16f" lines (TFIDF.c:245) in output order (TFIDF.c:273), written as one
 * contiguous text in HBM for output.txt (TFIDF.c:274-282).
 *
 *   %.16f        exact binary -> decimal: q = x * 10^16 rounded half-to-even from the
 *                double's integer significand with 128-bit arithmetic (glibc printf's
 *                result for every finite x >= 0 below 2^63 / 10^16; scores are
 *                tf * log(N/df) <= log(2^32) < 23)
 *   digits       u32 arithmetic only: 8-digit halves split into 4 and 2 digits by
 *                multiply-shift, packed as ASCII words
 *   lines        one wave per document: its lines' lengths, a wave scan for their
 *                offsets, then each lane writes its line into the wave's LDS stage with
 *                five unaligned stores and the wave copies the round out with 16-byte
 *                stores
 */
#include "kernels.h"
#include "dev_common.h"

namespace {

constexpr int NT = 256;
/* at least one workgroup: an empty launch is an error, every kernel bounds-checks its index */
inline unsigned grid_for(uint64_t n, int nt = NT) { return n ? (unsigned)((n + nt - 1) / nt) : 1u; }
int ok() { return hipGetLastError() == hipSuccess ? 0 : -1; }

constexpr uint64_t P16 = 10000000000000000ull;

/* q = round-half-even(x * 10^16); false when x is negative, not finite or >= 2^63/10^16 */
__device__ __forceinline__ bool fixed16(double x, uint64_t& q) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    if (b >> 63) return false;
    const uint32_t ex = (uint32_t)(b >> 52) & 0x7FFu;
    uint64_t m = b & ((1ull << 52) - 1ull);
    if (ex == 0x7FFu) return false;
    if (ex == 0u && m == 0ull) { q = 0; return true; }
    int e;
    if (ex == 0u) e = -1074;
    else { m |= 1ull << 52; e = (int)ex - 1075; }
    /* x = m * 2^e;  x * 10^16 = m * 10^16 * 2^e with m * 10^16 < 2^107 */
    unsigned __int128 p = (unsigned __int128)m * P16;
    if (e >= 0) {
        if (e > 10) return false;
        p <<= e;
        if ((p >> 63) != 0) return false;
        q = (uint64_t)p;
        return true;
    }
    const int s = -e;
    if (s >= 108) { q = 0; return true; } /* p < 2^107 <= 2^(s-1): below half */
    const unsigned __int128 hi = p >> s;
    if ((hi >> 63) != 0) return false;
    uint64_t r = (uint64_t)hi;
    const unsigned __int128 one = 1;
    const unsigned __int128 rem = p & ((one << s) - one), half = one << (s - 1);
    if (rem > half || (rem == half && (r & 1ull))) ++r;
    q = r;
    return true;
}

/* decimal digits of a u32 */
__device__ __forceinline__ uint32_t ndig32(uint32_t v) {
    uint32_t n = 1;
    for (uint32_t t = 10u; n < 10u && v >= t; t *= 10u) ++n;
    return n;
}

/* x < 10^4 as 4 ASCII digits, the most significant in the lowest byte */
__device__ __forceinline__ uint32_t ascii4(uint32_t x) {
    const uint32_t h = (x * 5243u) >> 19, l = x - h * 100u;   /* x / 100, exact below 43699 */
    const uint32_t h1 = (h * 103u) >> 10, l1 = (l * 103u) >> 10; /* y / 10, exact below 179 */
    return 0x30303030u | h1 | ((h - h1 * 10u) << 8) | (l1 << 16) | ((l - l1 * 10u) << 24);
}
/* x < 10^8 as 8 ASCII digits */
__device__ __forceinline__ uint64_t ascii8(uint32_t x) {
    const uint32_t a = x / 10000u;
    return (uint64_t)ascii4(a) | ((uint64_t)ascii4(x - a * 10000u) << 32);
}

/* unaligned stores (gfx950 DS and global accesses take any byte address) */
__device__ __forceinline__ void st16(uint8_t* p, uint64_t lo, uint64_t hi) {
    __builtin_memcpy(p, &lo, 8);
    __builtin_memcpy(p + 8, &hi, 8);
}
__device__ __forceinline__ void st4(uint8_t* p, uint32_t v) { __builtin_memcpy(p, &v, 4); }

/* A score's integer part: q / 10^16 = floor(x), since rounding x * 10^16 to an integer
 * never reaches the next multiple of 10^16 (the doubles below an integer n >= 1 are at
 * least 2^-53 > 0.5e-16 from it). */
struct Score {
    uint64_t q;      /* round(x * 10^16) */
    uint32_t ip;     /* integer part, < 923 */
    uint32_t ni;     /* its digits */
};
__device__ __forceinline__ uint32_t ndig3(uint32_t ip) { return ip < 10u ? 1u : ip < 100u ? 2u : 3u; }

/* "%.16f" of q: integer digits, '.', 16 fraction digits, written with three unaligned
 * stores (the first may write up to 3 bytes past the '.', which the next overwrites) */
__device__ __forceinline__ void put_score(uint8_t* p, const Score& sc) {
    const uint64_t fr = sc.q - (uint64_t)sc.ip * P16;
    const uint32_t f0 = (uint32_t)(fr / 100000000ull), f1 = (uint32_t)(fr - (uint64_t)f0 * 100000000ull);
    st4(p, (ascii4(sc.ip) >> (8u * (4u - sc.ni))) | (0x2Eu << (8u * sc.ni)));
    st16(p + sc.ni + 1u, ascii8(f0), ascii8(f1));
}

/* "doc" id '@' as 16 bytes (3 + at most 10 + 1 used, the rest zero) */
__device__ __forceinline__ void doc_prefix(uint32_t id, uint32_t nid, uint64_t& lo, uint64_t& hi) {
    const uint32_t h = id / 100000000u;                                  /* <= 42 */
    /* the zero-padded 10 digits at bytes 0..9, then the leading zeros shifted out */
    unsigned __int128 d = (unsigned __int128)(ascii4(h) >> 16) |
                          ((unsigned __int128)ascii8(id - h * 100000000u) << 16);
    d >>= 8u * (10u - nid);
    d = (d << 24) | (unsigned __int128)0x636F64u | ((unsigned __int128)0x40u << (8u * (3u + nid)));
    lo = (uint64_t)d;
    hi = (uint64_t)(d >> 64);
}

/* per term rank: its byte length and where its bytes are (short terms: the 16-byte key,
 * bytes up to the TAB terminator; long terms: a corpus position from the vocabulary rep) */
__global__ void k_term_meta(const uint4* __restrict__ vkeys, const uint64_t* __restrict__ vrep,
                            const uint32_t* __restrict__ slot_of_rank, uint32_t V, uint4* __restrict__ tkey,
                            uint32_t* __restrict__ tlen) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= V) return;
    const uint32_t sl = slot_of_rank[r];
    const uint4 k = vkeys[sl];
    if ((k.w >> 24) == 0xFFu) { /* long term: 120-bit hash key, bytes in the corpus */
        const uint64_t rep = vrep[sl];
        tkey[r] = make_uint4((uint32_t)rep, (uint32_t)(rep >> 32), 0u, 0xFFFFFFFFu);
        tlen[r] = (uint32_t)(rep >> 40);
        return;
    }
    const uint32_t w[4] = {k.x, k.y, k.z, k.w};
    uint32_t n = 16;
    for (uint32_t i = 0; i < 16; ++i)
        if (((w[i >> 2] >> (8 * (i & 3))) & 0xFFu) == 0x09u) { n = i; break; }
    tkey[r] = k;
    tlen[r] = n;
}

struct EmitArgs {
    const uint32_t* order;     /* output position -> local document */
    const uint32_t* doc_ids;   /* local document -> global id (NULL: index + 1) */
    const uint64_t* out_off;   /* N + 1 pair offsets per output position */
    const uint32_t* term;      /* per pair: term rank */
    const double* score;       /* per pair */
    const uint4* tkey;
    const uint32_t* tlen;
    const uint8_t* corpus;     /* long terms' bytes */
    uint32_t doc0, ndocs;      /* the output positions [doc0, ndocs) this launch covers */
    uint64_t* doc_bytes;       /* pass 1: text bytes per output position */
    const uint64_t* doc_text;  /* pass 2: text offset per output position */
    uint8_t* text;
    uint32_t* status;
};

__device__ __forceinline__ uint32_t doc_id_of(const EmitArgs& a, uint32_t i) {
    const uint32_t d = a.order[i];
    return a.doc_ids ? a.doc_ids[d] : d + 1u;
}

/* the score of pair p; an out-of-range score flags ST_BOUNDS and prints as 0 */
__device__ __forceinline__ Score score_of(const EmitArgs& a, uint64_t p) {
    Score sc;
    const double x = a.score[p];
    if (fixed16(x, sc.q)) {
        sc.ip = (uint32_t)x;
    } else {
        atomicOr(a.status, ST_BOUNDS);
        sc.q = 0;
        sc.ip = 0;
    }
    sc.ni = ndig3(sc.ip);
    return sc;
}
/* its integer digits only (the length pass): floor(x) without the exact product, which
 * only the range check at the top of the range needs */
__device__ __forceinline__ uint32_t score_ni(const EmitArgs& a, double x) {
    if (!((uint64_t)__double_as_longlong(x) >> 63) && x < 512.0) return ndig3((uint32_t)x);
    uint64_t q;
    if (!fixed16(x, q)) { atomicOr(a.status, ST_BOUNDS); return 1u; }
    return ndig3((uint32_t)x);
}

/* "doc" id '@' word '\t' score '\n': nid + wl + ni + 23 bytes */
__device__ __forceinline__ uint32_t line_len(uint32_t nid, uint32_t wl, uint32_t ni) { return nid + wl + ni + 23u; }

__global__ __launch_bounds__(NT) void k_doc_text_bytes(EmitArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * (NT / 64);
    for (uint32_t i = blockIdx.x * (NT / 64) + (threadIdx.x >> 6); i < a.ndocs; i += stride) {
        const uint64_t p0 = a.out_off[i], p1 = a.out_off[i + 1];
        const uint32_t nid = ndig32(doc_id_of(a, i));
        uint64_t sum = 0;
        /* four lines per lane in flight: the term -> length gathers wait on the term loads */
        for (uint64_t p = p0 + lane; p < p1; p += 4 * 64) {
            uint32_t t[4];
            double x[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t q = p + 64u * k;
                t[k] = q < p1 ? a.term[q] : 0u;
                x[k] = q < p1 ? a.score[q] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (p + 64u * k < p1) sum += line_len(nid, a.tlen[t[k]], score_ni(a, x[k]));
        }
        /* wave sum of 64-bit values: two 32-bit halves (a document's text < 2^32 * 64) */
        const uint32_t lo = wave_sum((uint32_t)sum & 0xFFFFFFu), hi = wave_sum((uint32_t)(sum >> 24));
        if (lane == 0) a.doc_bytes[i] = (uint64_t)lo + ((uint64_t)hi << 24);
    }
}

/* writes one line ("doc" id '@' word '\t' score '\n') of a short term at o, with
 * unaligned stores that stay inside the line: the 16-byte prefix (its zero tail is
 * overwritten by the word), the 16-byte key (word, its TAB, then bytes the score
 * overwrites), the score, the newline */
__device__ __forceinline__ void put_line(uint8_t* o, uint64_t pre_lo, uint64_t pre_hi, uint32_t nid, const uint4& k,
                                         uint32_t wl, const Score& sc) {
    st16(o, pre_lo, pre_hi);
    o += 4u + nid;
    st16(o, ((uint64_t)k.y << 32) | k.x, ((uint64_t)k.w << 32) | k.z);
    o += wl + 1u;
    put_score(o, sc);
    o[sc.ni + 17u] = '\n';
}

/* text[at + j] = stage[j] for j in [lo, hi) of one 16-byte chunk (hi <= 16): one byte per
 * lane — the chunks a document shares with its neighbours */
__device__ __forceinline__ void put_part(uint8_t* gb, const uint8_t* sg, uint32_t lo, uint32_t hi, uint32_t lane) {
    if (lane >= lo && lane < hi) gb[lane] = sg[lane];
}

/* One wave per document.  A round of 64 lines is assembled in the wave's LDS stage behind
 * the bytes the previous round left (fewer than 16: the stage starts at a 16-byte boundary
 * of the text), its whole 16-byte chunks go out with 16-byte stores and the partial last
 * chunk moves to the front of the stage for the next round.  Byte stores only where the
 * document's text shares a chunk with its neighbours (its first and last chunk).  Rounds
 * holding a long term (bytes in the corpus, up to any length) or more than the stage
 * write their lines directly. */
constexpr uint32_t STG = 4096;
__global__ __launch_bounds__(NT) void k_doc_text_write(EmitArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[NT / 64][STG + 16];
    const uint32_t lane = threadIdx.x & 63;
    uint8_t* sg = stage[threadIdx.x >> 6];
    const uint32_t stride = gridDim.x * (NT / 64);
    for (uint32_t i = a.doc0 + blockIdx.x * (NT / 64) + (threadIdx.x >> 6); i < a.ndocs; i += stride) {
        const uint64_t p0 = a.out_off[i], p1 = a.out_off[i + 1];
        const uint32_t id = doc_id_of(a, i), nid = ndig32(id);
        uint64_t pre_lo, pre_hi;
        doc_prefix(id, nid, pre_lo, pre_hi);
        /* stage byte j <-> text[g0 + j]; stage [lo0, fill) holds text not yet written, the
         * bytes before lo0 belong to the previous document (or were written directly) */
        uint64_t g0 = a.doc_text[i] & ~15ull;
        uint32_t fill = (uint32_t)(a.doc_text[i] & 15u), lo0 = fill;
        for (uint64_t r0 = p0; r0 < p1; r0 += 64) {
            const uint64_t p = r0 + lane;
            const bool v = p < p1;
            Score sc{0ull, 0u, 1u};
            uint32_t len = 0, wl = 0;
            uint4 k = make_uint4(0u, 0u, 0u, 0u);
            if (v) {
                const uint32_t t = a.term[p];
                k = a.tkey[t];
                wl = a.tlen[t];
                sc = score_of(a, p);
                len = line_len(nid, wl, sc.ni);
            }
            const uint32_t incl = wave_incl_scan(len);
            const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            const bool has_long = __ballot(v && k.w == 0xFFFFFFFFu) != 0ull;
            if (!has_long && tot <= STG - fill) {
                if (v) put_line(sg + fill + (incl - len), pre_lo, pre_hi, nid, k, wl, sc);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                uint8_t* gb = a.text + g0;
                const uint32_t end = fill + tot, nfull = end >> 4;
                for (uint32_t c = lane; c < nfull; c += 64)
                    if (c != 0u || lo0 == 0u)
                        *reinterpret_cast<uint4*>(gb + 16u * c) = *reinterpret_cast<const uint4*>(sg + 16u * c);
                if (nfull) {
                    if (lo0) put_part(gb, sg, lo0, 16u, lane);
                    lo0 = 0;
                    /* the partial last chunk to the front (this wave's LDS accesses are in order) */
                    if (lane == 0)
                        *reinterpret_cast<uint4*>(sg) = *reinterpret_cast<const uint4*>(sg + 16u * nfull);
                    g0 += 16u * nfull;
                }
                fill = end & (nfull ? 15u : ~0u);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            } else {
                if (fill > lo0) put_part(a.text + g0, sg, lo0, fill, lane);
                if (v) {
                    uint8_t* o = a.text + g0 + fill + (incl - len);
                    if (k.w == 0xFFFFFFFFu) { /* long term (a short key always holds its TAB): corpus bytes */
                        /* the prefix's zero tail lies inside the word (a long term has >= 16 bytes) */
                        st16(o, pre_lo, pre_hi);
                        o += 4u + nid;
                        const uint8_t* src = a.corpus + ((((uint64_t)k.y << 32) | k.x) & 0xFFFFFFFFFFull);
                        for (uint32_t j = 0; j < wl; ++j) o[j] = src[j];
                        o += wl;
                        *o++ = '\t';
                        put_score(o, sc);
                        o[sc.ni + 17u] = '\n';
                    } else {
                        put_line(o, pre_lo, pre_hi, nid, k, wl, sc);
                    }
                }
                const uint64_t nb = g0 + fill + tot;
                g0 = nb & ~15ull;
                fill = lo0 = (uint32_t)(nb & 15u);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        if (fill > lo0) put_part(a.text + g0, sg, lo0, fill, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

/* tests / diagnostics: "%.16f" of n values into 32-byte NUL-padded slots */
__global__ void k_format_f64(const double* __restrict__ v, uint64_t n, uint8_t* __restrict__ out,
                             uint32_t* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t* o = out + i * 32;
    for (int j = 0; j < 32; ++j) o[j] = 0;
    Score sc;
    if (!fixed16(v[i], sc.q)) { atomicOr(status, ST_BOUNDS); return; }
    sc.ip = (uint32_t)v[i];
    sc.ni = ndig3(sc.ip);
    put_score(o, sc);
}

}  // namespace

int launch_term_meta(const uint4* vkeys, const uint64_t* vrep, const uint32_t* slot_of_rank, uint32_t V,
                     uint4* tkey, uint32_t* tlen, hipStream_t s) {
    if (!V) return 0;
    k_term_meta<<<grid_for(V), NT, 0, s>>>(vkeys, vrep, slot_of_rank, V, tkey, tlen);
    return ok();
}

static unsigned emit_grid(uint32_t ndocs) {
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const uint32_t need = (ndocs + NT / 64 - 1) / (NT / 64);
    const uint32_t cap = (uint32_t)ncu * 8u;
    return need < cap ? (need ? need : 1u) : cap;
}

int launch_emit_bytes(const EmitLaunch& e, uint64_t* doc_bytes, hipStream_t s) {
    if (!e.ndocs) return 0;
    EmitArgs a{e.order, e.doc_ids, e.out_off, e.term, e.score, e.tkey, e.tlen, e.corpus, 0u, e.ndocs,
               doc_bytes, nullptr, nullptr, e.status};
    k_doc_text_bytes<<<emit_grid(e.ndocs), NT, 0, s>>>(a);
    return ok();
}

int launch_emit_write(const EmitLaunch& e, const uint64_t* doc_text, uint8_t* text, hipStream_t s, uint32_t d0,
                      uint32_t d1) {
    if (d1 > e.ndocs) d1 = e.ndocs;
    if (d0 >= d1) return 0;
    EmitArgs a{e.order, e.doc_ids, e.out_off, e.term, e.score, e.tkey, e.tlen, e.corpus, d0, d1,
               nullptr, doc_text, text, e.status};
    k_doc_text_write<<<emit_grid(d1 - d0), NT, 0, s>>>(a);
    return ok();
}

int launch_format_f64(const double* v, uint64_t n, uint8_t* out, uint32_t* status, hipStream_t s) {
    if (!n) return 0;
    k_format_f64<<<grid_for(n), NT, 0, s>>>(v, n, out, status);
    return ok();
}
