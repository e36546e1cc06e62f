/* dev_vocab.h — the global HBM vocabulary: lock-free 128-bit key insert shared by the
 * tokenize+count kernels (term identity keys: dev_common.h). */
#ifndef TFIDF_DEV_VOCAB_H
#define TFIDF_DEV_VOCAB_H

#include "dev_common.h"
#include "kernels.h"

/* A probe run this long only happens in a table close to full (expected runs are a few
 * slots at the engine's load limits): the insert flags ST_VOCAB_FULL and the engine
 * retries with a larger table.  Once the flag is up, every other insert stops within 64
 * probes, so a run over a too-small table (e.g. config 4's 1e7 terms against the first
 * 1M-slot table) ends after about one pass of tokens instead of probing the full table
 * per token. */
#define VOCAB_MAX_PROBE 4096u

/* Lock-free find-or-insert of a 128-bit key into the global vocabulary.
 * A slot is {lo, hi}; hi is the claim word: EMPTY -> PENDING (CAS) -> key (exchange)
 * after lo has been exchanged in, so a 16-byte snapshot whose hi is a real key always
 * carries its lo.  Plain loads may return stale EMPTY/PENDING lines from this XCD's L2;
 * those cases are re-read at the memory side with atomics (MI355X L2s are not coherent
 * across XCDs, device-scope atomics are).  Every case runs in one loop body: a lane that
 * finds a slot PENDING re-reads it in its next iteration, so a lane of the same wave that
 * holds the claim publishes in the same pass of the body (no lane waits in an inner spin
 * loop that its wave's claimer might be scheduled behind); the wait is bounded.
 * Probing starts at the EVEN slot of the key's hash (home = hash & mask & ~1): the K1
 * kernels load a key's home pair (two 16-byte slots, one aligned 32-byte piece, never
 * wrapping) and find every key that sits in its home pair without a dependent load.  A
 * table probed by quads (HOME = ~3: four slots, one aligned 64-byte line) starts at a
 * multiple of four instead; one run uses one form throughout. */
/* Identity of a long term (>= 16 bytes: its key is a 120-bit hash, dev_common.h) is exact:
 * when a long key matches the incumbent, the incumbent's first occurrence (its rep: length
 * << 40 | corpus offset, published before the key) is compared with this occurrence byte by
 * byte, as TFIDF.c:152,172's strcmp would; two distinct terms sharing a hash are reported
 * (ST_LONG_COLLIDE, the run fails) instead of being merged. */
__device__ __noinline__ bool long_term_differs(const uint8_t* __restrict__ bytes, const uint64_t* reps, uint64_t h,
                                               uint64_t rep) {
    const uint64_t inc = atomicOr(const_cast<unsigned long long*>(reinterpret_cast<const unsigned long long*>(&reps[h])),
                                  0ull);   /* memory side: published before the key */
    if ((inc >> 40) != (rep >> 40)) return true;
    const uint64_t n = rep >> 40, a = inc & 0xFFFFFFFFFFull, b = rep & 0xFFFFFFFFFFull;
    if (a == b) return false;
    for (uint64_t i = 0; i < n; ++i)
        if (bytes[a + i] != bytes[b + i]) return true;
    return false;
}

template <uint64_t HOME = ~1ull>   /* home alignment: ~1 even pairs (tokcount_sl/st), ~3 quads */
__device__ __forceinline__ uint32_t vocab_insert_s(uint4* __restrict__ keys, uint64_t* __restrict__ reps, uint64_t mask,
                                                uint64_t klo, uint64_t khi, uint64_t rep, uint32_t* status,
                                                const uint8_t* __restrict__ bytes = nullptr) {
    uint64_t h = key_hash(klo, khi) & mask & HOME;
    uint32_t spins = 0;
    bool reread = false;
    for (uint32_t probe = 0; probe < VOCAB_MAX_PROBE && probe <= mask;) {
        if ((probe & 63u) == 63u && (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ST_VOCAB_FULL))
            return INVALID_SLOT;
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
                if ((khi >> 56) == 0xFFu) {   /* once per distinct long term */
                    atomicExch(reinterpret_cast<unsigned long long*>(&reps[h]), (unsigned long long)rep);
                    atomicOr(status, ST_HAS_LONG);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                atomicExch(&slot[1], (unsigned long long)khi);
                return (uint32_t)h;
            }
            reread = true;                 /* another lane claimed it: look again */
            continue;
        }
        if (hi == KEY_PENDING_HI) {
            if (++spins > (1u << 24)) { atomicOr(status, ST_VOCAB_SPIN); return INVALID_SLOT; }
            __builtin_amdgcn_s_sleep(2);
            reread = true;
            continue;
        }
        /* a published hi carries its lo (lo is written first, both in one line) */
        if (hi == khi && lo == klo) {
            if (bytes && (khi >> 56) == 0xFFu && long_term_differs(bytes, reps, h, rep)) {
                atomicOr(status, ST_LONG_COLLIDE);
                return INVALID_SLOT;
            }
            return (uint32_t)h;
        }
        h = (h + 1) & mask;
        ++probe;
    }
    atomicOr(status, ST_VOCAB_FULL);
    return INVALID_SLOT;
}
template <uint64_t HOME = ~1ull>
__device__ __forceinline__ uint32_t vocab_insert(const VocabDev& v, uint64_t klo, uint64_t khi, uint64_t rep,
                                                 uint32_t* status, const uint8_t* __restrict__ bytes = nullptr) {
    return vocab_insert_s<HOME>(v.keys, v.rep, v.mask, klo, khi, rep, status, bytes);
}

#endif
