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
 * across XCDs, device-scope atomics are). */
__device__ __forceinline__ uint32_t vocab_insert_s(uint4* __restrict__ keys, uint64_t* __restrict__ reps, uint64_t mask,
                                                uint64_t klo, uint64_t khi, uint64_t rep, uint32_t* status) {
    uint64_t h = key_hash(klo, khi) & mask;
    for (uint32_t probe = 0; probe < VOCAB_MAX_PROBE && probe <= mask; ++probe, h = (h + 1) & mask) {
        if ((probe & 63u) == 63u && (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ST_VOCAB_FULL))
            return INVALID_SLOT;
        unsigned long long* slot = reinterpret_cast<unsigned long long*>(&keys[h]);
        uint4 s = keys[h];
        uint64_t lo = ((uint64_t)s.y << 32) | s.x, hi = ((uint64_t)s.w << 32) | s.z;
        if (hi == khi && lo == klo) return (uint32_t)h;
        if (hi != KEY_EMPTY_HI && hi != KEY_PENDING_HI) continue;
        if (hi == KEY_EMPTY_HI) {
            unsigned long long old = atomicCAS(&slot[1], (unsigned long long)KEY_EMPTY_HI,
                                               (unsigned long long)KEY_PENDING_HI);
            if (old == KEY_EMPTY_HI) {
                atomicExch(&slot[0], (unsigned long long)klo);
                if ((khi >> 56) == 0xFFu) {   /* once per distinct long term */
                    reps[h] = rep;
                    atomicOr(status, ST_HAS_LONG);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                atomicExch(&slot[1], (unsigned long long)khi);
                return (uint32_t)h;
            }
            hi = old;
        }
        uint32_t spins = 0;
        while (hi == KEY_PENDING_HI) {
            __builtin_amdgcn_s_sleep(2);
            hi = atomicOr(&slot[1], 0ull);
            if (++spins > (1u << 24)) { atomicOr(status, ST_VOCAB_SPIN); return INVALID_SLOT; }
        }
        if (hi == khi) {
            lo = atomicOr(&slot[0], 0ull);
            if (lo == klo) return (uint32_t)h;
        }
    }
    atomicOr(status, ST_VOCAB_FULL);
    return INVALID_SLOT;
}
/* ---- hot terms (k_tokcount_lean) ----
 * The first HOT_MAX distinct short terms of <= 13 bytes inserted during a run get a hot id
 * (first come, first served: in a Zipfian stream the early arrivals are mostly the frequent
 * terms — on c2 the first 1024 cover ~66 % of the tokens).  The id is published inside the
 * key itself, in bytes 14-15 (zero for such terms): byte 15 = 0x80 | id >> 8, byte 14 =
 * id & 0xFF, so the slot load that finds a term also tells whether it is hot (no other
 * sentinel or key has byte 15 in 0x80..0x87).  hot_slot[id] = its slot.  After K1 the
 * marks are cleared again (k_hot_unmark): every later stage sees plain keys. */
#define HOT_MAX 1024u
#define HOT_NONE 0xFFFFu
__device__ __forceinline__ bool hot_hi(uint64_t hi) { return (hi >> 59) == 0x10u; }
__device__ __forceinline__ uint64_t unhot_hi(uint64_t hi) { return hot_hi(hi) ? (hi & 0x0000FFFFFFFFFFFFull) : hi; }
__device__ __forceinline__ uint32_t hot_id_of(uint64_t hi) { return hot_hi(hi) ? (uint32_t)(hi >> 48) & 0x7FFu : HOT_NONE; }
/* the same on the key's last dword (bytes 12-15) */
__device__ __forceinline__ bool hot_w(uint32_t w) { return (w >> 27) == 0x10u; }
__device__ __forceinline__ uint32_t unhot_w(uint32_t w) { return hot_w(w) ? (w & 0xFFFFu) : w; }
__device__ __forceinline__ uint32_t hot_id_w(uint32_t w) { return hot_w(w) ? (w >> 16) & 0x7FFu : HOT_NONE; }

/* vocab_insert_s for a table that may hold hot marks: keys compare without them, and a
 * claim of a new eligible term takes the next hot id while there is one (*hot_closed: a
 * workgroup-local flag set once the ids ran out, so a high-cardinality run stops touching
 * the counter).  *hid = the term's hot id or HOT_NONE. */
__device__ __forceinline__ uint32_t vocab_insert_hot(uint4* __restrict__ keys, uint64_t* __restrict__ reps, uint64_t mask,
                                                     uint64_t klo, uint64_t khi, uint64_t rep, uint32_t* status,
                                                     uint32_t* hot_slot, uint32_t* hot_ctr, uint32_t* hot_closed,
                                                     uint32_t* hid) {
    *hid = HOT_NONE;
    uint64_t h = key_hash(klo, khi) & mask;
    for (uint32_t probe = 0; probe < VOCAB_MAX_PROBE && probe <= mask; ++probe, h = (h + 1) & mask) {
        if ((probe & 63u) == 63u && (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ST_VOCAB_FULL))
            return INVALID_SLOT;
        unsigned long long* slot = reinterpret_cast<unsigned long long*>(&keys[h]);
        uint4 s = gload(&keys[h]);
        uint64_t lo = ((uint64_t)s.y << 32) | s.x, hi = ((uint64_t)s.w << 32) | s.z;
        if (unhot_hi(hi) == khi && lo == klo) { *hid = hot_id_of(hi); return (uint32_t)h; }
        if (hi != KEY_EMPTY_HI && hi != KEY_PENDING_HI) continue;
        if (hi == KEY_EMPTY_HI) {
            unsigned long long old = atomicCAS(&slot[1], (unsigned long long)KEY_EMPTY_HI,
                                               (unsigned long long)KEY_PENDING_HI);
            if (old == KEY_EMPTY_HI) {
                atomicExch(&slot[0], (unsigned long long)klo);
                uint64_t pub = khi;
                if ((khi >> 48) == 0 && !*hot_closed) {   /* a short term of <= 13 bytes */
                    const uint32_t id = atomicAdd(hot_ctr, 1u);
                    if (id < HOT_MAX) {
                        pub = khi | ((uint64_t)(0x80u | (id >> 8)) << 56) | ((uint64_t)(id & 0xFFu) << 48);
                        atomicExch(&hot_slot[id], (uint32_t)h);
                        *hid = id;
                    } else {
                        *hot_closed = 1u;
                    }
                }
                if ((khi >> 56) == 0xFFu) {   /* once per distinct long term */
                    reps[h] = rep;
                    atomicOr(status, ST_HAS_LONG);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                atomicExch(&slot[1], (unsigned long long)pub);
                return (uint32_t)h;
            }
            hi = old;
        }
        uint32_t spins = 0;
        while (hi == KEY_PENDING_HI) {
            __builtin_amdgcn_s_sleep(2);
            hi = atomicOr(&slot[1], 0ull);
            if (++spins > (1u << 24)) { atomicOr(status, ST_VOCAB_SPIN); return INVALID_SLOT; }
        }
        if (unhot_hi(hi) == khi) {
            lo = atomicOr(&slot[0], 0ull);
            if (lo == klo) { *hid = hot_id_of(hi); return (uint32_t)h; }
        }
    }
    atomicOr(status, ST_VOCAB_FULL);
    return INVALID_SLOT;
}

__device__ __forceinline__ uint32_t vocab_insert(const VocabDev& v, uint64_t klo, uint64_t khi, uint64_t rep,
                                                 uint32_t* status) {
    return vocab_insert_s(v.keys, v.rep, v.mask, klo, khi, rep, status);
}

#endif
