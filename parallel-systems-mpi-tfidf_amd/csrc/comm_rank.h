/*
 * comm_rank.h — the abort protocol of the DF exchange's RCCL ranks, host-only and
 * independent of RCCL so that the state machine itself is tested on the CPU
 * (tests/native/comm_abort_test.cpp, a fake communicator whose collectives complete only
 * when every rank issued them).
 *
 * The reference stops a failing rank with exit() and leaves mpirun to kill its peers
 * (TFIDF.c:100-103,120-123,135-138).  Here a failed rank must instead release peers that are
 * waiting for it inside a collective.  Communicators are created NON-BLOCKING
 * (ncclConfig_t.blocking = 0): no RCCL call ever blocks its thread — a call returns
 * ncclInProgress and its owner thread polls ncclCommGetAsyncError; a collective's device
 * work is waited for by polling the stream.  Every poll loop also watches the ranks' shared
 * `aborted` flag (and a deadline), so:
 *
 *   - a rank that fails sets `aborted` and aborts its OWN communicator (fail());
 *   - every other rank of the clique sees the flag at its next poll — whether it is inside
 *     an RCCL call (lazy connection set-up waiting for the failed peer), waiting for a
 *     collective's kernels, or between calls (the next enqueue) — and aborts its own
 *     communicator, which also releases kernels still waiting for the failed peer;
 *   - no thread ever touches another rank's communicator, so no lock is needed and there is
 *     no window in which a blocked peer is skipped (the round-4 clique gave up on a rank
 *     whose lock it could not take within ~2 s).
 *
 * With one process per GPU (tfidf_comm_init) the flag is process-local; a peer process that
 * died is noticed by the deadline (TFIDF_COMM_TIMEOUT_S, default 600 s) or by an error that
 * RCCL reports through ncclCommGetAsyncError.
 *
 * B (the backend) provides:
 *   typename B::Comm;                 a communicator handle, value-initialised = none
 *   static int  B::async(Comm)        0 done, 1 in progress, < 0 a TFIDF_E_* error
 *   static void B::abort(Comm)        aborts this rank's communicator (called once, by its owner)
 */
#ifndef TFIDF_COMM_RANK_H
#define TFIDF_COMM_RANK_H

#include <stdint.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <memory>
#include <thread>

#include "../../include/tfidf.h"

/* what the ranks that fail together share: one tfidf_group clique, or a single
 * process-per-GPU rank */
struct CommShared {
    std::atomic<bool> aborted{false};
};

template <class B> struct CommRank {
    typename B::Comm comm{};
    bool dead = false;                  /* this rank's communicator was aborted */
    std::shared_ptr<CommShared> shared;
    int64_t timeout_ms = 0;             /* 0: no deadline */
    std::atomic<uint64_t>* polls = nullptr;   /* tests: poll iterations (optional) */

    CommRank() : shared(std::make_shared<CommShared>()) {}

    bool aborted() const { return shared->aborted.load(std::memory_order_acquire); }
    /* owner thread only */
    void abort_own() {
        if (!dead && comm != typename B::Comm{}) B::abort(comm);
        dead = true;
    }
    /* this rank failed: every rank of the clique gives up, this one at once */
    void fail() {
        shared->aborted.store(true, std::memory_order_release);
        abort_own();
    }
    /* poll() until it reports done (0) or an error (< 0); gives up with TFIDF_E_PEER when the
     * clique is aborted or the deadline passes (both abort this rank's communicator) */
    template <class Poll> int wait(Poll&& poll) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 0;; ++spin) {
            if (polls) polls->fetch_add(1, std::memory_order_relaxed);
            const int st = poll();
            if (st <= 0) {
                if (st < 0) fail();
                return st;
            }
            if (aborted()) {
                abort_own();
                return TFIDF_E_PEER;
            }
            if (timeout_ms > 0 && std::chrono::duration_cast<std::chrono::milliseconds>(
                                      std::chrono::steady_clock::now() - t0).count() > timeout_ms) {
                fail();
                return TFIDF_E_PEER;
            }
            if (spin < 64) std::this_thread::yield();
            else std::this_thread::sleep_for(std::chrono::microseconds(spin < 1024 ? 20 : 200));
        }
    }
    /* issue(comm): 0 issued, 1 in progress, < 0 error; then the call's completion */
    template <class Issue> int enqueue(Issue&& issue) {
        if (dead || aborted()) {
            abort_own();
            return TFIDF_E_PEER;
        }
        const int r = issue(comm);
        if (r < 0) {
            fail();
            return r;
        }
        return wait([&] { return B::async(comm); });
    }
    /* query(): 0 the stream's work is done, 1 not yet, < 0 error.  While it runs the
     * communicator's asynchronous errors are watched too. */
    template <class Query> int wait_stream(Query&& query) {
        return wait([&] {
            const int q = query();
            if (q != 1 || dead) return q;
            const int a = B::async(comm);
            return a < 0 ? a : 1;
        });
    }
};

/* TFIDF_COMM_TIMEOUT_S (seconds, 0 = none), default 600 */
inline int64_t comm_timeout_ms_from_env() {
    const char* e = getenv("TFIDF_COMM_TIMEOUT_S");
    if (!e || !*e) return 600000;
    const long long v = atoll(e);
    return v > 0 ? (int64_t)v * 1000 : 0;
}

#endif
