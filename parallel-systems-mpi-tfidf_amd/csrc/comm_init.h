/*
 * comm_init.h — communicator creation with a deadline, host-only and independent of RCCL so
 * that it is tested on the CPU (tests/native/comm_abort_test.cpp: a fake init that blocks
 * until the test releases it).
 *
 * The reference's ranks are created by mpirun and a missing one stops the job from outside
 * (TFIDF.c:78-92, 122, 137).  Here a rank joins a communicator itself (tfidf_comm_init), and
 * RCCL 2.27's ncclCommInitRankConfig blocks its caller in the bootstrap until every rank has
 * joined, even for a non-blocking communicator (round 5, measured on the GPU box).  So:
 *
 *   - the init runs on a helper thread and the caller waits for it at most the deadline
 *     (TFIDF_COMM_TIMEOUT_S): a peer that never joins gives TFIDF_E_PEER, not a hang;
 *   - a helper whose caller gave up is "abandoned": if its init ever returns (the peers
 *     join late), it aborts the communicator nobody will use and exits, so its thread, socket
 *     and RCCL state are reclaimed then;
 *   - a helper blocked in the bootstrap cannot be interrupted, so at most ONE abandoned helper
 *     exists per process: while one is still blocked, a further init is refused at once with
 *     TFIDF_E_PEER (it would block in the same bootstrap state) instead of starting another
 *     thread — a process leaks at most one blocked thread, whatever its callers retry.  The
 *     blocked helper holds no device memory: a communicator's buffers are allocated after the
 *     bootstrap it is waiting in.
 *
 * B (the backend) provides:
 *   typename B::Comm;                      a communicator handle, value-initialised = none
 *   static void B::abort(Comm)             aborts (frees) a communicator
 * and init(Comm*) -> TFIDF_OK or an error is the (possibly blocking) creation itself.
 */
#ifndef TFIDF_COMM_INIT_H
#define TFIDF_COMM_INIT_H

#include <stdint.h>
#include <stdio.h>

#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>

#include "../../include/tfidf.h"

/* the process's init helpers */
struct CommInitRegistry {
    std::mutex mu;
    std::condition_variable cv;
    int live = 0;        /* helper threads running */
    int abandoned = 0;   /* ... whose caller gave up (still blocked in their init) */
};
inline CommInitRegistry& comm_init_registry() {
    static CommInitRegistry* r = new CommInitRegistry();   /* never destroyed: a blocked helper may outlive main */
    return *r;
}

template <class B> struct CommInitJob {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    int rc = TFIDF_OK;
    typename B::Comm comm{};
};

/* Runs init(&comm) on a helper thread; waits for it at most timeout_ms (0: no deadline).
 * Returns TFIDF_OK with *out set, init's error, or TFIDF_E_PEER (deadline, or an earlier
 * abandoned init of this process still blocked). */
template <class B, class Init>
int comm_init_with_deadline(Init&& init, int64_t timeout_ms, typename B::Comm* out, const char* who) {
    *out = typename B::Comm{};
    CommInitRegistry& reg = comm_init_registry();
    {
        std::lock_guard<std::mutex> lk(reg.mu);
        if (reg.abandoned > 0) {
            fprintf(stderr,
                    "tfidf: %s: an earlier communicator init of this process is still blocked in its bootstrap "
                    "(its peers never joined); refusing another one\n",
                    who);
            return TFIDF_E_PEER;
        }
        ++reg.live;
    }
    auto job = std::make_shared<CommInitJob<B>>();
    std::thread([job, init = std::forward<Init>(init)]() mutable {
        typename B::Comm comm{};
        const int rc = init(&comm);
        bool abandoned;
        {
            std::lock_guard<std::mutex> lk(job->mu);
            abandoned = job->abandoned;
            if ((abandoned || rc) && comm != typename B::Comm{}) B::abort(comm);   /* nobody takes it */
            job->rc = rc;
            job->comm = (abandoned || rc) ? typename B::Comm{} : comm;
            job->done = true;
            job->cv.notify_all();
        }
        CommInitRegistry& r = comm_init_registry();
        std::lock_guard<std::mutex> lk(r.mu);
        --r.live;
        if (abandoned) --r.abandoned;
        r.cv.notify_all();
    }).detach();
    std::unique_lock<std::mutex> lk(job->mu);
    const bool done = timeout_ms > 0
                          ? job->cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return job->done; })
                          : (job->cv.wait(lk, [&] { return job->done; }), true);
    if (!done) {
        job->abandoned = true;
        {
            std::lock_guard<std::mutex> rl(reg.mu);
            ++reg.abandoned;
        }
        fprintf(stderr, "tfidf: %s: the other ranks did not join within %lld s (TFIDF_COMM_TIMEOUT_S)\n", who,
                (long long)(timeout_ms / 1000));
        return TFIDF_E_PEER;
    }
    if (job->rc) return job->rc;
    *out = job->comm;
    return TFIDF_OK;
}

/* Communicators whose init timed out after it returned handles (a clique created in one
 * group call): aborted on a helper thread, counted as abandoned until the aborts return (an
 * abort may wait in the same bootstrap), so the caller never blocks on them. */
template <class B, class V> void comm_reap_async(V comms) {
    CommInitRegistry& reg = comm_init_registry();
    {
        std::lock_guard<std::mutex> lk(reg.mu);
        ++reg.live;
        ++reg.abandoned;
    }
    std::thread([comms = std::move(comms)]() mutable {
        for (auto& c : comms)
            if (c != typename B::Comm{}) B::abort(c);
        CommInitRegistry& r = comm_init_registry();
        std::lock_guard<std::mutex> lk(r.mu);
        --r.live;
        --r.abandoned;
        r.cv.notify_all();
    }).detach();
}

/* tests: the helpers of this process (running, abandoned) */
inline void comm_init_counts(int* live, int* abandoned) {
    CommInitRegistry& reg = comm_init_registry();
    std::lock_guard<std::mutex> lk(reg.mu);
    *live = reg.live;
    *abandoned = reg.abandoned;
}

#endif
