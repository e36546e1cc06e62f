/*
 * CPU test of the DF exchange's abort protocol (parallel-systems-mpi-tfidf_amd/csrc/comm_rank.h)
 * with a fake communicator: a collective completes only when every rank of the clique has
 * issued it, so a rank waiting for a failed peer stays "in progress" until it is released.
 * The reference's failure mode is exit() + mpirun killing the peers (TFIDF.c:122,137); the
 * property checked here is that no rank is left waiting and no communicator is left
 * un-aborted once a rank failed.
 *
 * Built and run by tests/test_comm_abort_cpu.py:  g++ -std=c++17 -O1 -pthread ... && ./a.out
 * Prints one line per scenario and "ALL OK" at the end; exits non-zero on a failure.
 */
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "comm_init.h"
#include "comm_rank.h"

namespace {

/* the fake clique: issued[k] = ranks that issued collective k; a communicator is an index
 * into `aborted` + 1 (0 = none) */
struct FakeNet {
    int nranks = 0;
    std::mutex mu;
    std::vector<int> issued;              /* per collective index */
    std::vector<int> next;                /* per rank: index of its next collective */
    std::vector<std::atomic<int>> aborts; /* per rank: ncclCommAbort calls */
    std::vector<int> pending;             /* per rank: the collective it waits for, -1 none */
    explicit FakeNet(int n) : nranks(n), issued(64, 0), next(n, 0), aborts(n), pending(n, -1) {
        for (auto& a : aborts) a = 0;
    }
};
FakeNet* g_net = nullptr;

struct FakeB {
    using Comm = int;   /* rank + 1 */
    static int async(Comm c) {
        FakeNet& n = *g_net;
        const int r = c - 1;
        std::lock_guard<std::mutex> lk(n.mu);
        if (n.aborts[r].load()) return TFIDF_E_RCCL;   /* a call on an aborted communicator */
        const int k = n.pending[r];
        if (k < 0) return 0;
        if (n.issued[k] == n.nranks) {
            n.pending[r] = -1;
            return 0;
        }
        return 1;
    }
    static void abort(Comm c) { g_net->aborts[c - 1].fetch_add(1); }
};

/* issues this rank's next collective (non-blocking: "in progress" until all ranks issued it) */
int fake_collective(int c) {
    FakeNet& n = *g_net;
    const int r = c - 1;
    std::lock_guard<std::mutex> lk(n.mu);
    const int k = n.next[r]++;
    ++n.issued[k];
    n.pending[r] = k;
    return 1;
}

struct Outcome {
    int rc = 0;
    double ms = 0;
    bool dead = false;
};

/* every rank runs `ncoll` collectives, each followed by a wait for its "kernels" (a stream that
 * is done once the collective completed); rank `fail_rank` fails after `fail_after` of them */
std::vector<Outcome> run_clique(int nranks, int ncoll, int fail_rank, int fail_after, int64_t timeout_ms,
                                bool shared_flag, bool fail_in_stream_wait) {
    FakeNet net(nranks);
    g_net = &net;
    auto shared = std::make_shared<CommShared>();
    std::vector<Outcome> out(nranks);
    std::vector<std::thread> th;
    for (int r = 0; r < nranks; ++r) {
        th.emplace_back([&, r] {
            CommRank<FakeB> cr;
            cr.comm = r + 1;
            if (shared_flag) cr.shared = shared;
            cr.timeout_ms = timeout_ms;
            const auto t0 = std::chrono::steady_clock::now();
            int rc = 0;
            for (int k = 0; k < ncoll && !rc; ++k) {
                if (r == fail_rank && k == fail_after && !fail_in_stream_wait) {
                    cr.fail();   /* a rank-local error between collectives (engine: xp->abort()) */
                    rc = TFIDF_E_HIP;
                    break;
                }
                rc = cr.enqueue([](int c) { return fake_collective(c); });
                if (rc) break;
                if (r == fail_rank && k == fail_after && fail_in_stream_wait) {
                    /* this rank's "kernels" fail while it waits for them */
                    rc = cr.wait_stream([] { return TFIDF_E_HIP; });
                    break;
                }
                rc = cr.wait_stream([&] { return FakeB::async(cr.comm) == 1 ? 1 : 0; });
            }
            out[r].rc = rc;
            out[r].dead = cr.dead;
            out[r].ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        });
    }
    for (auto& t : th) t.join();
    for (int r = 0; r < nranks; ++r)
        if (net.aborts[r].load() > 1) out[r].rc = 12345;   /* aborted twice: a bug */
    g_net = nullptr;
    return out;
}

/* a fake communicator init (comm_init.h) that blocks until the test opens its gate, as RCCL's
 * bootstrap blocks until every rank joined */
struct InitGate {
    std::mutex mu;
    std::condition_variable cv;
    bool open = false;
};
InitGate g_gate;
std::atomic<int> g_init_aborts{0};
struct FakeInitB {
    using Comm = int;
    static void abort(Comm) { g_init_aborts.fetch_add(1); }
};
int fake_init(int* c) {
    std::unique_lock<std::mutex> lk(g_gate.mu);
    g_gate.cv.wait(lk, [] { return g_gate.open; });
    *c = 7;
    return TFIDF_OK;
}
double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int g_fail = 0;
void check(bool ok, const char* what) {
    printf("%s %s\n", ok ? "ok  " : "FAIL", what);
    if (!ok) g_fail = 1;
}

}  // namespace

int main() {
    {   /* success: nobody aborts */
        auto o = run_clique(4, 5, -1, 0, 0, true, false);
        bool ok = true;
        for (auto& x : o) ok &= x.rc == 0 && !x.dead;
        check(ok, "4 ranks, 5 collectives, no failure: all 0, no communicator aborted");
    }
    for (int fa = 0; fa < 3; ++fa) {   /* one rank fails between collectives; peers wait inside one */
        auto o = run_clique(4, 5, 2, fa, 0, true, false);
        bool ok = o[2].rc == TFIDF_E_HIP;
        for (int r = 0; r < 4; ++r) ok &= o[r].dead && o[r].ms < 5000;
        for (int r = 0; r < 4; ++r)
            if (r != 2) ok &= o[r].rc == TFIDF_E_PEER;
        char msg[160];
        snprintf(msg, sizeof msg,
                 "rank 2 fails before collective %d: it returns its error, ranks 0,1,3 TFIDF_E_PEER, every "
                 "communicator aborted exactly once, no deadline needed",
                 fa);
        check(ok, msg);
    }
    {   /* the failing rank's own kernels fail while its peers wait for the next collective */
        auto o = run_clique(3, 4, 0, 1, 0, true, true);
        bool ok = o[0].rc == TFIDF_E_HIP;
        for (int r = 0; r < 3; ++r) ok &= o[r].dead && o[r].ms < 5000;
        for (int r = 1; r < 3; ++r) ok &= o[r].rc == TFIDF_E_PEER;
        check(ok, "rank 0's stream wait fails: ranks 1,2 released with TFIDF_E_PEER, all communicators aborted");
    }
    {   /* process per GPU: no shared flag; a peer that never comes is noticed by the deadline */
        auto o = run_clique(2, 3, 1, 1, 300, false, false);
        bool ok = o[1].rc == TFIDF_E_HIP && o[0].rc == TFIDF_E_PEER && o[0].dead && o[1].dead;
        ok &= o[0].ms >= 250 && o[0].ms < 5000;
        check(ok, "process per GPU: the waiting rank gives up after its 300 ms deadline and aborts its communicator");
    }
    {   /* a call after the abort is refused without touching the network */
        FakeNet net(2);
        g_net = &net;
        CommRank<FakeB> a;
        a.comm = 1;
        a.fail();
        const int rc = a.enqueue([](int c) { return fake_collective(c); });
        check(rc == TFIDF_E_PEER && net.issued[0] == 0 && net.aborts[0].load() == 1,
              "an aborted rank's next call returns TFIDF_E_PEER and issues nothing");
        g_net = nullptr;
    }
    {   /* an init whose peers never join: the caller gets TFIDF_E_PEER at its deadline */
        int comm = -1, live = 0, ab = 0;
        auto t0 = std::chrono::steady_clock::now();
        const int rc = comm_init_with_deadline<FakeInitB>([](int* c) { return fake_init(c); }, 200, &comm, "test");
        const double ms = ms_since(t0);
        comm_init_counts(&live, &ab);
        check(rc == TFIDF_E_PEER && comm == 0 && ms >= 150 && ms < 5000 && live == 1 && ab == 1,
              "init never completes: TFIDF_E_PEER after the 200 ms deadline, one abandoned helper");
        /* a second init while that helper is still blocked: refused at once, no new thread */
        t0 = std::chrono::steady_clock::now();
        const int rc2 = comm_init_with_deadline<FakeInitB>([](int* c) { return fake_init(c); }, 200, &comm, "test");
        const double ms2 = ms_since(t0);
        comm_init_counts(&live, &ab);
        check(rc2 == TFIDF_E_PEER && ms2 < 100 && live == 1 && ab == 1,
              "a second init while the first is blocked: refused at once, still one helper thread");
        /* the peers join late: the abandoned helper aborts the communicator nobody takes, and exits */
        {
            std::lock_guard<std::mutex> lk(g_gate.mu);
            g_gate.open = true;
        }
        g_gate.cv.notify_all();
        t0 = std::chrono::steady_clock::now();
        do {
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            comm_init_counts(&live, &ab);
        } while ((live || ab) && ms_since(t0) < 5000);
        check(live == 0 && ab == 0 && g_init_aborts.load() == 1,
              "the late init's communicator is aborted and its helper thread exits (nothing left)");
        /* and the process can create a communicator again */
        const int rc3 = comm_init_with_deadline<FakeInitB>([](int* c) { return fake_init(c); }, 200, &comm, "test");
        do {
            comm_init_counts(&live, &ab);
        } while (live && ms_since(t0) < 5000);
        check(rc3 == TFIDF_OK && comm == 7 && g_init_aborts.load() == 1 && live == 0,
              "a later init succeeds and hands its communicator to the caller (not aborted)");
    }
    printf(g_fail ? "FAILED\n" : "ALL OK\n");
    return g_fail;
}
