/*
 * group.cpp — several GPU shards driven by one process (the drop-in for
 * `mpirun -np P ./TFIDF`, TFIDF.c:82-92,125-130), and the two rank transports of
 * xport.h.
 *
 *   tfidf_group_open   opens one context per rank (rank r on devices[r]) and connects
 *                      them: ncclCommInitAll when every rank has its own GPU (RCCL over
 *                      xGMI), the in-process LocalXport when a device carries several
 *                      ranks (or TFIDF_GROUP_LOCAL is asked for).
 *   tfidf_group_run    one host thread per rank, each runs tfidf_run on its shard; the
 *                      ranks meet only inside the DF exchange (engine.cpp).
 *   tfidf_group_write_output
 *                      every rank formats its lines on its GPU (in parallel), then the
 *                      texts are written in rank order — shards are contiguous ranges of
 *                      the "docN@" order, so this is the reference's gather + qsort
 *                      (TFIDF.c:253-273) without either.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/tfidf.h"
#include "kernels.h"
#include "xport.h"
#include "comm_rank.h"
#include "comm_init.h"

namespace {

/* ------------------------------------------------------------------ RCCL -- */

/* RCCL behind comm_rank.h's abort protocol: communicators are non-blocking, every call and
 * every wait for a collective's kernels is a poll that also watches the clique's `aborted`
 * flag, and each rank only ever aborts its own communicator (from its own thread). */
struct RcclB {
    using Comm = ncclComm_t;
    static int async(Comm c) {
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(c, &st) != ncclSuccess) return TFIDF_E_RCCL;
        return st == ncclInProgress ? 1 : (st == ncclSuccess ? 0 : TFIDF_E_RCCL);
    }
    static void abort(Comm c) { (void)ncclCommAbort(c); }
};
static int nccl_issue(ncclResult_t r) { return r == ncclSuccess ? 0 : (r == ncclInProgress ? 1 : TFIDF_E_RCCL); }

/* Finalizes (non-blocking: all at once, then polled) and destroys the live communicators of
 * one process — a clique's ranks must not be finalized one after the other, since a
 * finalize may wait for the peers'. Communicators that do not finalize within the deadline
 * are aborted. */
static void comms_close(std::vector<ncclComm_t>& comms, int64_t timeout_ms) {
    std::vector<int> st(comms.size(), 0);   /* 1 finalizing, 2 finalized, -1 failed */
    for (size_t r = 0; r < comms.size(); ++r)
        if (comms[r]) st[r] = nccl_issue(ncclCommFinalize(comms[r])) < 0 ? -1 : 1;
    const auto t0 = std::chrono::steady_clock::now();
    for (bool busy = true; busy;) {
        busy = false;
        for (size_t r = 0; r < comms.size(); ++r) {
            if (st[r] != 1) continue;
            const int a = RcclB::async(comms[r]);
            if (a == 1) busy = true;
            else st[r] = a == 0 ? 2 : -1;
        }
        if (busy && timeout_ms > 0 && std::chrono::duration_cast<std::chrono::milliseconds>(
                                          std::chrono::steady_clock::now() - t0).count() > timeout_ms) {
            for (size_t r = 0; r < comms.size(); ++r)
                if (st[r] == 1) st[r] = -1;
            break;
        }
        if (busy) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    for (size_t r = 0; r < comms.size(); ++r) {
        if (!comms[r]) continue;
        if (st[r] == 2) (void)ncclCommDestroy(comms[r]);
        else (void)ncclCommAbort(comms[r]);
        comms[r] = nullptr;
    }
}

/* The communicators of one tfidf_group clique (one process, one host thread per rank).
 * Created together (non-blocking ncclCommInitRankConfig in one group), closed together;
 * during runs rank r's communicator is touched by rank r's thread only. */
struct Clique {
    std::vector<ncclComm_t> comms;
    std::vector<char> dead;                 /* rank r aborted its communicator (written by rank r) */
    std::shared_ptr<CommShared> shared = std::make_shared<CommShared>();
    int64_t timeout_ms = comm_timeout_ms_from_env();
    explicit Clique(int n) : comms((size_t)n, nullptr), dead((size_t)n, 0) {}
    ~Clique() {
        for (size_t r = 0; r < comms.size(); ++r)
            if (dead[r]) comms[r] = nullptr;   /* ncclCommAbort freed it */
        comms_close(comms, timeout_ms);
    }
};

/* polls every communicator of a non-blocking init until it is ready (0), failed or timed out */
static int comms_ready(std::vector<ncclComm_t>& comms, int64_t timeout_ms) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        bool busy = false;
        for (ncclComm_t c : comms) {
            const int a = c ? RcclB::async(c) : TFIDF_E_RCCL;
            if (a < 0) return a;
            busy |= a == 1;
        }
        if (!busy) return TFIDF_OK;
        if (timeout_ms > 0 && std::chrono::duration_cast<std::chrono::milliseconds>(
                                  std::chrono::steady_clock::now() - t0).count() > timeout_ms)
            return TFIDF_E_PEER;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

struct RcclXport final : Xport {
    CommRank<RcclB> cr;                    /* this rank's communicator and the clique's flag */
    std::shared_ptr<Clique> clique;        /* a tfidf_group clique owns the communicator; else this */
    int device = 0;
    uint64_t* dwords = nullptr;   /* 2 (send) + 2 * nranks (recv) */
    ~RcclXport() override {
        if (!clique && !cr.dead && cr.comm) {
            std::vector<ncclComm_t> one{cr.comm};
            comms_close(one, cr.timeout_ms);
        }
        if (dwords) (void)hipFree(dwords);
    }
    void note_dead() {
        if (clique && cr.dead) clique->dead[rank] = 1;
    }
    /* one RCCL call f(comm) and its completion; TFIDF_E_PEER once the clique was aborted */
    template <class F> int enqueue(F&& f) {
        const int rc = cr.enqueue([&](ncclComm_t c) { return nccl_issue(f(c)); });
        note_dead();
        return rc;
    }
    /* the stream's work (a collective's kernels among it) done, polled; an abort of the
     * clique aborts this rank's communicator, which releases kernels still waiting for a
     * failed peer, and the stream is then drained */
    int wait(hipStream_t s) override {
        const int rc = cr.wait_stream([&] {
            const hipError_t e = hipStreamQuery(s);
            return e == hipSuccess ? 0 : (e == hipErrorNotReady ? 1 : TFIDF_E_HIP);
        });
        (void)hipGetLastError();   /* hipErrorNotReady must not linger as the thread's last error */
        note_dead();
        if (rc) (void)hipStreamSynchronize(s);
        return rc;
    }
    int words(const uint64_t mine[2], uint64_t* all, hipStream_t s) override {
        if (!dwords && tfidf_dev_malloc((void**)&dwords, 16 * (size_t)(nranks + 1)) != hipSuccess) return TFIDF_E_NOMEM;
        if (hipMemcpyAsync(dwords, mine, 16, hipMemcpyHostToDevice, s) != hipSuccess) return TFIDF_E_HIP;
        int rc = enqueue([&](ncclComm_t c) { return ncclAllGather(dwords, dwords + 2, 2, ncclUint64, c, s); });
        if (rc) return rc;
        if (hipMemcpyAsync(all, dwords + 2, 16 * (size_t)nranks, hipMemcpyDeviceToHost, s) != hipSuccess)
            return TFIDF_E_HIP;
        return wait(s);
    }
    int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        return enqueue([&](ncclComm_t c) { return ncclAllGather(send, recv, bytes, ncclUint8, c, s); });
    }
    int alltoallv(const void* send, const uint64_t* scnt, void* recv, const uint64_t* rcnt, size_t eb,
                  hipStream_t s) override {
        /* point-to-point pairs in one group: over xGMI every pair of GPUs has its own link */
        return enqueue([&](ncclComm_t c) {
            ncclResult_t r = ncclGroupStart();
            uint64_t so = 0, ro = 0;
            for (int p = 0; p < nranks && r == ncclSuccess; ++p) {
                if (scnt[p]) r = ncclSend((const uint8_t*)send + so * eb, scnt[p] * eb, ncclUint8, p, c, s);
                if (r == ncclSuccess && rcnt[p]) r = ncclRecv((uint8_t*)recv + ro * eb, rcnt[p] * eb, ncclUint8, p, c, s);
                so += scnt[p];
                ro += rcnt[p];
            }
            const ncclResult_t e = ncclGroupEnd();
            return (r != ncclSuccess && r != ncclInProgress) ? r : e;
        });
    }
    int allreduce_u32(uint32_t* buf, size_t n, hipStream_t s) override {
        return enqueue([&](ncclComm_t c) { return ncclAllReduce(buf, buf, n, ncclUint32, ncclSum, c, s); });
    }
    /* this rank failed between collectives: the clique gives up (each peer aborts its own
     * communicator at its next poll), this rank's communicator at once */
    void abort() override {
        cr.fail();
        note_dead();
    }
    const char* name() const override { return "rccl"; }
};

/* -------------------------------------------------------------- in-process -- */

struct Hub {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool poisoned = false;
    std::vector<const void*> ptr;
    std::vector<const void*> ptr2;   /* allreduce: every rank's reduced slice */
    std::vector<int> dev;
    std::vector<uint64_t> w;
    std::vector<uint64_t> sc;   /* alltoallv: rank r's count for peer p at sc[r * n + p] */
    /* returns false when a rank aborted */
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (poisoned) return false;
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        cv.wait(lk, [&] { return gen != g || poisoned; });
        return gen != g;   /* completed, or released by a poisoning rank */
    }
    void poison() {
        std::lock_guard<std::mutex> lk(mu);
        poisoned = true;
        cv.notify_all();
    }
    /* before a new group run, when no rank is inside the hub: an abort of the previous run
     * does not poison this one */
    void reset() {
        std::lock_guard<std::mutex> lk(mu);
        poisoned = false;
        arrived = 0;
    }
};

struct LocalXport final : Xport {
    Hub* hub = nullptr;
    int device = 0;
    /* every rank on this device (and few enough for one copy list): each collective is one
     * or two kernels reading the peers' buffers directly, instead of one copy per peer */
    bool one_device() const {
        if (nranks > XCOPY_MAX) return false;
        for (int r = 0; r < nranks; ++r)
            if (hub->dev[r] != device) return false;
        return true;
    }
    int words(const uint64_t mine[2], uint64_t* all, hipStream_t s) override {
        (void)s;
        hub->w[2 * rank] = mine[0];
        hub->w[2 * rank + 1] = mine[1];
        if (!hub->barrier()) return TFIDF_E_PEER;
        memcpy(all, hub->w.data(), 16 * (size_t)nranks);
        if (!hub->barrier()) return TFIDF_E_PEER;   /* nobody rewrites w before all have read */
        return TFIDF_OK;
    }
    int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        /* the send buffer is complete on this stream; peers copy from it after the barrier */
        if (hipStreamSynchronize(s) != hipSuccess) { abort(); return TFIDF_E_HIP; }
        hub->ptr[rank] = send;
        if (!hub->barrier()) return TFIDF_E_PEER;
        int rc = TFIDF_OK;
        if (bytes % 4 == 0 && one_device()) {
            XCopyList l;
            l.n = (uint32_t)nranks;
            l.off[0] = 0;
            for (int r = 0; r < nranks; ++r) {
                l.src[r] = (const uint32_t*)hub->ptr[r];
                l.dst[r] = (uint32_t*)((uint8_t*)recv + (size_t)r * bytes);
                l.off[r + 1] = l.off[r] + bytes / 4;
            }
            if (launch_xcopy(l, s)) rc = TFIDF_E_HIP;
        }
        for (int r = 0; r < nranks && !rc && bytes && !(bytes % 4 == 0 && one_device()); ++r) {
            uint8_t* dst = (uint8_t*)recv + (size_t)r * bytes;
            const hipError_t e = hub->dev[r] == device
                ? hipMemcpyAsync(dst, hub->ptr[r], bytes, hipMemcpyDeviceToDevice, s)
                : hipMemcpyPeerAsync(dst, device, hub->ptr[r], hub->dev[r], bytes, s);
            if (e != hipSuccess) rc = TFIDF_E_HIP;
        }
        if (hipStreamSynchronize(s) != hipSuccess) rc = TFIDF_E_HIP;
        if (rc) { abort(); return rc; }
        /* every rank has copied every send buffer before any of them is reused */
        if (!hub->barrier()) return TFIDF_E_PEER;
        return TFIDF_OK;
    }
    int alltoallv(const void* send, const uint64_t* scnt, void* recv, const uint64_t* rcnt, size_t eb,
                  hipStream_t s) override {
        if (hipStreamSynchronize(s) != hipSuccess) { abort(); return TFIDF_E_HIP; }
        hub->ptr[rank] = send;
        for (int p = 0; p < nranks; ++p) hub->sc[(size_t)rank * nranks + p] = scnt[p];
        if (!hub->barrier()) return TFIDF_E_PEER;
        int rc = TFIDF_OK;
        uint64_t ro = 0;
        const bool fast = eb % 4 == 0 && one_device();
        XCopyList l;
        l.n = 0;
        l.off[0] = 0;
        for (int p = 0; p < nranks && !rc; ++p) {
            /* peer p's segment for this rank starts after its segments for ranks < rank */
            uint64_t so = 0;
            for (int q = 0; q < rank; ++q) so += hub->sc[(size_t)p * nranks + q];
            const uint64_t n = hub->sc[(size_t)p * nranks + rank];
            if (n != rcnt[p]) rc = TFIDF_E_STATE;
            if (!rc && n && fast) {
                l.src[l.n] = (const uint32_t*)((const uint8_t*)hub->ptr[p] + so * eb);
                l.dst[l.n] = (uint32_t*)((uint8_t*)recv + ro * eb);
                l.off[l.n + 1] = l.off[l.n] + n * eb / 4;
                ++l.n;
            } else if (!rc && n) {
                uint8_t* dst = (uint8_t*)recv + ro * eb;
                const uint8_t* src = (const uint8_t*)hub->ptr[p] + so * eb;
                const hipError_t e = hub->dev[p] == device
                    ? hipMemcpyAsync(dst, src, n * eb, hipMemcpyDeviceToDevice, s)
                    : hipMemcpyPeerAsync(dst, device, src, hub->dev[p], n * eb, s);
                if (e != hipSuccess) rc = TFIDF_E_HIP;
            }
            ro += rcnt[p];
        }
        if (!rc && l.n && launch_xcopy(l, s)) rc = TFIDF_E_HIP;
        if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = TFIDF_E_HIP;
        if (rc) { abort(); return rc; }
        if (!hub->barrier()) return TFIDF_E_PEER;   /* no send buffer is reused before all copied */
        return TFIDF_OK;
    }
    /* every rank copies all ranks' vectors into its staging area (after a barrier: all are
     * complete), then (after a second barrier: nobody overwrites a vector still being read)
     * sums them into its own */
    uint32_t* stage = nullptr;
    size_t stage_n = 0;
    ~LocalXport() override {
        if (stage) (void)hipFree(stage);
    }
    int allreduce_u32(uint32_t* buf, size_t n, hipStream_t s) override {
        if (!n) return hub->barrier() && hub->barrier() && hub->barrier() ? TFIDF_OK : TFIDF_E_PEER;
        if (one_device()) return allreduce_slices(buf, n, s);
        if (stage_n < n * (size_t)nranks) {
            if (stage) (void)hipFree(stage);
            stage = nullptr;
            stage_n = 0;
            if (tfidf_dev_malloc((void**)&stage, n * (size_t)nranks * 4) != hipSuccess) { abort(); return TFIDF_E_NOMEM; }
            stage_n = n * (size_t)nranks;
        }
        if (hipStreamSynchronize(s) != hipSuccess) { abort(); return TFIDF_E_HIP; }
        hub->ptr[rank] = buf;
        if (!hub->barrier()) return TFIDF_E_PEER;
        int rc = TFIDF_OK;
        for (int r = 0; r < nranks && !rc; ++r) {
            const hipError_t e = hub->dev[r] == device
                ? hipMemcpyAsync(stage + (size_t)r * n, hub->ptr[r], n * 4, hipMemcpyDeviceToDevice, s)
                : hipMemcpyPeerAsync(stage + (size_t)r * n, device, hub->ptr[r], hub->dev[r], n * 4, s);
            if (e != hipSuccess) rc = TFIDF_E_HIP;
        }
        if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = TFIDF_E_HIP;
        if (rc) { abort(); return rc; }
        if (!hub->barrier()) return TFIDF_E_PEER;   /* every vector read before any is overwritten */
        if (launch_sum_rows_u32(stage, (uint32_t)nranks, n, buf, s)) { abort(); return TFIDF_E_HIP; }
        if (hipStreamSynchronize(s) != hipSuccess) { abort(); return TFIDF_E_HIP; }
        if (!hub->barrier()) return TFIDF_E_PEER;
        return TFIDF_OK;
    }
    /* one device: a reduce-scatter (rank r sums slice r of every rank's vector into its
     * staging) and an all-gather of the slices back into every vector; 2 launches per rank,
     * ~3n words of traffic instead of R copies of n words and a row sum */
    int allreduce_slices(uint32_t* buf, size_t n, hipStream_t s) {
        const size_t chunk = (n + nranks - 1) / nranks;
        if (stage_n < chunk) {
            if (stage) (void)hipFree(stage);
            stage = nullptr;
            stage_n = 0;
            if (tfidf_dev_malloc((void**)&stage, chunk * 4) != hipSuccess) { abort(); return TFIDF_E_NOMEM; }
            stage_n = chunk;
        }
        auto slice = [&](int r, size_t* lo) {
            *lo = chunk * r < n ? chunk * r : n;
            return (chunk * (r + 1) < n ? chunk * (r + 1) : n) - *lo;
        };
        if (hipStreamSynchronize(s) != hipSuccess) { abort(); return TFIDF_E_HIP; }
        hub->ptr[rank] = buf;
        hub->ptr2[rank] = stage;
        if (!hub->barrier()) return TFIDF_E_PEER;
        XCopyList l;
        l.n = (uint32_t)nranks;
        for (int r = 0; r < nranks; ++r) l.src[r] = (const uint32_t*)hub->ptr[r];
        size_t lo;
        const size_t len = slice(rank, &lo);
        int rc = launch_xsum_slice(l, lo, len, stage, s) ? TFIDF_E_HIP : TFIDF_OK;
        if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = TFIDF_E_HIP;
        if (rc) { abort(); return rc; }
        if (!hub->barrier()) return TFIDF_E_PEER;   /* every slice summed: the vectors are free */
        l.off[0] = 0;
        for (int r = 0; r < nranks; ++r) {
            const size_t m = slice(r, &lo);
            l.src[r] = (const uint32_t*)hub->ptr2[r];
            l.dst[r] = buf + lo;
            l.off[r + 1] = l.off[r] + m;
        }
        if (launch_xcopy(l, s)) rc = TFIDF_E_HIP;
        if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = TFIDF_E_HIP;
        if (rc) { abort(); return rc; }
        if (!hub->barrier()) return TFIDF_E_PEER;   /* every slice read before a staging is reused */
        return TFIDF_OK;
    }
    void abort() override { hub->poison(); }
    const char* name() const override { return "local"; }
};

}  // namespace

/* one rank of a process-per-GPU job (tfidf_comm_init): the init runs with a deadline on a
 * helper thread (comm_init.h: RCCL 2.27 blocks the caller in its bootstrap until every rank
 * joined; at most one abandoned helper per process) */
int rccl_init_rank(const void* unique_id, int rank, int nranks, int device, Xport** out) {
    *out = nullptr;
    ncclUniqueId u;
    memcpy(&u, unique_id, sizeof(u));
    const int64_t tmo = comm_timeout_ms_from_env();
    char who[64];
    snprintf(who, sizeof who, "rank %d of %d", rank, nranks);
    ncclComm_t comm = nullptr;
    const int rc = comm_init_with_deadline<RcclB>(
        [u, rank, nranks, device, tmo](ncclComm_t* c) -> int {
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 0;
            if (hipSetDevice(device) != hipSuccess) return TFIDF_E_HIP;
            if (nccl_issue(ncclCommInitRankConfig(c, nranks, u, rank, &cfg)) < 0 || !*c) return TFIDF_E_RCCL;
            std::vector<ncclComm_t> one{*c};
            return comms_ready(one, tmo);
        },
        tmo, &comm, who);
    if (rc) return rc;
    RcclXport* x = new RcclXport();
    x->cr.comm = comm;
    x->cr.timeout_ms = tmo;
    x->rank = rank;
    x->nranks = nranks;
    x->device = device;
    *out = x;
    return TFIDF_OK;
}

struct tfidf_group {
    int n = 0;
    bool local = false;
    std::vector<tfidf_ctx*> ctx;
    Hub* hub = nullptr;
};

extern "C" {

int tfidf_group_open(int nranks, const int* devices, uint32_t flags, tfidf_group** out) {
    if (!out || nranks < 1 || nranks > 1024) return TFIDF_E_INVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return TFIDF_E_NODEV;
    std::vector<int> dev((size_t)nranks);
    for (int r = 0; r < nranks; ++r) {
        dev[r] = devices ? devices[r] : r;
        if (dev[r] < 0 || dev[r] >= ndev) return TFIDF_E_NODEV;
    }
    bool distinct = true;
    for (int a = 0; a < nranks && distinct; ++a)
        for (int b = a + 1; b < nranks; ++b)
            if (dev[a] == dev[b]) { distinct = false; break; }
    tfidf_group* g = new tfidf_group();
    g->n = nranks;
    g->local = !distinct || (flags & TFIDF_GROUP_LOCAL) != 0;
    g->ctx.assign((size_t)nranks, nullptr);
    int rc = TFIDF_OK;
    for (int r = 0; r < nranks && !rc; ++r) rc = tfidf_open(dev[r], &g->ctx[r]);
    if (!rc && nranks > 1 && g->local) {
        g->hub = new Hub();
        g->hub->n = nranks;
        g->hub->ptr.assign((size_t)nranks, nullptr);
        g->hub->ptr2.assign((size_t)nranks, nullptr);
        g->hub->dev = dev;
        g->hub->w.assign(2 * (size_t)nranks, 0);
        g->hub->sc.assign((size_t)nranks * nranks, 0);
        for (int r = 0; r < nranks && !rc; ++r) {
            LocalXport* x = new LocalXport();
            x->hub = g->hub;
            x->rank = r;
            x->nranks = nranks;
            x->device = dev[r];
            rc = tfidf_ctx_attach_xport(g->ctx[r], x);
        }
    } else if (!rc) {
        /* one RCCL communicator per GPU of the clique (a 1-rank group gets one too, so the
         * exchange path is the same at every size), created non-blocking in one group and
         * owned by the clique: an error on one rank makes every rank abort its own */
        auto cl = std::make_shared<Clique>(nranks);
        ncclUniqueId u;
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (ncclGetUniqueId(&u) != ncclSuccess) rc = TFIDF_E_RCCL;
        if (!rc) {
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 0;
            int bad = nccl_issue(ncclGroupStart()) < 0;
            for (int r = 0; r < nranks && !bad; ++r) {
                if (hipSetDevice(dev[r]) != hipSuccess) bad = 1;
                else bad = nccl_issue(ncclCommInitRankConfig(&cl->comms[r], nranks, u, r, &cfg)) < 0;
            }
            if (nccl_issue(ncclGroupEnd()) < 0) bad = 1;
            (void)hipSetDevice(cur);
            if (bad) rc = TFIDF_E_RCCL;
            else rc = comms_ready(cl->comms, cl->timeout_ms);
            if (rc == TFIDF_E_PEER) {   /* timed out: aborted on a helper thread (an abort may wait in the
                                           same bootstrap; comm_init.h) */
                comm_reap_async<RcclB>(cl->comms);
                for (ncclComm_t& c : cl->comms) c = nullptr;
            } else if (rc) {   /* nothing usable: abort what was created */
                for (ncclComm_t& c : cl->comms)
                    if (c) { (void)ncclCommAbort(c); c = nullptr; }
            }
        }
        for (int r = 0; r < nranks && !rc; ++r) {
            RcclXport* x = new RcclXport();
            x->clique = cl;
            x->cr.comm = cl->comms[r];
            x->cr.shared = cl->shared;
            x->cr.timeout_ms = cl->timeout_ms;
            x->rank = r;
            x->nranks = nranks;
            x->device = dev[r];
            rc = tfidf_ctx_attach_xport(g->ctx[r], x);
        }
    }
    if (rc) {
        tfidf_group_close(g);
        return rc;
    }
    *out = g;
    return TFIDF_OK;
}

int tfidf_group_size(const tfidf_group* g) { return g ? g->n : 0; }

tfidf_ctx* tfidf_group_ctx(tfidf_group* g, int rank) {
    return (g && rank >= 0 && rank < g->n) ? g->ctx[rank] : nullptr;
}

int tfidf_group_run(tfidf_group* g, const tfidf_corpus* shards) {
    if (!g || !shards) return TFIDF_E_INVAL;
    std::vector<int> rc((size_t)g->n, TFIDF_OK);
    if (g->hub) g->hub->reset();   /* in-process ranks: a new run starts unpoisoned */
    std::vector<std::thread> th;
    for (int r = 1; r < g->n; ++r) th.emplace_back([&, r] { rc[r] = tfidf_run(g->ctx[r], &shards[r]); });
    rc[0] = tfidf_run(g->ctx[0], &shards[0]);
    for (auto& t : th) t.join();
    /* the first rank's own error; TFIDF_E_PEER only when no rank has a better reason */
    int peer = TFIDF_OK;
    for (int r = 0; r < g->n; ++r) {
        if (rc[r] == TFIDF_E_PEER) peer = TFIDF_E_PEER;
        else if (rc[r]) return rc[r];
    }
    return peer;
}

int tfidf_group_write_output(tfidf_group* g, const char* path) {
    if (!g || !path) return TFIDF_E_INVAL;
    std::vector<int> rc((size_t)g->n, TFIDF_OK);
    std::vector<uint64_t> nb((size_t)g->n, 0);
    {   /* every GPU formats its shard's lines at once */
        std::vector<std::thread> th;
        for (int r = 1; r < g->n; ++r) th.emplace_back([&, r] { rc[r] = tfidf_format(g->ctx[r], &nb[r]); });
        rc[0] = tfidf_format(g->ctx[0], &nb[0]);
        for (auto& t : th) t.join();
    }
    for (int r = 0; r < g->n; ++r)
        if (rc[r]) return rc[r];
    for (int r = 0; r < g->n; ++r) {
        const int e = tfidf_write_output_gpu(g->ctx[r], path, r > 0);
        if (e) return e;
    }
    return TFIDF_OK;
}

void tfidf_group_close(tfidf_group* g) {
    if (!g) return;
    for (tfidf_ctx* c : g->ctx)
        if (c) tfidf_close(c);
    delete g->hub;
    delete g;
}

}  // extern "C"
