/*
 * ingest.cpp — SURVEY §8f row 2: the reference's input contract read straight into HBM.
 *
 * Replaces the per-rank fopen/fscanf ingest of TFIDF.c:98-110 (N = entries of input/
 * other than "." and "..") and TFIDF.c:130-147 (documents input/doc1..docN, opened by
 * every rank for its round-robin share).  Instead of one malloc'd host copy followed by
 * one large H2D (tfidf_ingest_dir + tfidf_run), the corpus streams from the files into
 * HBM through a ring of pinned staging segments, so disk/page-cache reads and PCIe DMA
 * overlap:
 *
 *   scan   the directory entry count (N), then open+fstat of doc1..docN on a pool of
 *          threads -> sizes -> doc_off (exclusive prefix sum).  A document that cannot be
 *          opened is reported like TFIDF.c:134-138 (the smallest such i, TFIDF_E_NODOC).
 *   read   the corpus byte range is cut into SEG-byte segments; workers claim segments
 *          in order, pread() every document piece of their segment into pinned slot
 *          (j mod K), then issue the H2D of that slot on one copy stream.  A slot is
 *          reused only after the copy of segment j-K has completed (its event), and a
 *          worker only ever waits on a smaller segment, so the ring cannot deadlock.
 *
 * The result is a device corpus (TFIDF_CORPUS_DEVICE) whose buffers the context owns,
 * valid until the next ingest / host-corpus run / tfidf_close.  Host code only: no
 * kernels, no CPU compute on the path.
 */
#include <hip/hip_runtime.h>

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/tfidf.h"

/* engine.cpp: the context's host-input device buffers (grown as needed) */
int tfidf_ctx_ingest_buffers(tfidf_ctx* ctx, uint64_t nbytes, uint32_t ndocs, uint8_t** dbytes, uint64_t** doff);

namespace {

constexpr uint64_t SEG = 8ull << 20; /* staging segment: 8 MiB */

double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

void doc_path(char* buf, size_t n, const char* dir, uint64_t i) {
    snprintf(buf, n, "%s/doc%llu", dir, (unsigned long long)i);
}

int pick_threads(int nthreads) {
    if (nthreads > 0) return nthreads > 64 ? 64 : nthreads;
    const char* e = getenv("OMP_NUM_THREADS");
    int t = e ? atoi(e) : 0;
    if (t <= 0) t = (int)std::thread::hardware_concurrency();
    if (t <= 0) t = 4;
    return t > 16 ? 16 : t;
}

/* pread until n bytes or EOF/error; returns bytes read */
uint64_t pread_all(int fd, uint8_t* dst, uint64_t n, uint64_t off) {
    uint64_t got = 0;
    while (got < n) {
        const ssize_t r = pread(fd, dst + got, (size_t)(n - got), (off_t)(off + got));
        if (r <= 0) break;
        got += (uint64_t)r;
    }
    return got;
}

struct Slot {
    uint8_t* buf = nullptr;
    hipEvent_t ev = nullptr;
    int64_t issued = -1;   /* last segment whose copy was issued from this slot */
};

}  // namespace

extern "C" int tfidf_ingest_dir_device(tfidf_ctx* ctx, const char* dir, int nthreads, tfidf_corpus* out,
                                       uint32_t* bad_doc, tfidf_ingest_info* info) {
    if (!ctx || !dir || !out) return TFIDF_E_INVAL;
    const double t0 = now_ms();
    memset(out, 0, sizeof(*out));
    if (info) memset(info, 0, sizeof(*info));
    /* N (TFIDF.c:98-110): every entry except "." and ".." */
    DIR* d = opendir(dir);
    if (!d) return TFIDF_E_NOINPUT;
    uint64_t n = 0;
    for (struct dirent* e; (e = readdir(d)) != nullptr;)
        if (strcmp(e->d_name, ".") && strcmp(e->d_name, "..")) ++n;
    closedir(d);
    if (n > 0xFFFFFFFFull) return TFIDF_E_CAPACITY;
    const uint32_t N = (uint32_t)n;
    const int T = pick_threads(nthreads);
    const size_t plen = strlen(dir) + 32;

    /* scan: sizes of doc1..docN (TFIDF.c:130-138) */
    std::vector<uint64_t> off((size_t)N + 1, 0);
    std::atomic<uint64_t> next{0};
    std::atomic<uint64_t> first_bad{~0ull};
    {
        auto scan = [&]() {
            std::vector<char> path(plen);
            for (;;) {
                const uint64_t b = next.fetch_add(256);
                if (b >= N) break;
                const uint64_t e = b + 256 < N ? b + 256 : N;
                for (uint64_t i = b; i < e; ++i) {
                    doc_path(path.data(), plen, dir, i + 1);
                    const int fd = open(path.data(), O_RDONLY);
                    struct stat st;
                    if (fd < 0 || fstat(fd, &st) != 0) {
                        if (fd >= 0) close(fd);
                        uint64_t cur = first_bad.load();
                        while (i + 1 < cur && !first_bad.compare_exchange_weak(cur, i + 1)) {}
                        continue;
                    }
                    close(fd);
                    off[i + 1] = S_ISREG(st.st_mode) && st.st_size > 0 ? (uint64_t)st.st_size : 0;
                }
            }
        };
        std::vector<std::thread> th;
        const int ts = N < 4096 ? 1 : T;
        for (int k = 1; k < ts; ++k) th.emplace_back(scan);
        scan();
        for (auto& x : th) x.join();
    }
    if (first_bad.load() != ~0ull) {
        if (bad_doc) *bad_doc = (uint32_t)first_bad.load();
        out->ndocs = N;
        return TFIDF_E_NODOC;
    }
    for (uint32_t i = 0; i < N; ++i) off[i + 1] += off[i];
    const uint64_t total = off[N];
    const double t_scan = now_ms();

    uint8_t* dbytes = nullptr;
    uint64_t* doff = nullptr;
    int rc = tfidf_ctx_ingest_buffers(ctx, total, N, &dbytes, &doff);
    if (rc) return rc;

    /* read: segments through a ring of pinned slots, H2D on one copy stream */
    const uint64_t nseg = (total + SEG - 1) / SEG;
    const int W = (int)(nseg < (uint64_t)T ? (nseg ? nseg : 1) : (uint64_t)T);
    const int K = (int)(nseg < (uint64_t)(2 * W) ? (nseg ? nseg : 1) : (uint64_t)(2 * W));
    hipStream_t cs = nullptr;
    if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return TFIDF_E_HIP;
    std::vector<Slot> slots((size_t)K);
    bool ok = true;
    for (auto& s : slots) {
        if (nseg == 0) break;
        if (hipHostMalloc((void**)&s.buf, SEG, hipHostMallocDefault) != hipSuccess) { s.buf = nullptr; ok = false; }
        if (hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) { s.ev = nullptr; ok = false; }
    }
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<uint64_t> seg_next{0};
    std::atomic<int> err{ok ? TFIDF_OK : TFIDF_E_NOMEM};
    std::atomic<uint64_t> err_doc{~0ull};
    auto worker = [&]() {
        std::vector<char> path(plen);
        for (;;) {
            const uint64_t j = seg_next.fetch_add(1);
            if (j >= nseg) break;
            Slot& s = slots[(size_t)(j % (uint64_t)K)];
            {   /* the slot's previous segment (j-K) must have been issued ... */
                std::unique_lock<std::mutex> lk(mu);
                const int64_t prev = j >= (uint64_t)K ? (int64_t)j - K : -1;   /* -1: never used */
                cv.wait(lk, [&] { return s.issued == prev; });
            }
            /* ... and its copy finished before the buffer is overwritten */
            if (s.issued >= 0 && hipEventSynchronize(s.ev) != hipSuccess) err = TFIDF_E_HIP;
            const uint64_t a = j * SEG, b = a + SEG < total ? a + SEG : total;
            if (err.load() == TFIDF_OK) {
                /* documents overlapping [a, b): the first is the last i with off[i] <= a */
                uint64_t i = (uint64_t)(std::upper_bound(off.begin(), off.end(), a) - off.begin()) - 1;
                for (; i < N && off[i] < b; ++i) {
                    if (off[i + 1] <= a) continue;   /* empty document */
                    const uint64_t lo = off[i] > a ? off[i] : a, hi = off[i + 1] < b ? off[i + 1] : b;
                    doc_path(path.data(), plen, dir, i + 1);
                    const int fd = open(path.data(), O_RDONLY);
                    const uint64_t got = fd >= 0 ? pread_all(fd, s.buf + (lo - a), hi - lo, lo - off[i]) : 0;
                    if (fd >= 0) close(fd);
                    if (got != hi - lo) {   /* vanished or shrank since the scan */
                        uint64_t cur = err_doc.load();
                        while (i + 1 < cur && !err_doc.compare_exchange_weak(cur, i + 1)) {}
                        err = TFIDF_E_NODOC;
                        break;
                    }
                }
            }
            if (err.load() == TFIDF_OK) {
                if (hipMemcpyAsync(dbytes + a, s.buf, b - a, hipMemcpyHostToDevice, cs) != hipSuccess ||
                    hipEventRecord(s.ev, cs) != hipSuccess)
                    err = TFIDF_E_HIP;
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                s.issued = (int64_t)j;   /* issued (or skipped after an error): unblocks j+K */
            }
            cv.notify_all();
        }
    };
    if (nseg && err.load() == TFIDF_OK) {
        std::vector<std::thread> th;
        for (int k = 1; k < W; ++k) th.emplace_back(worker);
        worker();
        for (auto& x : th) x.join();
    }
    if (hipMemcpyAsync(doff, off.data(), ((size_t)N + 1) * 8, hipMemcpyHostToDevice, cs) != hipSuccess) err = TFIDF_E_HIP;
    if (hipStreamSynchronize(cs) != hipSuccess) err = TFIDF_E_HIP;
    for (auto& s : slots) {
        if (s.buf) (void)hipHostFree(s.buf);
        if (s.ev) (void)hipEventDestroy(s.ev);
    }
    (void)hipStreamDestroy(cs);
    const int e = err.load();
    if (e != TFIDF_OK) {
        if (e == TFIDF_E_NODOC && bad_doc) *bad_doc = (uint32_t)err_doc.load();
        out->ndocs = N;
        return e;
    }
    out->bytes = dbytes;
    out->nbytes = total;
    out->doc_off = doff;
    out->doc_ids = nullptr;
    out->ndocs = N;
    out->flags = TFIDF_CORPUS_DEVICE;
    out->ndocs_total = N;
    if (info) {
        const double t1 = now_ms();
        info->nbytes = total;
        info->ndocs = N;
        info->threads = (uint32_t)W;
        info->segments = nseg;
        info->ms_scan = t_scan - t0;
        info->ms_read = t1 - t_scan;
        info->ms_total = t1 - t0;
    }
    return TFIDF_OK;
}
