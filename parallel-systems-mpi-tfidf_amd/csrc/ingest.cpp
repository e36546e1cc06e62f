/*
 * ingest.cpp — SURVEY §8f row 2: the reference's input contract read straight into HBM,
 * and the byte-balanced shard plan of an input directory (§8e).
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
 * Sharding (tfidf_plan_dir): the reference deals documents to ranks round-robin by id
 * (TFIDF.c:130), so one rank can hold several of the longest documents.  The plan orders
 * the documents by "docN@" (the output's strcmp order, so shard outputs concatenate) and
 * cuts that sequence where the byte prefix sum crosses r * total / nshards: every shard
 * holds at most total / nshards + the largest document.
 *
 * The result of an ingest is a device corpus (TFIDF_CORPUS_DEVICE) whose buffers the
 * context owns, valid until the next ingest / host-corpus run / tfidf_close.  Host code
 * only: no kernels, no CPU compute on the path.
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

/* engine.cpp: the context's host-input device buffers (grown as needed); dids only when
 * requested (non-NULL) */
int tfidf_ctx_ingest_buffers(tfidf_ctx* ctx, uint64_t nbytes, uint32_t ndocs, uint8_t** dbytes, uint64_t** doff,
                             uint32_t** dids);

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

/* N (TFIDF.c:98-110): every entry except "." and ".." */
int count_entries(const char* dir, uint32_t* n_out) {
    DIR* d = opendir(dir);
    if (!d) return TFIDF_E_NOINPUT;
    uint64_t n = 0;
    for (struct dirent* e; (e = readdir(d)) != nullptr;)
        if (strcmp(e->d_name, ".") && strcmp(e->d_name, "..")) ++n;
    closedir(d);
    if (n > 0xFFFFFFFFull) return TFIDF_E_CAPACITY;
    *n_out = (uint32_t)n;
    return TFIDF_OK;
}

/* sizes of dir/doc<ids[i]> (ids == NULL: i + 1) on T threads; TFIDF_E_NODOC with *bad =
 * the smallest document id that cannot be opened (TFIDF.c:130-138) */
int scan_sizes(const char* dir, const uint32_t* ids, uint32_t n, int T, uint64_t* size, uint32_t* bad) {
    const size_t plen = strlen(dir) + 32;
    std::atomic<uint64_t> next{0};
    std::atomic<uint64_t> first_bad{~0ull};
    auto scan = [&]() {
        std::vector<char> path(plen);
        for (;;) {
            const uint64_t b = next.fetch_add(256);
            if (b >= n) break;
            const uint64_t e = b + 256 < n ? b + 256 : n;
            for (uint64_t i = b; i < e; ++i) {
                const uint64_t id = ids ? ids[i] : i + 1;
                doc_path(path.data(), plen, dir, id);
                const int fd = open(path.data(), O_RDONLY);
                struct stat st;
                if (fd < 0 || fstat(fd, &st) != 0) {
                    if (fd >= 0) close(fd);
                    uint64_t cur = first_bad.load();
                    while (id < cur && !first_bad.compare_exchange_weak(cur, id)) {}
                    size[i] = 0;
                    continue;
                }
                close(fd);
                size[i] = S_ISREG(st.st_mode) && st.st_size > 0 ? (uint64_t)st.st_size : 0;
            }
        }
    };
    std::vector<std::thread> th;
    const int ts = n < 4096 ? 1 : T;
    for (int k = 1; k < ts; ++k) th.emplace_back(scan);
    scan();
    for (auto& x : th) x.join();
    if (first_bad.load() != ~0ull) {
        if (bad) *bad = (uint32_t)first_bad.load();
        return TFIDF_E_NODOC;
    }
    return TFIDF_OK;
}

/* Streams documents dir/doc<ids[i]> (ids == NULL: i + 1), whose byte offsets are off[0..n]
 * (off[0] = 0), into the context's device buffers; see the header comment. */
int read_to_device(tfidf_ctx* ctx, const char* dir, const uint32_t* ids, uint32_t n, const std::vector<uint64_t>& off,
                   int T, uint8_t** dbytes_out, uint64_t** doff_out, uint32_t** dids_out, uint64_t* nseg_out,
                   int* workers_out, uint32_t* bad_doc) {
    const uint64_t total = off[n];
    const size_t plen = strlen(dir) + 32;
    uint8_t* dbytes = nullptr;
    uint64_t* doff = nullptr;
    uint32_t* dids = nullptr;
    int rc = tfidf_ctx_ingest_buffers(ctx, total, n, &dbytes, &doff, ids ? &dids : nullptr);
    if (rc) return rc;

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
                uint64_t i = (uint64_t)(std::upper_bound(off.begin(), off.begin() + n + 1, a) - off.begin()) - 1;
                for (; i < n && off[i] < b; ++i) {
                    if (off[i + 1] <= a) continue;   /* empty document */
                    const uint64_t lo = off[i] > a ? off[i] : a, hi = off[i + 1] < b ? off[i + 1] : b;
                    const uint64_t id = ids ? ids[i] : i + 1;
                    doc_path(path.data(), plen, dir, id);
                    const int fd = open(path.data(), O_RDONLY);
                    const uint64_t got = fd >= 0 ? pread_all(fd, s.buf + (lo - a), hi - lo, lo - off[i]) : 0;
                    if (fd >= 0) close(fd);
                    if (got != hi - lo) {   /* vanished or shrank since the scan */
                        uint64_t cur = err_doc.load();
                        while (id < cur && !err_doc.compare_exchange_weak(cur, id)) {}
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
    if (hipMemcpyAsync(doff, off.data(), ((size_t)n + 1) * 8, hipMemcpyHostToDevice, cs) != hipSuccess) err = TFIDF_E_HIP;
    if (ids && n && hipMemcpyAsync(dids, ids, (size_t)n * 4, hipMemcpyHostToDevice, cs) != hipSuccess) err = TFIDF_E_HIP;
    if (hipStreamSynchronize(cs) != hipSuccess) err = TFIDF_E_HIP;
    for (auto& s : slots) {
        if (s.buf) (void)hipHostFree(s.buf);
        if (s.ev) (void)hipEventDestroy(s.ev);
    }
    (void)hipStreamDestroy(cs);
    const int e = err.load();
    if (e == TFIDF_E_NODOC && bad_doc) *bad_doc = (uint32_t)err_doc.load();
    if (e) return e;
    *dbytes_out = dbytes;
    *doff_out = doff;
    *dids_out = dids;
    *nseg_out = nseg;
    *workers_out = W;
    return TFIDF_OK;
}

/* post-order of the decimal trie: "doc" + x + "@" sorts after every extension of x (all
 * digits are below '@', TFIDF.c:49,273), so children come before their parent */
void name_order_visit(uint64_t x, uint64_t N, std::vector<uint32_t>& out) {
    for (uint64_t d = 0; d < 10; ++d) {
        const uint64_t c = x * 10 + d;
        if (c > N) break;
        name_order_visit(c, N, out);
    }
    out.push_back((uint32_t)x);
}

}  // namespace

extern "C" int tfidf_ingest_dir_device(tfidf_ctx* ctx, const char* dir, int nthreads, tfidf_corpus* out,
                                       uint32_t* bad_doc, tfidf_ingest_info* info) {
    if (!ctx || !dir || !out) return TFIDF_E_INVAL;
    const double t0 = now_ms();
    memset(out, 0, sizeof(*out));
    if (info) memset(info, 0, sizeof(*info));
    uint32_t N = 0;
    int rc = count_entries(dir, &N);
    if (rc) return rc;
    const int T = pick_threads(nthreads);
    /* scan: sizes of doc1..docN (TFIDF.c:130-138) */
    std::vector<uint64_t> off((size_t)N + 1, 0);
    rc = scan_sizes(dir, nullptr, N, T, off.data() + 1, bad_doc);
    if (rc) { out->ndocs = N; return rc; }
    for (uint32_t i = 0; i < N; ++i) off[i + 1] += off[i];
    const double t_scan = now_ms();
    uint8_t* dbytes = nullptr;
    uint64_t* doff = nullptr;
    uint32_t* dids = nullptr;
    uint64_t nseg = 0;
    int W = 0;
    rc = read_to_device(ctx, dir, nullptr, N, off, T, &dbytes, &doff, &dids, &nseg, &W, bad_doc);
    if (rc) { out->ndocs = N; return rc; }
    out->bytes = dbytes;
    out->nbytes = off[N];
    out->doc_off = doff;
    out->doc_ids = nullptr;
    out->ndocs = N;
    out->flags = TFIDF_CORPUS_DEVICE;
    out->ndocs_total = N;
    if (info) {
        const double t1 = now_ms();
        info->nbytes = off[N];
        info->ndocs = N;
        info->threads = (uint32_t)W;
        info->segments = nseg;
        info->ms_scan = t_scan - t0;
        info->ms_read = t1 - t_scan;
        info->ms_total = t1 - t0;
    }
    return TFIDF_OK;
}

extern "C" int tfidf_shard_split(const uint64_t* bytes, uint32_t n, uint32_t nshards, uint32_t* first) {
    if (!first || nshards == 0 || (n && !bytes)) return TFIDF_E_INVAL;
    std::vector<uint64_t> pre((size_t)n + 1, 0);
    for (uint32_t i = 0; i < n; ++i) pre[i + 1] = pre[i] + bytes[i];
    const uint64_t total = pre[n];
    first[0] = 0;
    for (uint32_t r = 1; r < nshards; ++r) {
        /* the cut nearest to r * total / nshards (128-bit product: no overflow) */
        const uint64_t target = (uint64_t)(((unsigned __int128)total * r) / nshards);
        uint32_t i = (uint32_t)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
        if (i > n) i = n;
        if (i > 0 && target - pre[i - 1] < pre[i] - target) --i;
        first[r] = i < first[r - 1] ? first[r - 1] : i;
    }
    first[nshards] = n;
    return TFIDF_OK;
}

extern "C" int tfidf_doc_name_order(uint32_t n, uint32_t* ids) {
    if (n && !ids) return TFIDF_E_INVAL;
    std::vector<uint32_t> out;
    out.reserve(n);
    for (uint64_t d = 1; d <= 9 && d <= n; ++d) name_order_visit(d, n, out);
    memcpy(ids, out.data(), (size_t)n * 4);
    return TFIDF_OK;
}

extern "C" void tfidf_plan_free(tfidf_dir_plan* p) {
    if (!p) return;
    free(p->doc_ids);
    free(p->doc_bytes);
    free(p->shard_first);
    free(p->shard_bytes);
    memset(p, 0, sizeof(*p));
}

extern "C" int tfidf_plan_dir(const char* dir, uint32_t nshards, int nthreads, tfidf_dir_plan* p, uint32_t* bad_doc) {
    if (!dir || !p || nshards == 0) return TFIDF_E_INVAL;
    memset(p, 0, sizeof(*p));
    uint32_t N = 0;
    int rc = count_entries(dir, &N);
    if (rc) return rc;
    p->ndocs = N;
    p->nshards = nshards;
    p->doc_ids = (uint32_t*)malloc((size_t)N * 4 + 4);
    p->doc_bytes = (uint64_t*)malloc((size_t)N * 8 + 8);
    p->shard_first = (uint32_t*)malloc(((size_t)nshards + 1) * 4);
    p->shard_bytes = (uint64_t*)malloc((size_t)nshards * 8);
    if (!p->doc_ids || !p->doc_bytes || !p->shard_first || !p->shard_bytes) { tfidf_plan_free(p); return TFIDF_E_NOMEM; }
    rc = tfidf_doc_name_order(N, p->doc_ids);
    if (!rc) rc = scan_sizes(dir, p->doc_ids, N, pick_threads(nthreads), p->doc_bytes, bad_doc);
    if (!rc) rc = tfidf_shard_split(p->doc_bytes, N, nshards, p->shard_first);
    if (rc) {
        tfidf_plan_free(p);
        p->ndocs = N;   /* for the reference's error message */
        return rc;
    }
    for (uint32_t r = 0; r < nshards; ++r) {
        uint64_t b = 0;
        for (uint32_t i = p->shard_first[r]; i < p->shard_first[r + 1]; ++i) b += p->doc_bytes[i];
        p->shard_bytes[r] = b;
    }
    return TFIDF_OK;
}

extern "C" int tfidf_ingest_shard_device(tfidf_ctx* ctx, const char* dir, const tfidf_dir_plan* p, uint32_t shard,
                                         int nthreads, tfidf_corpus* out, uint32_t* bad_doc, tfidf_ingest_info* info) {
    if (!ctx || !dir || !p || !out || shard >= p->nshards) return TFIDF_E_INVAL;
    const double t0 = now_ms();
    memset(out, 0, sizeof(*out));
    if (info) memset(info, 0, sizeof(*info));
    const uint32_t a = p->shard_first[shard], n = p->shard_first[shard + 1] - a;
    std::vector<uint64_t> off((size_t)n + 1, 0);
    for (uint32_t i = 0; i < n; ++i) off[i + 1] = off[i] + p->doc_bytes[a + i];
    uint8_t* dbytes = nullptr;
    uint64_t* doff = nullptr;
    uint32_t* dids = nullptr;
    uint64_t nseg = 0;
    int W = 0;
    const int rc = read_to_device(ctx, dir, p->doc_ids + a, n, off, pick_threads(nthreads), &dbytes, &doff, &dids,
                                  &nseg, &W, bad_doc);
    if (rc) return rc;
    out->bytes = dbytes;
    out->nbytes = off[n];
    out->doc_off = doff;
    out->doc_ids = dids;
    out->ndocs = n;
    out->flags = TFIDF_CORPUS_DEVICE;
    out->ndocs_total = p->ndocs;
    if (info) {
        const double t1 = now_ms();
        info->nbytes = off[n];
        info->ndocs = n;
        info->threads = (uint32_t)W;
        info->segments = nseg;
        info->ms_read = t1 - t0;
        info->ms_total = t1 - t0;
    }
    return TFIDF_OK;
}
