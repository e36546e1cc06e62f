/*
 * engine.cpp — C-ABI implementation (include/tfidf.h): context, HBM buffers, stage
 * orchestration on one HIP stream, RCCL exchange, result fetch.
 *
 * Pipeline of tfidf_run (reference lines replaced in brackets):
 *   K0 plan chunks                                       [TFIDF.c:125-130 doc->rank split]
 *   K1 tokenize + LDS-hash count + global vocabulary     [TFIDF.c:130-196]
 *   vocabulary ranking (radix sort of strcmp keys)        [TFIDF.c:227-234 linear joins]
 *   partial-document merge (radix sort + reduce-by-key)
 *   DF histogram                                          [TFIDF.c:169-188,291-326]
 *   RCCL: identity-key all-gather + DF all-reduce         [TFIDF.c:209-222 MPI_Reduce/Bcast]
 *   idf LUT over the distinct df values, host libm log    [TFIDF.c:243]
 *   document order + per-document term sort + score       [TFIDF.c:202,244-245,253-273]
 * No stage has a CPU fallback: a missing device or HIP error is returned as an error.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tfidf.h"
#include "kernels.h"
#include "synth.h"
#include "xport.h"

extern "C" void tfidf_synth_spec(syn_spec* s, uint64_t seed, uint32_t V, uint32_t mode, const double* cdf);

namespace {

/* every device allocation of the engine goes through dev_malloc: the counters behind
 * tfidf_run_info.device_allocs / device_alloc_bytes (a steady-state run makes none) */
std::atomic<uint64_t> g_dev_allocs{0}, g_dev_alloc_bytes{0};

}  // namespace

hipError_t tfidf_dev_malloc(void** p, size_t bytes) {
    const hipError_t e = hipMalloc(p, bytes);
    if (e == hipSuccess) {
        g_dev_allocs.fetch_add(1, std::memory_order_relaxed);
        g_dev_alloc_bytes.fetch_add(bytes, std::memory_order_relaxed);
    }
    return e;
}

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return 0;
        const bool regrow = p != nullptr;
        if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
        /* 1/8 headroom (at least 4 KiB) on the first allocation, 1/2 on a regrowth: sizes
         * that vary from run to run (the record totals after K1's overflow records, the
         * partial-record sort buffers: K1's overflow mode depends on the order in which
         * workgroups claim LDS entries) must not reallocate in steady state — hipFree
         * synchronises the device and a 1 GB hipMalloc inside a stage left the GPU idle for
         * ~0.7 ms (the bench counts allocations in its timed steps).  Near the HBM capacity
         * the headroom is dropped rather than failing a size that fits exactly. */
        const size_t head = regrow ? bytes / 2 : bytes / 8;
        const size_t want = bytes < 256 ? 256 : bytes + (head > 4096 ? head : 4096);
        if (tfidf_dev_malloc(&p, want) == hipSuccess) { cap = want; return 0; }
        (void)hipGetLastError();
        p = nullptr;
        if (want != bytes && tfidf_dev_malloc(&p, bytes) == hipSuccess) { cap = bytes; return 0; }
        (void)hipGetLastError();
        p = nullptr;
        return -1;
    }
    /* grow preserving the first `keep` bytes */
    int grow_keep(size_t bytes, size_t keep, hipStream_t s) {
        if (bytes <= cap && p) return 0;
        void* q = nullptr;
        if (tfidf_dev_malloc(&q, bytes) != hipSuccess) return -1;
        if (p && keep) {
            if (hipMemcpyAsync(q, p, keep, hipMemcpyDeviceToDevice, s) != hipSuccess) return -1;
            if (hipStreamSynchronize(s) != hipSuccess) return -1;
        }
        if (p) (void)hipFree(p);
        p = q;
        cap = bytes;
        return 0;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
    template <typename T> T* as() const { return (T*)p; }
};

enum Stage { S_PREP, S_TOKCOUNT, S_VOCAB, S_MERGE, S_DF, S_EXCHANGE, S_IDF, S_ORDER, S_SCORE, S_NSTAGES };
const char* kStageNames[S_NSTAGES] = {"prep", "tokcount", "vocab", "merge", "df", "exchange", "idf", "order", "score"};

}  // namespace

struct tfidf_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    Xport* xp = nullptr;    /* peers of the DF exchange (RCCL or in-process); owned */
    int rank = 0, nranks = 1;
    int timing = 1;         /* tfidf_set_timing: 0 none, 1 every stage, 2 K1 and the whole run only */
    int k1_mode = 0;        /* 0 auto (k_tokcount_sl up to K1_SL_MAX_CAP slots, k_tokcount_vs beyond),
                               1 round-1 kernel (TFIDF_K1=vs), 2 general K1 (TFIDF_K1=general),
                               3 k_tokcount_sl (TFIDF_K1=sl) — cross-checks and A/B timing;
                               round 3's k_tokcount_st was retired in round 5, round 6's two-pass form of
                               k_tokcount_sl (measured slower: DESIGN §8) in round 6 (git history) */
    bool stamps_on = false; /* env TFIDF_STAMPS=1 with the diagnostic library build */
    int xfail_rank = -1;    /* env TFIDF_TEST_XFAIL_RANK (tests): this rank fails inside the exchange of
                               its first run, right after the key all-gather (the abort path of
                               exchange_df) */
    int xnomem_rank = -1;   /* env TFIDF_TEST_XNOMEM_RANK (tests): this rank's receive-side allocation
                               of its first exchange fails (the agreed path: no abort) */
    DevBuf stamps;
    bool k1_vs = false;     /* last run used the slot-keyed kernel (default) */
    bool k1_sl = false;     /* ... or tokcount_sl (else tokcount_vs) */
    uint64_t sl_maxcap = K1_SL_MAX_CAP;   /* env TFIDF_SL_MAXCAP: tokcount_sl up to this many vocabulary slots */
    K1Out* k1out_host = nullptr;   /* pinned: tokcount_sl's output block, copied to k1out_dev per run */
    DevBuf k1out_dev;
    bool k1out_valid = false;      /* k1out_dev holds *k1out_host (the copy is skipped when a run's block is the same) */
    hipEvent_t ev[S_NSTAGES + 1];
    Arena arena;
    DevBuf arena_buf;
    /* side stream: the document-order sort (needs only the document ids) runs beside the
     * vocabulary / merge / DF stages, after K1 (K1's persistent grid wants every CU) */
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_order = nullptr;
    hipEvent_t ev_spin = nullptr;   /* the run's host waits (spin_sync) */
    uint64_t wait_token = 0;        /* the last completion token of a status-words kernel (words_wait) */
    hipStream_t stream3 = nullptr;  /* the idf table's upload, beside the merge / DF stages */
    hipEvent_t ev_idf_up = nullptr;
    bool idf_early = false;         /* this run's table is on its way up stream3 (run_post waits on ev_idf_up) */
    /* split DF (runs with partial records): the main records' histogram runs on stream2
     * beside the merge stage, the merged records' is added on the main stream after it */
    bool df_split = true;           /* env TFIDF_DF_SPLIT=0: one DF pass after the merge */
    hipEvent_t ev_vrank = nullptr, ev_dfmain = nullptr;
    DevBuf df_scratch;
    size_t df_scratch_min = 0;      /* grown when the split DF pass reported a shortfall (retried) */
    Arena arena2;
    DevBuf arena2_buf;
    /* host-input staging */
    DevBuf in_bytes, in_off, in_ids;
    /* synthetic corpus */
    DevBuf syn_bytes, syn_off, syn_ids, syn_ntok, syn_blkfirst, syn_blkbytes, syn_cdf;
    /* stage buffers */
    DevBuf chunk_start, chunk_doc;
    DevBuf vkeys, vrep;
    /* vocabulary table: K1 is measurably faster at low load (fewer displaced keys behind
     * the two slots it loads per token): 1M slots (16 MB) to start, x4 past 12 % load */
    uint64_t vcap = 1ull << 20;
#define VOCAB_LOW_LOAD_CAP (1ull << 24)
#define IDF_FULL_MAX (1ull << 18)   /* documents up to which the idf table covers every df (beyond:
                                       the distinct df values of the run, one host round trip) */
    uint32_t vload_pct = 12;
    uint32_t vload_big_pct = 45;   /* load limit of tables of VOCAB_LOW_LOAD_CAP slots and more */
    DevBuf rec_slot, rec_cnt;
    uint64_t rec_cap = 0;
    DevBuf part_doc, part_slot, part_cnt;
    uint64_t part_cap = 0;
    DevBuf doc_recoff, doc_npairs, doc_size, doc_flags;
    DevBuf counters;
    /* pinned host words for the per-run device-to-host reads (corpus bounds, K1 counters,
     * final status): asynchronous copies on the stream and one synchronisation each, instead
     * of pageable or synchronous copies (two round trips per run saved) */
    uint64_t* hpin = nullptr;
    uint64_t* hpin_dev = nullptr;   /* hpin as the device addresses it (status words written by kernels) */
    DevBuf dense, vslot, skey0, skey1, seq0, seq1, rank_of_slot, slot_of_rank, rank16;
    DevBuf pkey0, pkey1, pseq0, pseq1, phead;
    DevBuf big_list, big_idx, dense_cnt, kcnt, tile_cnt;   /* dense merge of long documents */
    DevBuf df_local, df_global, present, idf_vals;
    uint64_t idf_full_n = 0;   /* idf_vals holds log(N/df) for df = 0..N of this N (0: not) */
    /* the per-run idf table (N <= IDF_FULL_MAX): host threads fill the pinned idf_pin with
     * log(N/df) for df = 0..N while the device runs the stages before the score; run_post
     * joins them and uploads it (every run: round 4's per-N cache was retired in round 6) */
    double* idf_pin = nullptr;
    size_t idf_pin_n = 0;
    bool idf_pin_busy = false;            /* an upload from idf_pin is enqueued and not known complete (the
                                             run's final wait clears it; no event record: each costs
                                             the stream ~5 us, scripts/micro/host_api_cost.hip) */
    struct IdfPool {                      /* persistent workers: no thread start per run */
        std::mutex mu;
        std::condition_variable go, done;
        std::vector<std::thread> th;
        uint64_t gen = 0;
        bool stop = false, busy = false;
        unsigned active = 0, left = 0;
        double* lut = nullptr;
        uint64_t Nt = 0;
        const uint32_t* vals = nullptr;   /* null: lut[d] for every df d = 1..Nt; else lut[k] for df vals[k], k < n */
        uint64_t n = 0;
        std::chrono::steady_clock::time_point t0;
        int64_t end_ns = 0;
    } idf_pool;
    uint64_t idf_logs = 0;                /* log() calls of the last run */
    tfidf_run_totals totals{};            /* sums over the runs since the last tfidf_run_totals_get reset */
    double ms_idf_host = 0, ms_idf_wait = 0;
    DevBuf dkey0, dkey1, dseq0, dseq1, npairs_ord, out_off, doc_meta;
    DevBuf out_term, out_cnt, out_score, idf_rank, large_list, split_tasks, cls_off;
    /* DF exchange (hash owners): this rank's keys by term rank, the send side grouped by
     * owner (key, local df, term rank), the owner side (received keys and df, their table
     * slots, the replies, the aggregation table), the returned global df, the count matrix */
    DevBuf x_mine, x_srec, x_sidx, x_back, x_cnt;
    DevBuf x_rrec, x_rslot, x_reply, x_tkey, x_tdf;
    /* dense exchange (small vocabularies): gathered keys, shared positions, the DF vector */
    DevBuf x_gkeys, x_pos, x_dense;
    /* cross-rank check of long terms (exchange_long_check): this rank's list, its send block
     * (entries + bytes), the gathered blocks, the check's key table */
    DevBuf x_lloc, x_lsend, x_lgath, x_ltab;
    int xchg_mode = 0;      /* env TFIDF_XCHG: 0 auto (dense up to DENSE_XCHG_MAXV terms per rank), 1 owner, 2 dense,
                               3 dense with table numbering */
    bool last_dense = false;   /* the last exchange used the dense form */
    bool local_long = false;   /* this rank's vocabulary holds terms of >= 16 bytes (K1 status) */
    bool xagg_table = false;   /* env TFIDF_XAGG=table: the owner aggregates in an HBM table (A/B) */
    uint32_t xb_stage_max = ~0u;   /* env TFIDF_XB_STAGE_MAX (tests): the owner's largest bucket staged in LDS */
    /* sizes the local part of a run hands to the exchange and the stages after it */
    uint32_t run_N = 0, run_V = 0;
    uint64_t run_cap = 0, run_R_total = 0;
    const uint32_t* run_merged = nullptr;
    /* output text (emit.hip) */
    DevBuf t_key, t_len, doc_tbytes, doc_toff, text;
#define WR_NBUF 8
#define WR_BUF (16ull << 20)
#define WR_GROUPS 8
    uint8_t* wr_buf[WR_NBUF] = {};   /* pinned output staging ring */
    hipEvent_t wr_ev[WR_NBUF] = {};
    hipEvent_t wr_fmt[WR_GROUPS] = {};
#define WR_WRITERS 8   /* page-cache writes run ~3 GB/s per thread (profiles/r04_cli_c2.json) */
    tfidf_output_info out_info{};
    uint64_t text_bytes = 0;
    bool text_valid = false;
    uint32_t* sorted_dense = nullptr; /* points into seq0/seq1 */
    uint4* sorted_skey = nullptr;
    const uint32_t* order = nullptr;
    /* last run */
    bool have_result = false;
    bool have_info = false;   /* run counters/timings valid */
    uint64_t run_nbytes = 0;  /* corpus bytes of the last run (its bounds, read once by the run) */
    tfidf_corpus corpus{};
    const uint8_t* dev_bytes = nullptr;
    const uint32_t* dev_ids = nullptr;
    uint64_t npairs = 0, ntokens = 0, nchunks = 0, nrec_part = 0, ndocs_total = 0;
    uint32_t ndocs = 0, V = 0, Vg = 0;
    double ms_stage[S_NSTAGES] = {0};
    double ms_total = 0;
    hipError_t last_err = hipSuccess;
};
static void idf_pool_stop(tfidf_ctx* ctx);   /* the per-run idf table's workers (idf_start) */
static bool idf_done(tfidf_ctx* ctx);
static void idf_join(tfidf_ctx* ctx);
/* open contexts in this process: the idf workers of all of them share IDF_POOL threads' worth
 * of work (a group of K shards in one process would otherwise start 8 K of them) */
static std::atomic<int> g_live_ctx{0};

#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            ctx->last_err = e_;                                                            \
            fprintf(stderr, "tfidf: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return TFIDF_E_HIP;                                                            \
        }                                                                                  \
    } while (0)
/* a wait for the run's stream once collectives may be in it: through the transport, so
 * that a failed peer cannot leave this rank waiting (xport.h, comm_rank.h) */
#define XSYNC(s_)                                                                          \
    do {                                                                                   \
        if (ctx->xp) {                                                                     \
            const int w_ = ctx->xp->wait(s_);                                              \
            if (w_) return w_;                                                             \
        } else {                                                                           \
            HIPCHK(spin_sync(ctx, s_));                                                    \
        }                                                                                  \
    } while (0)
/* TFIDF_DEBUG_ALLOC=1: every (re)allocation of a stage buffer is named on stderr (which
 * buffer still grows after the warm-up runs) */
static int debug_alloc() {
    static const int on = [] { const char* e = getenv("TFIDF_DEBUG_ALLOC"); return e && e[0] == '1'; }();
    return on;
}
static int ensure_named(DevBuf& b, size_t bytes, const char* name) {
    const void* p0 = b.p;
    const int rc = b.ensure(bytes);
    if (debug_alloc() && (b.p != p0 || rc))
        fprintf(stderr, "tfidf: alloc %s %zu bytes (asked %zu)%s\n", name, b.cap, bytes, rc ? " FAILED" : "");
    return rc;
}
#define ENSURE(buf, bytes)                                   \
    do {                                                     \
        if (ensure_named((buf), (size_t)(bytes), #buf) != 0) return TFIDF_E_NOMEM; \
    } while (0)
#define LCHK(x)                                              \
    do {                                                     \
        int l_ = (x);                                        \
        if (l_ == -2) return 1; /* arena too small: retry */ \
        if (l_ < 0) { HIPCHK(hipGetLastError()); return TFIDF_E_HIP; } \
    } while (0)

static int arena_reset(tfidf_ctx* ctx, size_t want) {
    if (want > ctx->arena_buf.cap) {
        if (ctx->arena_buf.ensure(want) != 0) return TFIDF_E_NOMEM;
    }
    ctx->arena.base = (uint8_t*)ctx->arena_buf.p;
    ctx->arena.cap = ctx->arena_buf.cap;
    ctx->arena.used = 0;
    return 0;
}

/* each event record costs the stream ~5 us (scripts/micro/host_api_cost.hip): level 2 records
 * only the four K1 and whole-run bounds */
static void mark(tfidf_ctx* ctx, int stage) {
    if (ctx->timing == 1 ||
        (ctx->timing == 2 && (stage == S_PREP || stage == S_TOKCOUNT || stage == S_VOCAB || stage == S_NSTAGES)))
        (void)hipEventRecord(ctx->ev[stage], ctx->stream);
}

/* Status words into hpin (launch_words_to_host at hpin_dev + at) and the wait for them: in
 * a single-context process the kernel also writes a completion token after the words and
 * the host polls that word in pinned memory — no event record on the stream (~5 us each) and
 * no blocking wake-up; bounded (2 s, then the stream is synchronised, which also reports a
 * failed kernel).  Several contexts in the process: the stream is synchronised. */
static hipError_t words_wait(tfidf_ctx* ctx, WordList& wl, uint32_t at, hipStream_t s) {
    const bool poll = g_live_ctx.load() <= 1;
    wl.token = poll ? (0x7A5E000000000000ull | ++ctx->wait_token) : 0ull;
    if (launch_words_to_host(wl, ctx->hpin_dev + at, s)) return hipErrorLaunchFailure;
    if (!poll) return hipStreamSynchronize(s);
    volatile uint64_t* tok = ctx->hpin + at + wl.n;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t it = 0; *tok != wl.token; ++it) {
        if ((it & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
            const hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
            return *tok == wl.token ? hipSuccess : hipErrorUnknown;
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return hipSuccess;
}

/* the run's global df by term rank: the exchange's result, or with one rank the local df */
static uint32_t* df_of_run(tfidf_ctx* ctx) {
    return ctx->xp ? ctx->df_global.as<uint32_t>() : ctx->df_local.as<uint32_t>();
}

/* The run's waits for its own stream (K1's counters, the final status): the host polls an
 * event instead of blocking in hipStreamSynchronize, whose wake-up after a millisecond-long
 * kernel left the device idle for tens of microseconds before the next launches. */
static hipError_t spin_sync(tfidf_ctx* ctx, hipStream_t s) {
    if (g_live_ctx.load() > 1) return hipStreamSynchronize(s);   /* several ranks' threads in this process */
    hipError_t e = hipEventRecord(ctx->ev_spin, s);
    if (e != hipSuccess) return e;
    while ((e = hipEventQuery(ctx->ev_spin)) == hipErrorNotReady) {
    }
    return e;
}

extern "C" {

int tfidf_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && n > 0 ? n : 0;
}

int tfidf_open(int device, tfidf_ctx** out) {
    if (!out) return TFIDF_E_INVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return TFIDF_E_NODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return TFIDF_E_NODEV;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        fprintf(stderr, "tfidf: device %d is %s, need gfx950\n", device, prop.gcnArchName);
        return TFIDF_E_NODEV;
    }
    if (hipSetDevice(device) != hipSuccess) return TFIDF_E_NODEV;
    tfidf_ctx* ctx = new tfidf_ctx();
    ctx->device = device;
    const char* km = getenv("TFIDF_K1");
    if (km && !strcmp(km, "general")) ctx->k1_mode = 2;
    if (km && !strcmp(km, "vs")) ctx->k1_mode = 1;
    if (km && !strcmp(km, "sl")) ctx->k1_mode = 3;
    {
        const char* sm = getenv("TFIDF_SL_MAXCAP");
        const unsigned long long v = sm ? strtoull(sm, nullptr, 0) : 0ull;
        if (v >= 1024 && v <= K1_SL_MAX_CAP) ctx->sl_maxcap = v;
    }
    const char* ks = getenv("TFIDF_STAMPS");
    ctx->stamps_on = ks && ks[0] == '1';
    const char* kx = getenv("TFIDF_TEST_XFAIL_RANK");
    ctx->xfail_rank = kx ? atoi(kx) : -1;
    const char* kxm = getenv("TFIDF_XCHG");
    if (kxm && !strcmp(kxm, "owner")) ctx->xchg_mode = 1;
    if (kxm && !strcmp(kxm, "dense")) ctx->xchg_mode = 2;
    if (kxm && !strcmp(kxm, "dense_table")) ctx->xchg_mode = 3;
    const char* kxa = getenv("TFIDF_XAGG");
    ctx->xagg_table = kxa && !strcmp(kxa, "table");
    const char* kxb = getenv("TFIDF_XB_STAGE_MAX");
    ctx->xb_stage_max = kxb ? (uint32_t)atoi(kxb) : ~0u;
    const char* kds = getenv("TFIDF_DF_SPLIT");
    ctx->df_split = !(kds && !strcmp(kds, "0"));
    const char* kn = getenv("TFIDF_TEST_XNOMEM_RANK");
    ctx->xnomem_rank = kn ? atoi(kn) : -1;
    /* diagnostics: initial vocabulary capacity (power of two) and the loads it may reach
     * before the run is repeated with a larger table (TFIDF_VLOAD percent below 16M slots,
     * default 12; TFIDF_VLOAD_BIG from 16M slots on, default 45) */
    const char* kv = getenv("TFIDF_VCAP");
    if (kv) {
        uint64_t c = strtoull(kv, nullptr, 0);
        if (c >= 1024 && (c & (c - 1)) == 0) ctx->vcap = c;
    }
    const char* kb = getenv("TFIDF_VLOAD_BIG");
    if (kb) {
        uint32_t l = (uint32_t)strtoul(kb, nullptr, 0);
        if (l >= 10 && l <= 90) ctx->vload_big_pct = l;
    }
    const char* kl = getenv("TFIDF_VLOAD");
    if (kl) {
        uint32_t l = (uint32_t)strtoul(kl, nullptr, 0);
        if (l >= 10 && l <= 90) ctx->vload_pct = l;
    }
    HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&ctx->stream3, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ctx->ev_order, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ctx->ev_spin, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ctx->ev_idf_up, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ctx->ev_vrank, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ctx->ev_dfmain, hipEventDisableTiming));
    for (int i = 0; i <= S_NSTAGES; ++i) HIPCHK(hipEventCreate(&ctx->ev[i]));
    if (arena_reset(ctx, 64ull << 20) != 0) { delete ctx; return TFIDF_E_NOMEM; }
    if (ctx->counters.ensure(256) != 0) { delete ctx; return TFIDF_E_NOMEM; }
    /* coherent: the status words a kernel writes (and its completion token) reach the host
     * without a cache flush at the kernel's end */
    if (hipHostMalloc((void**)&ctx->hpin, 256, hipHostMallocCoherent) != hipSuccess) { delete ctx; return TFIDF_E_NOMEM; }
    if (hipHostGetDevicePointer((void**)&ctx->hpin_dev, ctx->hpin, 0) != hipSuccess || !ctx->hpin_dev) {
        delete ctx;
        return TFIDF_E_NOMEM;
    }
    if (hipHostMalloc((void**)&ctx->k1out_host, sizeof(K1Out), hipHostMallocDefault) != hipSuccess ||
        ctx->k1out_dev.ensure(sizeof(K1Out)) != 0) { delete ctx; return TFIDF_E_NOMEM; }
    g_live_ctx.fetch_add(1);
    *out = ctx;
    return TFIDF_OK;
}

void tfidf_close(tfidf_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    delete ctx->xp;
    if (ctx->stream2) { (void)hipStreamSynchronize(ctx->stream2); (void)hipStreamDestroy(ctx->stream2); }
    if (ctx->stream3) { (void)hipStreamSynchronize(ctx->stream3); (void)hipStreamDestroy(ctx->stream3); }
    if (ctx->ev_idf_up) (void)hipEventDestroy(ctx->ev_idf_up);
    if (ctx->ev_vrank) (void)hipEventDestroy(ctx->ev_vrank);
    if (ctx->ev_dfmain) (void)hipEventDestroy(ctx->ev_dfmain);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_spin) (void)hipEventDestroy(ctx->ev_spin);
    if (ctx->ev_order) (void)hipEventDestroy(ctx->ev_order);
    idf_pool_stop(ctx);
    g_live_ctx.fetch_sub(1);
    if (ctx->idf_pin) (void)hipHostFree(ctx->idf_pin);
    for (int i = 0; i < WR_NBUF; ++i) {
        if (ctx->wr_buf[i]) (void)hipHostFree(ctx->wr_buf[i]);
        if (ctx->wr_ev[i]) (void)hipEventDestroy(ctx->wr_ev[i]);
    }
    for (int i = 0; i < WR_GROUPS; ++i)
        if (ctx->wr_fmt[i]) (void)hipEventDestroy(ctx->wr_fmt[i]);
    ctx->arena2_buf.release();
    ctx->df_scratch.release();
    DevBuf* bufs[] = {&ctx->arena_buf, &ctx->in_bytes, &ctx->in_off, &ctx->in_ids, &ctx->syn_bytes, &ctx->syn_off,
                      &ctx->syn_ids, &ctx->syn_ntok, &ctx->syn_blkfirst, &ctx->syn_blkbytes, &ctx->syn_cdf,
                      &ctx->chunk_start, &ctx->chunk_doc, &ctx->vkeys, &ctx->vrep, &ctx->rec_slot, &ctx->rec_cnt,
                      &ctx->part_doc, &ctx->part_slot, &ctx->part_cnt, &ctx->doc_recoff, &ctx->doc_npairs,
                      &ctx->doc_size, &ctx->doc_flags, &ctx->counters, &ctx->dense, &ctx->vslot, &ctx->skey0,
                      &ctx->skey1, &ctx->seq0, &ctx->seq1, &ctx->rank_of_slot, &ctx->slot_of_rank, &ctx->rank16, &ctx->pkey0,
                      &ctx->pkey1, &ctx->pseq0, &ctx->pseq1, &ctx->phead, &ctx->df_local, &ctx->df_global,
                      &ctx->present, &ctx->idf_vals, &ctx->dkey0, &ctx->dkey1, &ctx->dseq0, &ctx->dseq1,
                      &ctx->npairs_ord, &ctx->out_off, &ctx->doc_meta, &ctx->t_key, &ctx->t_len, &ctx->doc_tbytes,
                      &ctx->doc_toff, &ctx->text, &ctx->out_term, &ctx->out_cnt,
                      &ctx->out_score, &ctx->idf_rank, &ctx->large_list, &ctx->split_tasks, &ctx->cls_off, &ctx->x_mine, &ctx->x_srec,
                      &ctx->x_sidx, &ctx->x_back, &ctx->x_cnt, &ctx->x_rrec, &ctx->x_rslot, &ctx->x_reply, &ctx->x_gkeys,
                      &ctx->x_pos, &ctx->x_dense, &ctx->x_lloc, &ctx->x_lsend, &ctx->x_lgath, &ctx->x_ltab,
                      &ctx->x_tkey, &ctx->x_tdf, &ctx->stamps, &ctx->big_list, &ctx->big_idx, &ctx->dense_cnt, &ctx->kcnt,
                      &ctx->tile_cnt};
    for (DevBuf* b : bufs) b->release();
    for (int i = 0; i <= S_NSTAGES; ++i) (void)hipEventDestroy(ctx->ev[i]);
    if (ctx->hpin) (void)hipHostFree(ctx->hpin);
    if (ctx->k1out_host) (void)hipHostFree(ctx->k1out_host);
    ctx->k1out_dev.release();
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int tfidf_set_timing(tfidf_ctx* ctx, int enable) {
    if (!ctx) return TFIDF_E_INVAL;
    ctx->timing = enable == 2 ? 2 : (enable != 0 ? 1 : 0);
    return TFIDF_OK;
}

const char* tfidf_stage_name(int stage) { return (stage >= 0 && stage < S_NSTAGES) ? kStageNames[stage] : "?"; }

int tfidf_comm_unique_id(uint8_t id[TFIDF_UNIQUE_ID_BYTES]) {
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return TFIDF_E_RCCL;
    memcpy(id, &u, TFIDF_UNIQUE_ID_BYTES);
    return TFIDF_OK;
}

int tfidf_comm_init(tfidf_ctx* ctx, const uint8_t id[TFIDF_UNIQUE_ID_BYTES], int rank, int nranks) {
    /* ranks <= 1024: the DF exchange's per-owner counts live in LDS (k_owner_count) */
    if (!ctx || !id || nranks < 1 || nranks > 1024 || rank < 0 || rank >= nranks) return TFIDF_E_INVAL;
    HIPCHK(hipSetDevice(ctx->device));
    tfidf_ctx_attach_xport(ctx, nullptr);
    static_assert(sizeof(ncclUniqueId) == TFIDF_UNIQUE_ID_BYTES, "unique id size");
    Xport* x = nullptr;
    const int rc = rccl_init_rank(id, rank, nranks, ctx->device, &x);
    if (rc) return rc;
    return tfidf_ctx_attach_xport(ctx, x);
}

}  // extern "C"

int tfidf_ctx_attach_xport(tfidf_ctx* ctx, Xport* xp) {
    if (!ctx) { delete xp; return TFIDF_E_INVAL; }
    delete ctx->xp;
    ctx->xp = xp;
    ctx->rank = xp ? xp->rank : 0;
    ctx->nranks = xp ? xp->nranks : 1;
    return TFIDF_OK;
}
int tfidf_ctx_device(const tfidf_ctx* ctx) { return ctx->device; }
hipStream_t tfidf_ctx_stream(const tfidf_ctx* ctx) { return ctx->stream; }

/* ------------------------------------------------------------------------------ */

/* ---- the DF exchange (replaces MPI_Reduce(CustomReduce) + MPI_Bcast, TFIDF.c:209-222,
 * 291-326).  Every rank enters it once per attempt, also when its local stages failed or
 * asked for a retry, so the ranks always agree:
 *   1. words(status, V): any error -> every rank returns an error (its own, or
 *      TFIDF_E_PEER); any retry -> every rank returns 1 and repeats the run in step.  Every
 *      rank learns every rank's V, which sizes everything after it.
 *   2. one of two forms (the same results; TFIDF_XCHG=owner|dense forces one):
 *      dense  (every rank's V <= DENSE_XCHG_MAXV: c2, c3, c5) — north_star's form: the
 *             ranks' term keys are all-gathered (padded to the largest V), every rank numbers
 *             the distinct keys identically, scatters its local df into a dense vector over
 *             those numbers, and ONE all-reduce (sum) gives every rank the global df; global
 *             V = the distinct keys.  The numbering: when no rank holds terms of >= 16 bytes
 *             (a flag in step 1's word) each gathered list is in term order and a key's
 *             number is its position in the merged lists (binary searches, no table:
 *             launch_dense_merge_ids); otherwise its smallest gathered position, from a hash
 *             table of all gathered keys (TFIDF_XCHG=dense_table forces this).  Buffers are sized
 *             before step 1 from the rank's own V (padded by a quarter), so their allocation
 *             status travels in step 1's word; only when the largest V exceeds some rank's
 *             padding do all ranks grow them and agree once more.  Then one all-gather and
 *             one all-reduce: one host synchronisation in all (step 1's).
 *      owner  (larger V: c4) — SURVEY §8e's hash-owner partitioning: every term goes to an
 *             owner rank (a hash of its key); the per-owner counts are all-gathered together
 *             with each rank's allocation status (an allocation failure is agreed there, no
 *             extra exchange), one all-to-all sends 20-byte (key, local df) records, each owner
 *             sums equal keys (LDS tables over hash buckets of the received records; an HBM
 *             hash table with TFIDF_XAGG=table) and one all-to-all returns the global df of
 *             each record plus, per sender, the owner's distinct-key count (global V = their sum).
 *             Per rank ~V entries move; the owner aggregates ~ΣV/R.
 *   Global V stays on the device and is read with the run's final status (no host round
 *   trip of its own).  From step 2 on no stage of the run returns "retry" (run_local checked
 *   the post-exchange stages' scratch before step 1); an error inside a collective sequence
 *   aborts the transport (releasing the peers), an agreed failure does not. */
static uint64_t status_word(int rc) { return rc < 0 ? 0x100ull | (uint64_t)(-rc) : (uint64_t)rc; }

static size_t scan_scratch(uint64_t n) { return (size_t)(n / 16) + 8192; }

#define DENSE_XCHG_MAXV (1u << 17)

/* words(status, v) over the ranks: 0 all fine, 1 retry (some rank asked), <0 an error (this
 * rank's own, else TFIDF_E_PEER); vs (optional) = every rank's v */
static int exchange_agree(tfidf_ctx* ctx, int local_rc, uint64_t v, std::vector<uint64_t>* vs) {
    Xport* xp = ctx->xp;
    std::vector<uint64_t> all(2 * (size_t)xp->nranks);
    const uint64_t mine[2] = {status_word(local_rc), v};
    const int rc = xp->words(mine, all.data(), ctx->stream);
    if (rc) return rc;
    uint64_t worst = 0;
    if (vs) vs->assign((size_t)xp->nranks, 0);
    for (int r = 0; r < xp->nranks; ++r) {
        worst = all[2 * r] > worst ? all[2 * r] : worst;
        if (vs) (*vs)[r] = all[2 * r + 1];
    }
    if (worst >= 0x100) return local_rc < 0 ? local_rc : TFIDF_E_PEER;
    return worst ? 1 : 0;
}

/* errors inside the collective sequence: no retry is possible any more */
#define XCHK(x)                                                             \
    do {                                                                    \
        int l_ = (x);                                                       \
        if (l_ == -2) return TFIDF_E_CAPACITY;                              \
        if (l_ < 0) { HIPCHK(hipGetLastError()); return TFIDF_E_HIP; }      \
    } while (0)

static uint64_t table_cap(uint64_t n) {   /* load <= 2/3: short probe runs */
    uint64_t t = 1024;
    while (t < n + n / 2) t *= 2;
    return t;
}

/* the hash-owner form (step 2 above); *agreed = true when the returned failure was decided
 * by all ranks together (nothing half-done in a collective: the transport stays usable) */
static int exchange_owner(tfidf_ctx* ctx, uint32_t V, const std::vector<uint64_t>& vs, bool* agreed) {
    hipStream_t s = ctx->stream;
    Xport* xp = ctx->xp;
    const int R = xp->nranks, me = xp->rank;
    unsigned long long* cnt = ctx->counters.as<unsigned long long>();
    uint64_t sumv = 0;
    for (uint64_t x : vs) sumv += x;
    /* everything sized here from the agreed V's: the receive side holds at most every
     * rank's terms; a failure travels as the status word of the count row (below) */
    int arc = 0;
    auto ens = [&](DevBuf& b, size_t bytes) { if (!arc && b.ensure(bytes) != 0) arc = TFIDF_E_NOMEM; };
    if (!ctx->sorted_skey) ens(ctx->x_mine, (size_t)V * 16 + 16);
    ens(ctx->x_srec, (size_t)V * 20 + 20);
    ens(ctx->x_sidx, (size_t)V * 4 + 4);
    ens(ctx->x_back, ((size_t)V + R) * 4 + 4);
    ens(ctx->x_rrec, sumv * 20 + 20);
    ens(ctx->x_reply, (sumv + R) * 4 + 4);
    if (ctx->xagg_table) {   /* TFIDF_XAGG=table: the HBM table and its df column */
        ens(ctx->x_tkey, table_cap(sumv) * 16);
        ens(ctx->x_tdf, table_cap(sumv) * 4);
        ens(ctx->x_rslot, sumv * 4 + 4);
    } else {                 /* the bucketed form's sort scratch */
        ens(ctx->x_tkey, owner_bucket_scratch(sumv));
    }
    if (ctx->xnomem_rank == me) {   /* tests: an agreed allocation failure (once) */
        ctx->xnomem_rank = -1;
        arc = TFIDF_E_NOMEM;
    }
    /* x_cnt (sized in run_local): [R + 1] this rank's row (counts per owner + status),
     * [R (R + 1)] all rows, [R + 1] soff, [R + 1] roff */
    uint32_t* row = ctx->x_cnt.as<uint32_t>();
    uint32_t* mat = row + (R + 1);
    uint32_t* soff = mat + (size_t)R * (R + 1);
    uint32_t* roff = soff + (R + 1);
    uint32_t* cur = roff + (R + 1);
    if (!arc) {
        /* the keys straight from the vocabulary sort (run_local): sorted by rank after the
         * tile sort (and gathered so for the long-term fix-up after the radix sort), else
         * gathered here from the radix sort's compact keys in dense order */
        OwnerKeySrc ks;
        ks.skey = ctx->sorted_skey;
        if (!ks.skey) {
            XCHK(launch_gather_u128(ctx->skey0.as<uint4>(), ctx->sorted_dense, V, ctx->x_mine.as<uint4>(), s));
            ks.skey = ctx->x_mine.as<uint4>();
        }
        ks.slot_of_rank = ctx->slot_of_rank.as<uint32_t>();
        ks.vkeys = ctx->vkeys.as<uint4>();
        XCHK(launch_owner_partition(ks, ctx->df_local.as<uint32_t>(), V, (uint32_t)R, row, cur,
                                    ctx->x_srec.as<uint32_t>(), ctx->x_sidx.as<uint32_t>(), s));
    } else {
        HIPCHK(hipMemsetAsync(row, 0, (size_t)R * 4, s));
    }
    ctx->hpin[15] = (uint64_t)(uint32_t)arc;
    HIPCHK(hipMemcpyAsync(row + R, ctx->hpin + 15, 4, hipMemcpyHostToDevice, s));
    int rc = xp->allgather(row, mat, (size_t)(R + 1) * 4, s);
    if (rc) return rc;
    std::vector<uint32_t> m((size_t)R * (R + 1));
    HIPCHK(hipMemcpyAsync(m.data(), mat, m.size() * 4, hipMemcpyDeviceToHost, s));
    XSYNC(s);
    int peer_fail = 0;
    for (int p = 0; p < R; ++p)
        if (m[(size_t)p * (R + 1) + R]) peer_fail = 1;
    if (peer_fail) { *agreed = true; return arc ? arc : TFIDF_E_PEER; }
    std::vector<uint64_t> scnt(R), rcnt(R), scnt1(R), rcnt1(R);
    uint64_t nrecv = 0, nsend = 0;
    for (int p = 0; p < R; ++p) {
        scnt[p] = m[(size_t)me * (R + 1) + p];
        rcnt[p] = m[(size_t)p * (R + 1) + me];
        scnt1[p] = scnt[p] + 1;   /* the replies carry one trailer word per owner */
        rcnt1[p] = rcnt[p] + 1;
        nrecv += rcnt[p];
        nsend += scnt[p];
    }
    if (nsend != V || nrecv > sumv) return TFIDF_E_STATE;
    if (ctx->xfail_rank == me) {   /* tests: a rank-local failure after a collective (once) */
        ctx->xfail_rank = -1;
        fprintf(stderr, "tfidf: rank %d: injected exchange failure (TFIDF_TEST_XFAIL_RANK)\n", me);
        return TFIDF_E_HIP;
    }
    XCHK(launch_owner_offsets(mat, (uint32_t)R, (uint32_t)me, soff, roff, s));
    /* (key, local df) records to the owners */
    rc = xp->alltoallv(ctx->x_srec.p, scnt.data(), ctx->x_rrec.p, rcnt.data(), 20, s);
    if (rc) return rc;
    /* the owner: df summed per distinct key, every received record answered in order */
    unsigned long long* used = cnt + 10;
    if (ctx->xagg_table) {   /* TFIDF_XAGG=table: round 3's table of 1.5x the records (A/B) */
        XCHK(launch_owner_aggregate(ctx->x_rrec.as<uint32_t>(), nrecv, roff, (uint32_t)R, ctx->x_tkey.as<uint4>(),
                                    table_cap(nrecv), ctx->x_tdf.as<uint32_t>(), ctx->x_rslot.as<uint32_t>(),
                                    ctx->x_reply.as<uint32_t>(), used, (uint32_t*)(cnt + 3), s));
    } else {   /* bucketed: x_tkey is its scratch */
        XCHK(launch_owner_aggregate_buckets(ctx->x_rrec.as<uint32_t>(), nrecv, roff, (uint32_t)R, ctx->x_tkey.p,
                                            ctx->x_tkey.cap, ctx->x_reply.as<uint32_t>(), used, (uint32_t*)(cnt + 3),
                                            ctx->xb_stage_max, s));
    }
    rc = xp->alltoallv(ctx->x_reply.p, rcnt1.data(), ctx->x_back.p, scnt1.data(), 4, s);
    if (rc) return rc;
    XCHK(launch_owner_back(ctx->x_back.as<uint32_t>(), soff, (uint32_t)R, ctx->x_sidx.as<uint32_t>(), V,
                           ctx->df_global.as<uint32_t>(), (uint32_t*)(cnt + 12), s));
    return 0;
}

/* The dense form's buffers for gathers of R blocks of `maxv` keys.  Sized before the
 * agreement from this rank's own V (padded: dense_pad) so that, when every rank's padded V
 * covers the largest V, no second agreement is needed (allocation failures travel in the
 * agreement's status word). */
static uint64_t dense_pad(uint64_t v) { return v + v / 4 + 64; }
static int dense_alloc(tfidf_ctx* ctx, uint32_t V, uint64_t maxv, uint64_t R) {
    const uint64_t n = R * maxv, sumv = R * maxv;
    if (ctx->x_mine.ensure(maxv * 16 + 16) || ctx->x_gkeys.ensure(n * 16 + 16) ||
        ctx->x_tkey.ensure(table_cap(sumv) * 16) || ctx->x_tdf.ensure(table_cap(sumv) * 4) ||
        ctx->x_pos.ensure((size_t)V * 4 + 4) || ctx->x_dense.ensure(n * 4 + 4))
        return TFIDF_E_NOMEM;
    return 0;
}

/* the dense form (step 2 above) */
static int exchange_dense(tfidf_ctx* ctx, uint32_t V, const std::vector<uint64_t>& vs, bool merge, bool* agreed) {
    hipStream_t s = ctx->stream;
    Xport* xp = ctx->xp;
    const int R = xp->nranks, me = xp->rank;
    unsigned long long* cnt = ctx->counters.as<unsigned long long>();
    uint64_t maxv = 1, sumv = 0, minpad = ~0ull;
    for (uint64_t x : vs) {
        maxv = x > maxv ? x : maxv;
        sumv += x;
        minpad = dense_pad(x) < minpad ? dense_pad(x) : minpad;
    }
    const uint64_t n = (uint64_t)R * maxv;   /* gathered positions */
    /* every rank sized its buffers for R blocks of dense_pad(its V) before the agreement
     * (exchange_df); only when some rank's padding is short of the largest V do all ranks
     * grow them and agree once more (the same decision on every rank: it depends on vs) */
    if (maxv > minpad) {
        int arc = dense_alloc(ctx, V, maxv, (uint64_t)R);
        if (ctx->xnomem_rank == me) {   /* tests: an agreed allocation failure (once) */
            ctx->xnomem_rank = -1;
            arc = TFIDF_E_NOMEM;
        }
        int rc = exchange_agree(ctx, arc, 0, nullptr);
        if (rc == 1) rc = TFIDF_E_STATE;
        if (rc) { *agreed = true; return rc; }
    }
    int rc = 0;
    if (ctx->xfail_rank == me) {   /* tests: a rank-local failure after a collective (once) */
        ctx->xfail_rank = -1;
        fprintf(stderr, "tfidf: rank %d: injected exchange failure (TFIDF_TEST_XFAIL_RANK)\n", me);
        return TFIDF_E_HIP;
    }
    uint4* mine = ctx->x_mine.as<uint4>();
    /* padding: all-ones keys (above every short key) for the merge numbering, else EMPTY */
    HIPCHK(hipMemsetAsync(mine, merge ? 0xFF : 0xEE, maxv * 16, s));
    XCHK(launch_keys_by_rank(ctx->vkeys.as<uint4>(), ctx->slot_of_rank.as<uint32_t>(), V, mine, s));
    rc = xp->allgather(mine, ctx->x_gkeys.p, maxv * 16, s);
    if (rc) return rc;
    if (merge) {   /* positions in the merged term order: no table (x_tdf holds the R x V lb's) */
        HIPCHK(hipMemsetAsync(ctx->x_dense.p, 0, (sumv + 1) * 4, s));
        XCHK(launch_dense_merge_ids(ctx->x_gkeys.as<uint4>(), maxv, (uint32_t)R, (uint32_t)me, V,
                                    ctx->x_tdf.as<uint32_t>(), ctx->df_local.as<uint32_t>(), sumv,
                                    ctx->x_pos.as<uint32_t>(), ctx->x_dense.as<uint32_t>(), s));
        rc = xp->allreduce_u32(ctx->x_dense.as<uint32_t>(), sumv + 1, s);
        if (rc) return rc;
        XCHK(launch_dense_gather(ctx->x_dense.as<uint32_t>(), ctx->x_pos.as<uint32_t>(), V,
                                 ctx->df_global.as<uint32_t>(), s));
        HIPCHK(hipMemcpyAsync(cnt + 12, ctx->x_dense.as<uint32_t>() + sumv, 4, hipMemcpyDeviceToDevice, s));
        return 0;
    }
    const uint64_t tcap = table_cap(sumv);
    uint32_t* status = (uint32_t*)(cnt + 3);
    XCHK(launch_dense_ids(ctx->x_gkeys.as<uint4>(), n, ctx->x_tkey.as<uint4>(), ctx->x_tdf.as<uint32_t>(), tcap, cnt + 10,
                          status, s));
    HIPCHK(hipMemsetAsync(ctx->x_dense.p, 0, n * 4, s));
    XCHK(launch_dense_scatter(mine, ctx->df_local.as<uint32_t>(), V, ctx->x_tkey.as<uint4>(), tcap,
                              ctx->x_tdf.as<uint32_t>(), ctx->x_pos.as<uint32_t>(), ctx->x_dense.as<uint32_t>(), status,
                              s));
    rc = xp->allreduce_u32(ctx->x_dense.as<uint32_t>(), n, s);
    if (rc) return rc;
    XCHK(launch_dense_gather(ctx->x_dense.as<uint32_t>(), ctx->x_pos.as<uint32_t>(), V, ctx->df_global.as<uint32_t>(), s));
    /* global V = the distinct keys (the same on every rank) */
    HIPCHK(hipMemcpyAsync(cnt + 12, cnt + 10, 4, hipMemcpyDeviceToDevice, s));
    return 0;
}

/* Cross-rank identity of terms of >= 16 bytes (TFIDF.c:229 joins words across ranks with
 * strcmp).  A long term's identity key is a 120-bit hash of its bytes: inside a rank every
 * key match is checked against the bytes (dev_vocab.h), and here, after the DF exchange, so is
 * every key that two ranks share.  The ranks agree on the largest byte total of their long
 * terms, all-gather their lists (key, length, blob offset; padded with EMPTY keys) and blobs,
 * and every rank compares each entry with the first entry of its key (finalize.hip
 * k_long_verify).  Every rank checks the same gathered data, so all reach the same verdict: a
 * mismatch fails the run everywhere with TFIDF_E_CAPACITY (the terms are never merged), with
 * the transport still usable (*agreed).  Only when some rank holds a long term (bit 32 of the
 * agreement word), so runs without long terms pay nothing. */
static int exchange_long_check(tfidf_ctx* ctx, uint32_t V, const uint8_t* bytes, bool* agreed) {
    hipStream_t s = ctx->stream;
    Xport* xp = ctx->xp;
    const uint64_t R = (uint64_t)xp->nranks;
    int arc = ctx->x_lloc.ensure((size_t)V * (sizeof(LongEnt) + 8) + 64) ? TFIDF_E_NOMEM : 0;
    LongEnt* ents = ctx->x_lloc.as<LongEnt>();
    uint64_t* src = reinterpret_cast<uint64_t*>(ents + V);
    unsigned long long* lc = reinterpret_cast<unsigned long long*>(src + V);
    uint64_t L = 0, B = 0;
    if (!arc) {
        XCHK(launch_long_list(ctx->vkeys.as<uint4>(), ctx->vrep.as<uint64_t>(), ctx->slot_of_rank.as<uint32_t>(), V, ents,
                              src, lc, s));
        HIPCHK(hipMemcpyAsync(ctx->hpin + 28, lc, 16, hipMemcpyDeviceToHost, s));
        XSYNC(s);
        L = ctx->hpin[28];
        B = ctx->hpin[29];
    }
    std::vector<uint64_t> bs;
    int rc = exchange_agree(ctx, arc, B, &bs);
    if (rc) { *agreed = true; return rc == 1 ? TFIDF_E_STATE : rc; }
    uint64_t maxb = 0;
    for (uint64_t x : bs) maxb = x > maxb ? x : maxb;
    const uint64_t lcap = maxb / 16 + 1;            /* a long term has >= 16 bytes */
    const uint64_t bcap = (maxb + 16) & ~15ull;
    const uint64_t n = R * lcap, tcap = table_cap(n);
    arc = (ctx->x_lsend.ensure(lcap * sizeof(LongEnt) + bcap) || ctx->x_lgath.ensure(n * sizeof(LongEnt) + R * bcap) ||
           ctx->x_ltab.ensure(tcap * 20))
              ? TFIDF_E_NOMEM
              : 0;
    rc = exchange_agree(ctx, arc, 0, nullptr);
    if (rc) { *agreed = true; return rc == 1 ? TFIDF_E_STATE : rc; }
    LongEnt* se = ctx->x_lsend.as<LongEnt>();
    uint8_t* sblob = reinterpret_cast<uint8_t*>(se + lcap);
    HIPCHK(hipMemsetAsync(se, 0xEE, lcap * sizeof(LongEnt), s));
    if (L) HIPCHK(hipMemcpyAsync(se, ents, L * sizeof(LongEnt), hipMemcpyDeviceToDevice, s));
    XCHK(launch_long_bytes(ents, src, (uint32_t)L, bytes, sblob, s));
    LongEnt* ge = ctx->x_lgath.as<LongEnt>();
    uint8_t* gblob = reinterpret_cast<uint8_t*>(ge + n);
    rc = xp->allgather(se, ge, lcap * sizeof(LongEnt), s);
    if (rc) return rc;
    rc = xp->allgather(sblob, gblob, bcap, s);
    if (rc) return rc;
    uint4* tkey = ctx->x_ltab.as<uint4>();
    uint32_t* status = reinterpret_cast<uint32_t*>(lc);   /* the list's counters are read: reused */
    HIPCHK(hipMemsetAsync(status, 0, 4, s));
    XCHK(launch_long_verify(ge, n, lcap, gblob, bcap, tkey, reinterpret_cast<uint32_t*>(tkey + tcap), tcap, status, s));
    ctx->hpin[30] = 0;
    HIPCHK(hipMemcpyAsync(ctx->hpin + 30, status, 4, hipMemcpyDeviceToHost, s));
    XSYNC(s);
    const uint32_t st = (uint32_t)ctx->hpin[30];
    *agreed = true;   /* the same verdict on every rank */
    if (st & ST_LONG_COLLIDE) {
        fprintf(stderr, "tfidf: two distinct terms of 16 bytes or more on different ranks share their 120-bit identity key\n");
        return TFIDF_E_CAPACITY;
    }
    if (st & (ST_BOUNDS | ST_VOCAB_SPIN)) {
        fprintf(stderr, "tfidf: internal bounds check tripped in the long-term check (status 0x%x)\n", st);
        return TFIDF_E_STATE;
    }
    return 0;
}

static int exchange_df(tfidf_ctx* ctx, int local_rc, uint32_t V, const uint8_t* bytes) {
    std::vector<uint64_t> vs;
    /* the dense form's buffers, sized from this rank's V before the agreement; a failure
     * travels as bit 33 of step 1's word (no extra exchange): the ranks then take the owner
     * form, which sizes its own buffers, unless the dense form is forced */
    bool dense_nomem = false;
    if (local_rc == 0 && (ctx->xchg_mode >= 2 || (ctx->xchg_mode == 0 && V <= DENSE_XCHG_MAXV))) {
        int arc = dense_alloc(ctx, V, dense_pad(V), (uint64_t)ctx->xp->nranks);
        if (ctx->xnomem_rank == ctx->xp->rank && ctx->xchg_mode != 1) {   /* tests: an allocation failure (once) */
            ctx->xnomem_rank = -1;
            arc = TFIDF_E_NOMEM;
        }
        dense_nomem = arc != 0;
    }
    /* step 1; bit 32 of the word: this rank holds terms of >= 16 bytes; bit 33: its dense
     * buffers could not be allocated */
    int rc = exchange_agree(ctx, local_rc,
                            (uint64_t)V | (ctx->local_long ? 1ull << 32 : 0ull) | (dense_nomem ? 1ull << 33 : 0ull), &vs);
    if (rc) return rc;
    uint64_t maxv = 0;
    bool any_long = false, any_dense_nomem = false;
    for (uint64_t& x : vs) {
        any_long |= ((x >> 32) & 1u) != 0;
        any_dense_nomem |= ((x >> 33) & 1u) != 0;
        x &= 0xFFFFFFFFull;
        maxv = x > maxv ? x : maxv;
    }
    if (any_dense_nomem && ctx->xchg_mode >= 2)   /* the dense form forced: an agreed failure */
        return dense_nomem ? TFIDF_E_NOMEM : TFIDF_E_PEER;
    const bool dense = ctx->xchg_mode >= 2 || (ctx->xchg_mode == 0 && maxv <= DENSE_XCHG_MAXV && !any_dense_nomem);
    ctx->last_dense = dense;
    bool agreed = false;
    rc = dense ? exchange_dense(ctx, V, vs, !any_long && ctx->xchg_mode != 3, &agreed)
               : exchange_owner(ctx, V, vs, &agreed);
    if (!rc && any_long) {
        agreed = false;
        rc = exchange_long_check(ctx, V, bytes, &agreed);
    }
    if (rc && rc != TFIDF_E_PEER && !agreed) ctx->xp->abort();
    return rc;
}

/* The document order (`docN@` strcmp order of the run's documents) on the side stream,
 * joined before the per-position metadata (run_post).  Enqueued right after K1 for a large
 * N (its radix sort is long: started early, it is done long before it is needed), after the
 * vocabulary stage's launches for up to SORT_TILE_MAXN documents (two short launches: the
 * device runs the vocabulary stage while the host enqueues them; c2 +0.9 %, while c5's
 * 1e6-document sort beside its merge stage slowed that by 0.07 ms). */
static int enqueue_doc_order(tfidf_ctx* ctx, const uint32_t* dev_ids, uint32_t N, hipStream_t s2) {
    ENSURE(ctx->dkey0, (size_t)N * 8 + 8);
    ENSURE(ctx->dkey1, (size_t)N * 8 + 8);
    ENSURE(ctx->dseq0, (size_t)N * 4 + 4);
    ENSURE(ctx->dseq1, (size_t)N * 4 + 4);
    {
        /* the radix histograms, or the tile sort's staging (20 B per document) */
        const size_t need2 = (size_t)256 * 4 * ((N + 2047) / 2048 + 1) + (size_t)N * 20 + (1u << 20);
        if (need2 > ctx->arena2_buf.cap && ctx->arena2_buf.ensure(need2) != 0) return TFIDF_E_NOMEM;
        ctx->arena2.base = (uint8_t*)ctx->arena2_buf.p;
        ctx->arena2.cap = ctx->arena2_buf.cap;
        ctx->arena2.used = 0;
        HIPCHK(hipStreamWaitEvent(s2, ctx->ev_fork, 0));   /* recorded when the attempt started */
        LCHK(launch_doc_keys(dev_ids, N, ctx->dkey0.as<uint64_t>(), ctx->dseq0.as<uint32_t>(), s2));
        /* base-11 keys of 10 digits are < 11^10 < 2^35: five bytes, no probe */
        /* up to SORT_TILE_MAXN documents: two launches (tile bitonic sort + rank) instead of
         * two per digit byte */
        int dc = N <= SORT_TILE_MAXN
            ? tile_sort_u64(ctx->dkey0.as<uint64_t>(), ctx->dseq0.as<uint32_t>(), ctx->dkey1.as<uint64_t>(),
                            ctx->dseq1.as<uint32_t>(), N, ctx->arena2, s2)
            : radix_sort_u64(ctx->dkey0.as<uint64_t>(), ctx->dseq0.as<uint32_t>(), ctx->dkey1.as<uint64_t>(),
                             ctx->dseq1.as<uint32_t>(), N, 0x1Fu, ctx->arena2, s2);
        LCHK(dc);
        ctx->order = dc ? ctx->dseq1.as<uint32_t>() : ctx->dseq0.as<uint32_t>();
        HIPCHK(hipEventRecord(ctx->ev_order, s2));
    }
    return 0;
}

/* The local stages of one attempt (this shard only, no collective): K0, K1, vocabulary,
 * merge, local DF.  Returns 0, 1 to retry with grown capacities, <0 on error.  Also
 * checks that the main arena holds what the stages after the exchange need, so that they
 * never ask for a retry. */
static int run_local(tfidf_ctx* ctx, const CorpusDev& c, const uint32_t* dev_ids, uint64_t Nt) {
    hipStream_t s = ctx->stream;
    Arena& ar = ctx->arena;
    const uint32_t N = c.ndocs;
    ar.used = 0;
    ctx->run_N = N;
    ctx->run_V = 0;
    mark(ctx, S_PREP);
    /* the side stream's fork point (the document order needs only the run's inputs): recorded
     * first, while the device still waits for the host's first launches, since a record costs
     * the stream ~5 us wherever it sits */
    HIPCHK(hipEventRecord(ctx->ev_fork, s));
    /* ---- buffers ---- */
    if (ctx->xp) {   /* the exchange's count rows (sized before its agreement: see exchange_owner) */
        const size_t R = (size_t)ctx->nranks;
        ENSURE(ctx->x_cnt, ((R + 1) * (R + 4)) * 4);
    }
    const uint64_t span = c.hi - c.lo;
    /* K1 variant: the slot-keyed kernels (tokcount_st / tokcount_vs) need a 16-byte aligned
     * corpus base; TFIDF_K1=general selects the general kernel (cross-checks).  The LDS-staged
     * kernel runs up to the largest table it addresses (2^25 slots): round 6's leaner rounds
     * made it faster than the round-1 kernel on config 4 too (a 32M-slot table for ~1e7 terms,
     * nearly every token a new (doc, term) pair: K1 4.67 vs 5.02 ms, c4 76.8 vs 75.0 GB/s,
     * profiles/r06_k1_ab_c2.txt call r06l); beyond, k_tokcount_vs */
    const bool aligned = (((uintptr_t)c.bytes & 15u) == 0);
    ctx->k1_vs = aligned && ctx->k1_mode != 2;
    if (ctx->k1_vs && ctx->vcap > K1_VS_MAX_CAP) return TFIDF_E_CAPACITY;
    ctx->k1_sl = ctx->k1_vs && (ctx->k1_mode == 0 || ctx->k1_mode == 3) &&
                 ctx->vcap <= ctx->sl_maxcap;
    /* tokcount_sl over a high-cardinality table (past K1_ST_MAX_CAP slots): half-size chunks,
     * as tokcount_vs, since nearly every token is a new pair for its LDS table */
    const uint32_t cb = ctx->k1_sl ? (ctx->vcap > K1_ST_MAX_CAP ? CHUNK_BYTES : CHUNK_BYTES_ST) : CHUNK_BYTES;
    const uint64_t nchunks = span ? (span + cb - 1) / cb : 0;
    if (ctx->rec_cap == 0) ctx->rec_cap = span / 6 + 4096;
    if (ctx->part_cap == 0) ctx->part_cap = span / 64 + 4096;
    ENSURE(ctx->chunk_start, (nchunks + 1) * 8);
    ENSURE(ctx->chunk_doc, (nchunks + 1) * 4);
    ENSURE(ctx->vkeys, ctx->vcap * 16);
    ENSURE(ctx->vrep, ctx->vcap * 8);
    ENSURE(ctx->rec_slot, ctx->rec_cap * 4);
    ENSURE(ctx->rec_cnt, ctx->rec_cap * 4);
    ENSURE(ctx->part_doc, ctx->part_cap * 4);
    ENSURE(ctx->part_slot, ctx->part_cap * 4);
    ENSURE(ctx->part_cnt, ctx->part_cap * 4);
    ENSURE(ctx->doc_recoff, (size_t)N * 8 + 8);
    ENSURE(ctx->doc_npairs, (size_t)N * 4 + 4);
    ENSURE(ctx->doc_size, (size_t)N * 4 + 4);
    ENSURE(ctx->doc_flags, (size_t)N + 1);
    unsigned long long* cnt = ctx->counters.as<unsigned long long>(); /* rec, part, ntok, status */
    {   /* the run's clears in one launch: the vocabulary table (EMPTY keys), K1's counters,
         * status and sharded chunk counters, the per-document pairs / sizes / flags */
        FillList fl{};
        auto add = [&](void* p, uint64_t bytes, uint32_t byte) {
            fl.p[fl.n] = p;
            fl.bytes[fl.n] = bytes;
            fl.val[fl.n] = byte * 0x01010101u;
            ++fl.n;
        };
        add(ctx->vkeys.p, ctx->vcap * 16, 0xEEu);
        add(cnt, 256, 0u);
        add(ctx->doc_npairs.p, (size_t)N * 4 + 4, 0u);
        add(ctx->doc_size.p, (size_t)N * 4 + 4, 0u);
        add(ctx->doc_flags.p, (size_t)N + 1, 0u);
        LCHK(launch_fill_multi(fl, s));
    }
    ENSURE(ctx->big_list, (size_t)BIG_LIST_CAP * 4);
    if (nchunks)
        LCHK(launch_plan_chunks(c, nchunks, cb, ctx->chunk_start.as<uint64_t>(), ctx->chunk_doc.as<uint32_t>(),
                                ctx->big_list.as<uint32_t>(), cnt + 6, s));
    /* ---- K1 ---- */
    mark(ctx, S_TOKCOUNT);
    VocabDev vd{ctx->vkeys.as<uint4>(), ctx->vrep.as<uint64_t>(), ctx->vcap - 1};
    K1Out o{};
    o.rec_slot = ctx->rec_slot.as<uint32_t>();
    o.rec_cnt = ctx->rec_cnt.as<uint32_t>();
    o.rec_alloc = cnt + 0;
    o.rec_cap = ctx->rec_cap;
    o.part_doc = ctx->part_doc.as<uint32_t>();
    o.part_slot = ctx->part_slot.as<uint32_t>();
    o.part_cnt = ctx->part_cnt.as<uint32_t>();
    o.part_alloc = cnt + 1;
    o.part_cap = ctx->part_cap;
    o.doc_recoff = ctx->doc_recoff.as<uint64_t>();
    o.doc_npairs = ctx->doc_npairs.as<uint32_t>();
    o.doc_size = ctx->doc_size.as<uint32_t>();
    o.doc_flags = ctx->doc_flags.as<uint8_t>();
    o.ntokens = cnt + 2;
    o.chunk_ctr = cnt + 5;
    o.chunk_shard = cnt + 16;
    o.status = (uint32_t*)(cnt + 3);
    o.stamps = nullptr;
    if (ctx->stamps_on) {
        ENSURE(ctx->stamps, 8 * K1_DEBUG_WORDS);
        HIPCHK(hipMemsetAsync(ctx->stamps.p, 0, 8 * K1_DEBUG_WORDS, s));
        o.stamps = ctx->stamps.as<unsigned long long>();
    }
    if (nchunks && ctx->k1_sl) {
        /* pinned source: the copy is stream-ordered before the launch, and the block is not
         * rewritten before the next run (every run synchronises with the host after K1) */
        if (!ctx->k1out_valid || memcmp(ctx->k1out_host, &o, sizeof(K1Out)) != 0) {   /* steady state: unchanged */
            ctx->k1out_valid = false;   /* until the copy of the new block is enqueued */
            *ctx->k1out_host = o;
            HIPCHK(hipMemcpyAsync(ctx->k1out_dev.p, ctx->k1out_host, sizeof(K1Out), hipMemcpyHostToDevice, s));
            ctx->k1out_valid = true;
        }
        LCHK(launch_tokcount_sl(c, ctx->chunk_start.as<uint64_t>(), ctx->chunk_doc.as<uint32_t>(), 0, nchunks, vd,
                                ctx->k1out_dev.as<K1Out>(), s));
    } else if (nchunks && ctx->k1_vs)
        LCHK(launch_tokcount_vs(c, ctx->chunk_start.as<uint64_t>(), ctx->chunk_doc.as<uint32_t>(), 0, nchunks, vd, o, s));
    else if (nchunks)
        LCHK(launch_tokcount(c, ctx->chunk_start.as<uint64_t>(), ctx->chunk_doc.as<uint32_t>(), 0, nchunks, vd, o, s));
    mark(ctx, S_VOCAB);
    /* the vocabulary's used-slot flags and count are enqueued before the host reads K1's
     * counters: one host round trip for both */
    const uint64_t cap = ctx->vcap;
    ENSURE(ctx->dense, (cap + 1) * 4);
    LCHK(launch_vocab_flags(vd, cap, ctx->dense.as<uint32_t>(), s));
    LCHK(scan_excl_u32(ctx->dense.as<uint32_t>(), ctx->dense.as<uint32_t>(), cap, ar, s));
    uint64_t* hp = ctx->hpin;
    {   /* K1's counters (hp[0..7]) and the vocabulary size (hp[8]): one launch */
        WordList wl{};
        for (int i = 0; i < 8; ++i) { wl.src[i] = cnt + i; wl.bytes[i] = 8; }
        wl.src[8] = ctx->dense.as<uint32_t>() + cap;
        wl.bytes[8] = 4;
        wl.n = 9;
        HIPCHK(words_wait(ctx, wl, 0, s));
    }
    const uint32_t V = (uint32_t)hp[8];
    unsigned long long hc[8];
    for (int i = 0; i < 8; ++i) hc[i] = hp[i];
    const uint64_t R_main = hc[0], Q = hc[1], nbig = hc[6];
    const uint32_t st = (uint32_t)hc[3];
    ctx->local_long = (st & ST_HAS_LONG) != 0;
    ctx->ntokens = hc[2];
    ctx->nchunks = nchunks;
    ctx->nrec_part = Q;
    if (st & (ST_VOCAB_SPIN | ST_TERM_LONG)) return TFIDF_E_CAPACITY;
    if (st & ST_LONG_COLLIDE) {   /* dev_vocab.h: reported, never merged */
        fprintf(stderr, "tfidf: two distinct terms of 16 bytes or more share their 120-bit identity key\n");
        return TFIDF_E_CAPACITY;
    }
    bool retry = false;
    if (st & ST_BOUNDS) {
        fprintf(stderr, "tfidf: internal bounds check tripped in K1 (status 0x%x)\n", st);
        return TFIDF_E_STATE;
    }
    if (st & ST_VOCAB_FULL) {   /* the run stopped inserting early: V unknown */
        if (ctx->vcap >= K1_VS_MAX_CAP) return TFIDF_E_CAPACITY;
        ctx->vcap = ctx->vcap * 4 < K1_VS_MAX_CAP ? ctx->vcap * 4 : K1_VS_MAX_CAP;
        retry = true;
    }
    if (st & ST_REC_FULL) { ctx->rec_cap = R_main + R_main / 4 + 4096; retry = true; }
    if (st & ST_PART_FULL) { ctx->part_cap = Q + Q / 4 + 4096; retry = true; }
    if (retry) return 1;
    if (N > SORT_TILE_MAXN) {   /* see enqueue_doc_order */
        const int rc = enqueue_doc_order(ctx, dev_ids, N, ctx->stream2);
        if (rc) return rc;
    }
    /* ---- vocabulary ---- */
    ctx->V = V;
    /* keep probes short: the low load pays while the table is L2/MALL-sized (<= 16M slots,
     * 256 MB of keys); past that every probe is an HBM access anyway, so up to 45 % */
    if ((uint64_t)V * 100 > cap * (cap < VOCAB_LOW_LOAD_CAP ? ctx->vload_pct : ctx->vload_big_pct)) {
        /* the smallest table within the load limit: a table twice too large costs its
         * clear and a sparser compaction pass (c4: 64M -> 32M slots, vocabulary stage
         * 3.1 -> 2.65 ms) */
        while ((uint64_t)V * 100 > ctx->vcap * (ctx->vcap < VOCAB_LOW_LOAD_CAP ? ctx->vload_pct : ctx->vload_big_pct))
            ctx->vcap *= 2;
        if (ctx->vcap > K1_VS_MAX_CAP && cap < K1_VS_MAX_CAP) ctx->vcap = K1_VS_MAX_CAP;
        if (ctx->vcap != cap) return 1;
    }
    ENSURE(ctx->vslot, (size_t)V * 4 + 4);
    ENSURE(ctx->skey0, (size_t)V * 16 + 16);
    ENSURE(ctx->skey1, (size_t)V * 16 + 16);
    ENSURE(ctx->seq0, (size_t)V * 4 + 4);
    ENSURE(ctx->seq1, (size_t)V * 4 + 4);
    /* rank maps: one entry per slot */
    ENSURE(ctx->rank_of_slot, cap * 4);
    ENSURE(ctx->slot_of_rank, (size_t)V * 4 + 4);
    LCHK(launch_vocab_compact(vd, cap, ctx->dense.as<uint32_t>(), c, ctx->vslot.as<uint32_t>(), ctx->skey0.as<uint4>(),
                              ctx->seq0.as<uint32_t>(), s));
    if (V <= SORT_TILE_MAXN) { /* two launches, no varying-byte probe (no host sync) */
        const int cur = tile_sort_u128(ctx->skey0.as<uint4>(), ctx->seq0.as<uint32_t>(), ctx->skey1.as<uint4>(),
                             ctx->seq1.as<uint32_t>(), V, ar, s);
        LCHK(cur);
        ctx->sorted_skey = cur ? ctx->skey1.as<uint4>() : ctx->skey0.as<uint4>();
        ctx->sorted_dense = cur ? ctx->seq1.as<uint32_t>() : ctx->seq0.as<uint32_t>();
    } else {
        /* a u64 LSD sort of the keys' high halves (their first 8 bytes) over the varying
         * bytes, then the runs of equal prefixes re-ordered by the low halves
         * (launch_vocab_prefix_ties: few at c4, so 8 digit passes instead of 13; vocabulary
         * 2.19 -> 2.00 ms, profiles/r04_c4_ab.txt); skey0 stays in dense order,
         * skey1 holds the two u64 ping-pong buffers */
        uint32_t vm = 0;
        LCHK(key_varying_bytes_u128(ctx->skey0.as<uint4>(), V, &vm, ar, s));
        uint64_t* const ka = (uint64_t*)ctx->skey1.p;
        uint64_t* const kb = ka + V;
        uint32_t* const sa = ctx->seq0.as<uint32_t>();
        uint32_t* const sbq = ctx->seq1.as<uint32_t>();
        LCHK(launch_sortkey_half(ctx->skey0.as<uint4>(), V, nullptr, 1, ka, s));
        const int c1 = radix_sort_u64(ka, sa, kb, sbq, V, (vm >> 8) & 0xFFu, ar, s);
        LCHK(c1);
        ctx->sorted_dense = c1 ? sbq : sa;
        LCHK(launch_vocab_prefix_ties(c1 ? kb : ka, ctx->sorted_dense, ctx->skey0.as<uint4>(), V, vm & 0xFFu, ar, s));
        ctx->sorted_skey = nullptr;
        if (st & ST_HAS_LONG) {   /* the fix-up reads the keys in sorted order */
            LCHK(launch_gather_u128(ctx->skey0.as<uint4>(), ctx->sorted_dense, V, ctx->skey1.as<uint4>(), s));
            ctx->sorted_skey = ctx->skey1.as<uint4>();
        }
    }
    if (st & ST_HAS_LONG)   /* terms of >= 16 bytes exist: order the ones tied on 16 bytes */
        LCHK(launch_vocab_long_fixup(ctx->sorted_skey, ctx->sorted_dense, ctx->vslot.as<uint32_t>(), vd, c, V, ar, s));
    uint16_t* r16 = nullptr;
    if (V <= 65536u) { ENSURE(ctx->rank16, cap * 2); r16 = ctx->rank16.as<uint16_t>(); }
    LCHK(launch_vocab_rank(ctx->sorted_dense, ctx->vslot.as<uint32_t>(), V, ctx->rank_of_slot.as<uint32_t>(),
                           ctx->slot_of_rank.as<uint32_t>(), r16, s));
    if (N <= SORT_TILE_MAXN) {   /* see enqueue_doc_order */
        const int rc = enqueue_doc_order(ctx, dev_ids, N, ctx->stream2);
        if (rc) return rc;
    }
    /* split DF: with partial records to merge, the main records' histogram (which needs only
     * the term ranks) starts on stream2 now and runs beside the merge stage's short
     * launches; the merged records are added after the merge (accumulate pass below) */
    const bool df_split = ctx->df_split && Q && R_main;
    ENSURE(ctx->df_local, (size_t)V * 4 + 4);
    ENSURE(ctx->df_global, (size_t)V * 4 + 4);
    if (df_split) {
        if (R_main + Q > ctx->rec_cap) {   /* the merge's growth, done before stream2 reads the records */
            uint64_t ncap = R_main + Q + (R_main + Q) / 8 + 4096;
            if (ctx->rec_slot.grow_keep(ncap * 4, R_main * 4, s) || ctx->rec_cnt.grow_keep(ncap * 4, R_main * 4, s))
                return TFIDF_E_NOMEM;
            ctx->rec_cap = ncap;
        }
        const size_t dneed = df_hist_scratch(R_main, V);
        ENSURE(ctx->df_scratch, dneed > ctx->df_scratch_min ? dneed : ctx->df_scratch_min);
        Arena da;
        da.base = (uint8_t*)ctx->df_scratch.p;
        da.cap = ctx->df_scratch.cap;
        HIPCHK(hipEventRecord(ctx->ev_vrank, s));
        HIPCHK(hipStreamWaitEvent(ctx->stream2, ctx->ev_vrank, 0));
        const int dl = launch_df_hist(ctx->rec_slot.as<uint32_t>(), R_main, nullptr, R_main, ctx->rank_of_slot.as<uint32_t>(),
                                      r16, V, cap, (uint32_t*)(cnt + 3), ctx->df_local.as<uint32_t>(), da, ctx->stream2);
        if (dl == -2) {   /* its own scratch was short: grow it (not the arena) and retry */
            ctx->df_scratch_min = da.peak + da.peak / 2 + 4096;
            return 1;
        }
        LCHK(dl);
        HIPCHK(hipEventRecord(ctx->ev_dfmain, ctx->stream2));
    }
    /* this run's full idf table (idf_start's workers finish during K1 in practice) goes up
     * on its own copy stream now, beside the merge and DF stages, instead of inside the idf
     * stage on the main stream (an SDMA copy of (N+1) doubles: ~35 us there for c2) */
    if (ctx->idf_pool.busy && !ctx->idf_early && idf_done(ctx)) {
        idf_join(ctx);
        ENSURE(ctx->idf_vals, (size_t)(Nt + 1) * 8);
        HIPCHK(hipMemcpyAsync(ctx->idf_vals.p, ctx->idf_pin, (size_t)(Nt + 1) * 8, hipMemcpyHostToDevice,
                              ctx->stream3));
        HIPCHK(hipEventRecord(ctx->ev_idf_up, ctx->stream3));
        ctx->idf_pin_busy = true;
        ctx->idf_early = true;
    }
    /* ---- partial documents ---- */
    mark(ctx, S_MERGE);
    uint64_t R_total = R_main;
    const uint32_t* merged_count = nullptr;   /* device: merged + dense records beyond R_main */
    {
        /* Q follows K1's overflow records, which vary from run to run (the order of the LDS
         * claims): at least 2^20 entries (28 MB in all), also when this run has none, so that
         * a shard with few or no partial records does not allocate in steady state (c5 at 8
         * shards: 0 -> 28 K -> 90 K, ten device allocations in its timed steps,
         * TFIDF_DEBUG_ALLOC=1) */
        const uint64_t Qc = Q < (1ull << 20) ? (1ull << 20) : Q;
        ENSURE(ctx->pkey0, Qc * 8);
        ENSURE(ctx->pkey1, Qc * 8);
        ENSURE(ctx->pseq0, Qc * 4);
        ENSURE(ctx->pseq1, Qc * 4);
        ENSURE(ctx->phead, (Qc + 1) * 4);
    }
    if (Q) {
        /* merged (and dense) records land in [R_main, R_main + Q): size for the worst case */
        if (R_main + Q > ctx->rec_cap) {
            uint64_t ncap = R_main + Q + (R_main + Q) / 8 + 4096;
            if (ctx->rec_slot.grow_keep(ncap * 4, R_main * 4, s) || ctx->rec_cnt.grow_keep(ncap * 4, R_main * 4, s))
                return TFIDF_E_NOMEM;
            ctx->rec_cap = ncap;
        }
        /* documents longer than DENSE_DOC (listed by K0): their partial records are summed
         * in dense per-document arrays over ranks (<= 256 MB of them) instead of sorted */
        uint32_t nb = 0;
        if (nbig && V) {
            const uint64_t lim = (256ull << 20) / (4ull * V * DENSE_REP);
            uint64_t m = nbig < (uint64_t)BIG_LIST_CAP ? nbig : (uint64_t)BIG_LIST_CAP;
            nb = (uint32_t)(m < lim ? m : lim);
        }
        uint64_t Qs = Q;                                  /* records to sort */
        const uint32_t* scnt = ctx->part_cnt.as<uint32_t>();
        if (nb) {
            ENSURE(ctx->big_idx, (size_t)N * 4 + 4);
            ENSURE(ctx->dense_cnt, (size_t)nb * V * 4 * DENSE_REP);
            ENSURE(ctx->kcnt, Q * 4);
            uint32_t* nkeep = (uint32_t*)(cnt + 7);   /* zeroed with the run's counters */
            HIPCHK(hipMemsetAsync(ctx->big_idx.p, 0xFF, (size_t)N * 4 + 4, s));
            HIPCHK(hipMemsetAsync(ctx->dense_cnt.p, 0, (size_t)nb * V * 4 * DENSE_REP, s));
            LCHK(launch_set_big_idx(ctx->big_list.as<uint32_t>(), nb, ctx->big_idx.as<uint32_t>(), s));
            LCHK(launch_part_dense(ctx->part_doc.as<uint32_t>(), ctx->part_slot.as<uint32_t>(), ctx->part_cnt.as<uint32_t>(),
                                   Q, ctx->big_idx.as<uint32_t>(), ctx->rank_of_slot.as<uint32_t>(), V,
                                   ctx->dense_cnt.as<uint32_t>(), ctx->pkey0.as<uint64_t>(), ctx->pseq0.as<uint32_t>(),
                                   ctx->kcnt.as<uint32_t>(), nkeep, s));
            /* the sort needs its size on the host: one round trip, dense runs only */
            ctx->hpin[9] = 0;
            HIPCHK(hipMemcpyAsync(ctx->hpin + 9, nkeep, 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            const uint32_t qk = (uint32_t)ctx->hpin[9];
            Qs = qk;
            scnt = ctx->kcnt.as<uint32_t>();
        } else {
            LCHK(launch_part_keys(ctx->part_doc.as<uint32_t>(), ctx->part_slot.as<uint32_t>(),
                                  ctx->rank_of_slot.as<uint32_t>(), Q, ctx->pkey0.as<uint64_t>(),
                                  ctx->pseq0.as<uint32_t>(), s));
        }
        uint32_t* ph = ctx->phead.as<uint32_t>();
        if (Qs) {
            uint32_t pm = 0;
            /* key = (local doc << 32) | rank: the varying bytes follow from N and V (no probe,
             * no host sync) */
            {
                const uint32_t rb = V > 1 ? 32u - (uint32_t)__builtin_clz(V - 1) : 1u;
                const uint32_t db = N > 1 ? 32u - (uint32_t)__builtin_clz(N - 1) : 1u;
                for (uint32_t b = 0; b < (rb + 7) / 8; ++b) pm |= 1u << b;
                for (uint32_t b = 0; b < (db + 7) / 8; ++b) pm |= 1u << (4 + b);
            }
            int pc = Qs <= SORT_TILE_MAXN   /* c2's ~1e5 partial records: two launches, not two per byte */
                ? tile_sort_u64(ctx->pkey0.as<uint64_t>(), ctx->pseq0.as<uint32_t>(), ctx->pkey1.as<uint64_t>(),
                                ctx->pseq1.as<uint32_t>(), Qs, ar, s)
                : radix_sort_u64(ctx->pkey0.as<uint64_t>(), ctx->pseq0.as<uint32_t>(), ctx->pkey1.as<uint64_t>(),
                                 ctx->pseq1.as<uint32_t>(), Qs, pm, ar, s);
            LCHK(pc);
            uint64_t* pk = pc ? ctx->pkey1.as<uint64_t>() : ctx->pkey0.as<uint64_t>();
            uint32_t* ps = pc ? ctx->pseq1.as<uint32_t>() : ctx->pseq0.as<uint32_t>();
            LCHK(launch_part_heads(pk, Qs, ph, s));
            LCHK(scan_excl_u32(ph, ph, Qs, ar, s));
            /* U = ph[Qs] merged records (<= Qs) stays on the device: no host round trip */
            LCHK(launch_part_merge(pk, ps, scnt, ph, Qs, ctx->slot_of_rank.as<uint32_t>(), R_main,
                                   ctx->rec_slot.as<uint32_t>(), ctx->rec_cnt.as<uint32_t>(),
                                   ctx->doc_recoff.as<uint64_t>(), ctx->doc_npairs.as<uint32_t>(),
                                   ctx->doc_flags.as<uint8_t>(), s));
        } else {
            HIPCHK(hipMemsetAsync(ph, 0, 4, s));
        }
        if (nb) {
            const uint64_t nt = ((uint64_t)V + 1023) / 1024;
            ENSURE(ctx->tile_cnt, (nt * nb + 1) * 4);
            LCHK(launch_dense_emit(ctx->dense_cnt.as<uint32_t>(), nb, V, ctx->big_list.as<uint32_t>(),
                                   ctx->slot_of_rank.as<uint32_t>(), R_main, ph + Qs, ctx->tile_cnt.as<uint32_t>(),
                                   ctx->rec_slot.as<uint32_t>(), ctx->rec_cnt.as<uint32_t>(),
                                   ctx->doc_recoff.as<uint64_t>(), ctx->doc_npairs.as<uint32_t>(),
                                   ctx->doc_flags.as<uint8_t>(), ar, s));
        }
        merged_count = ph + Qs;
        R_total = R_main + Q; /* an upper bound: the true count is R_main + *merged_count */
    }
    /* ---- DF ---- */
    mark(ctx, S_DF);
    if (df_split) {   /* the merged records (term ranks) added to the main records' df */
        HIPCHK(hipStreamWaitEvent(s, ctx->ev_dfmain, 0));
        LCHK(launch_df_hist(ctx->rec_slot.as<uint32_t>() + R_main, 0, merged_count, R_total - R_main,
                            ctx->rank_of_slot.as<uint32_t>(), r16, V, cap, (uint32_t*)(cnt + 3),
                            ctx->df_local.as<uint32_t>(), ar, s, true));
    } else {
        /* also rewrites every record's slot as its term rank (K5 then needs no rank gather) */
        LCHK(launch_df_hist(ctx->rec_slot.as<uint32_t>(), R_main, merged_count, R_total,
                            ctx->rank_of_slot.as<uint32_t>(), r16, V, cap, (uint32_t*)(cnt + 3),
                            ctx->df_local.as<uint32_t>(), ar, s));
    }
    ctx->run_V = V;
    ctx->run_cap = cap;
    ctx->run_R_total = R_total;
    ctx->run_merged = merged_count;
    /* the stages after the exchange take their scratch from what is left of the arena */
    const size_t post_need = scan_scratch(Nt + 1) + (size_t)(Nt + 2) * 4 + 512 + scan_scratch(N) +
                             scan_scratch(3ull * ((N + 255) / 256) + 1);   /* K5's document classes */
    if (ar.cap - ar.used < post_need) {
        ar.peak = ar.used + post_need > ar.peak ? ar.used + post_need : ar.peak;
        return 1;
    }
    return 0;
}

/* ---- the per-run idf table: log(N/df) for every df = 0..N on the host's libm
 * (TFIDF.c:243 evaluates log(1.0*N/df) per pair; the table holds the same doubles), on up to
 * eight host threads per process (shared out over its open contexts) posted when the run
 * starts, so the logs run beside K1 .. DF on the device.  run_post waits for them (ms_idf_wait: normally 0) and uploads the table. */
#define IDF_POOL 8
static void idf_worker(tfidf_ctx::IdfPool* P, unsigned i) {
    uint64_t seen = 0;
    for (;;) {
        std::unique_lock<std::mutex> lk(P->mu);
        P->go.wait(lk, [&] { return P->stop || P->gen != seen; });
        if (P->stop) return;
        seen = P->gen;
        if (i >= P->active) continue;
        double* lut = P->lut;
        const uint32_t* vals = P->vals;
        const uint64_t Nt = P->Nt, n = P->n, lo = (n * i) / P->active, hi = (n * (i + 1)) / P->active;
        const auto t0 = P->t0;
        lk.unlock();
        if (vals)
            for (uint64_t k = lo; k < hi; ++k) lut[k] = log(1.0 * (double)Nt / (double)vals[k]);
        else
            for (uint64_t d = lo + 1; d < hi + 1; ++d) lut[d] = log(1.0 * (double)Nt / (double)d);
        const int64_t e = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        lk.lock();
        P->end_ns = e > P->end_ns ? e : P->end_ns;
        if (--P->left == 0) P->done.notify_all();
    }
}
static void idf_pool_stop(tfidf_ctx* ctx) {
    tfidf_ctx::IdfPool& P = ctx->idf_pool;
    {
        std::unique_lock<std::mutex> lk(P.mu);
        P.done.wait(lk, [&] { return P.left == 0; });
        P.stop = true;
    }
    P.go.notify_all();
    for (auto& t : P.th) t.join();
    P.th.clear();
}
/* posts a table job to the context's workers (lut: n values; vals null = every df 1..n) */
static void idf_post(tfidf_ctx* ctx, double* lut, uint64_t Nt, const uint32_t* vals, uint64_t n) {
    tfidf_ctx::IdfPool& P = ctx->idf_pool;
    const int live = g_live_ctx.load();
    const unsigned share = live > 1 ? (unsigned)(IDF_POOL / live > 1 ? IDF_POOL / live : 1) : IDF_POOL;
    const unsigned want = (unsigned)(n / 16384 < 1 ? 1 : (n / 16384 > share ? share : n / 16384));
    while (P.th.size() < want) P.th.emplace_back(idf_worker, &P, (unsigned)P.th.size());   /* started once, as needed */
    {
        std::lock_guard<std::mutex> lk(P.mu);
        P.active = want;
        P.left = P.active;
        P.lut = lut;
        P.Nt = Nt;
        P.vals = vals;
        P.n = n;
        P.t0 = std::chrono::steady_clock::now();
        P.end_ns = 0;
        P.busy = true;
        ++P.gen;
    }
    P.go.notify_all();
}
/* Waits for every upload that may still read idf_pin or write idf_vals: a failed run can leave
 * the early upload (stream3, run_local) or the late one (the main stream, run_post) queued, and
 * the next run must neither rewrite / free idf_pin under it nor have it land after its own copy */
static int idf_pin_quiesce(tfidf_ctx* ctx) {
    if (!ctx->idf_pin_busy) return TFIDF_OK;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream3));
    ctx->idf_pin_busy = false;
    return TFIDF_OK;
}
static int idf_start(tfidf_ctx* ctx, uint64_t Nt) {
    ctx->idf_logs = 0;
    ctx->idf_early = false;
    ctx->ms_idf_host = ctx->ms_idf_wait = 0;
    if (Nt > IDF_FULL_MAX) return TFIDF_OK;                          /* distinct-df path in run_post */
    if (const int q = idf_pin_quiesce(ctx)) return q;   /* a failed run left an upload of idf_pin unwaited */
    const size_t n = (size_t)Nt + 1;
    if (ctx->idf_pin_n < n) {
        if (ctx->idf_pin) (void)hipHostFree(ctx->idf_pin);
        ctx->idf_pin = nullptr;
        ctx->idf_pin_n = 0;
        if (hipHostMalloc((void**)&ctx->idf_pin, n * 8, hipHostMallocDefault) != hipSuccess) return TFIDF_E_NOMEM;
        ctx->idf_pin_n = n;
    }
    ctx->idf_full_n = 0;   /* idf_vals is rewritten by this run */
    ctx->idf_pin[0] = 0.0;   /* df >= 1 for every term that occurs */
    idf_post(ctx, ctx->idf_pin, Nt, nullptr, Nt);
    ctx->idf_logs = Nt;
    return TFIDF_OK;
}
/* waits for the table's workers (also on every error path of tfidf_run) */
static void idf_join(tfidf_ctx* ctx) {
    tfidf_ctx::IdfPool& P = ctx->idf_pool;
    if (!P.busy) return;
    const auto w0 = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(P.mu);
    P.done.wait(lk, [&] { return P.left == 0; });
    P.busy = false;
    ctx->ms_idf_wait = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    ctx->ms_idf_host = (double)P.end_ns * 1e-6;
}
struct IdfJoin {
    tfidf_ctx* c;
    ~IdfJoin() { idf_join(c); }
};
/* the table finished by now? (no wait) */
static bool idf_done(tfidf_ctx* ctx) {
    tfidf_ctx::IdfPool& P = ctx->idf_pool;
    std::lock_guard<std::mutex> lk(P.mu);
    return P.left == 0;
}

/* The stages after the DF exchange: idf LUT, document order, score.  They never return 1
 * (run_local checked their scratch before the exchange), so no rank can ever enter the
 * collectives of a repeated attempt alone: every `return` below is an error or success. */
static int run_post(tfidf_ctx* ctx, uint64_t Nt) {
    hipStream_t s = ctx->stream;
    Arena& ar = ctx->arena;
    const uint32_t N = ctx->run_N, V = ctx->run_V;
    const uint64_t cap = ctx->run_cap, R_total = ctx->run_R_total;
    unsigned long long* cnt = ctx->counters.as<unsigned long long>();
    /* ---- idf: log(N/df) on the host's libm (TFIDF.c:243) ----
     * Up to IDF_FULL_MAX documents the host tabulates every possible value, df = 1..N,
     * once per N (cached with the context and uploaded once): the device then reads
     * idf[df] directly and the run needs no host round trip between DF and the score.
     * Above it (c3-size N on one rank) the distinct df values are listed on the device and
     * come back in one round trip with the pair total. */
    mark(ctx, S_IDF);
    const bool full_lut = Nt <= IDF_FULL_MAX;
    uint32_t K = 0;
    uint32_t* vals_dev = nullptr;
    constexpr uint32_t IDF_SPEC = 16384;
    std::vector<uint32_t> vals;
    if (full_lut) {
        if (ctx->idf_early) {       /* on its way up stream3 (run_local) */
            HIPCHK(hipStreamWaitEvent(s, ctx->ev_idf_up, 0));
            ctx->idf_full_n = Nt;
        } else if (ctx->idf_pool.busy) {   /* this run's table (idf_start): join, upload */
            ENSURE(ctx->idf_vals, (size_t)(Nt + 1) * 8);
            idf_join(ctx);
            HIPCHK(hipMemcpyAsync(ctx->idf_vals.p, ctx->idf_pin, (size_t)(Nt + 1) * 8, hipMemcpyHostToDevice, s));
            ctx->idf_pin_busy = true;
            ctx->idf_full_n = Nt;
        } else if (ctx->idf_full_n != Nt) {
            return TFIDF_E_STATE;   /* idf_start made no table and none is cached: not reachable */
        }
    } else {
        ctx->idf_full_n = 0;   /* idf_vals is rewritten below */
        ENSURE(ctx->present, (Nt + 2) * 4);
        HIPCHK(hipMemsetAsync(ctx->present.p, 0, (Nt + 2) * 4, s));
        XCHK(launch_df_mark(df_of_run(ctx), V, ctx->present.as<uint32_t>(), s));
        XCHK(scan_excl_u32(ctx->present.as<uint32_t>(), ctx->present.as<uint32_t>(), Nt + 1, ar, s));
        vals_dev = (uint32_t*)ar.get((size_t)(Nt + 2) * 4);
        if (!vals_dev) return TFIDF_E_CAPACITY;   /* checked by run_local: not reachable */
        XCHK(launch_df_list(ctx->present.as<uint32_t>(), Nt + 1, vals_dev, s));
        const uint32_t spec = (uint32_t)((Nt + 1) < IDF_SPEC ? (Nt + 1) : IDF_SPEC);
        vals.resize(spec);
        HIPCHK(hipMemcpyAsync(&K, ctx->present.as<uint32_t>() + Nt + 1, 4, hipMemcpyDeviceToHost, s));
        if (spec) HIPCHK(hipMemcpyAsync(vals.data(), vals_dev, (size_t)spec * 4, hipMemcpyDeviceToHost, s));
    }
    /* ---- document order: per-position metadata and pair offsets ---- */
    mark(ctx, S_ORDER);
    ENSURE(ctx->npairs_ord, (size_t)N * 8 + 8);
    ENSURE(ctx->out_off, (size_t)N * 8 + 8);
    HIPCHK(hipStreamWaitEvent(s, ctx->ev_order, 0)); /* join the side stream's document order */
    ENSURE(ctx->doc_meta, (size_t)N * 16 + 16);
    XCHK(launch_gather_meta(ctx->order, ctx->doc_npairs.as<uint32_t>(), ctx->doc_recoff.as<uint64_t>(),
                            ctx->doc_size.as<uint32_t>(), ctx->doc_flags.as<uint8_t>(), N,
                            ctx->npairs_ord.as<uint64_t>(), ctx->doc_meta.as<uint4>(), s));
    XCHK(scan_excl_u64(ctx->npairs_ord.as<uint64_t>(), ctx->out_off.as<uint64_t>(), N, ar, s));
    if (!full_lut) {
        XSYNC(s);
        const uint32_t spec = (uint32_t)vals.size();
        if (K > spec) {
            vals.resize(K);
            HIPCHK(hipMemcpy(vals.data() + spec, vals_dev + spec, (size_t)(K - spec) * 4, hipMemcpyDeviceToHost));
        }
        ENSURE(ctx->idf_vals, (size_t)K * 8 + 8);
        /* the distinct df values' logs on the context's workers, into pinned memory */
        if (const int q = idf_pin_quiesce(ctx)) return q;   /* a failed run left an upload of idf_pin unwaited */
        if (ctx->idf_pin_n < (size_t)K + 1) {
            if (ctx->idf_pin) (void)hipHostFree(ctx->idf_pin);
            ctx->idf_pin = nullptr;
            ctx->idf_pin_n = 0;
            if (hipHostMalloc((void**)&ctx->idf_pin, ((size_t)K + 1) * 8, hipHostMallocDefault) != hipSuccess)
                return TFIDF_E_NOMEM;
            ctx->idf_pin_n = (size_t)K + 1;
        }
        if (K) {
            if (K < 2 * 16384) {   /* one worker's share: on this thread, no hand-off and wake-up */
                const auto t0 = std::chrono::steady_clock::now();
                for (uint32_t k = 0; k < K; ++k) ctx->idf_pin[k] = log(1.0 * (double)Nt / (double)vals[k]);
                ctx->ms_idf_host = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            } else {
                idf_post(ctx, ctx->idf_pin, Nt, vals.data(), K);
                idf_join(ctx);
            }
            HIPCHK(hipMemcpyAsync(ctx->idf_vals.p, ctx->idf_pin, (size_t)K * 8, hipMemcpyHostToDevice, s));
            ctx->idf_pin_busy = true;
        }
        ctx->idf_logs = K;   /* this run's distinct df values */
    }
    /* the output arrays are sized by the record bound (pairs <= records): the pair total P
     * comes back with the final status word */
    const uint64_t Pmax = R_total;
    /* ---- score + per-document term order ---- */
    mark(ctx, S_SCORE);
    ENSURE(ctx->out_term, Pmax * 4 + 4);
    ENSURE(ctx->out_cnt, Pmax * 4 + 4);
    ENSURE(ctx->out_score, Pmax * 8 + 8);
    ENSURE(ctx->idf_rank, (size_t)V * 8 + 8);
    ENSURE(ctx->large_list, (size_t)N * 8 + 16);   /* wide ranks: handed-off documents; then the K5 class list */
    K5Args a{};
    a.order = ctx->order;
    a.meta = ctx->doc_meta.as<uint4>();
    a.out_off = ctx->out_off.as<uint64_t>();
    a.doc_recoff = ctx->doc_recoff.as<uint64_t>();
    a.doc_npairs = ctx->doc_npairs.as<uint32_t>();
    a.doc_size = ctx->doc_size.as<uint32_t>();
    a.doc_flags = ctx->doc_flags.as<uint8_t>();
    a.rec_slot = ctx->rec_slot.as<uint32_t>();
    a.rec_cnt = ctx->rec_cnt.as<uint32_t>();
    a.rank_of_slot = ctx->rank_of_slot.as<uint32_t>();
    a.df_of_rank = df_of_run(ctx);
    a.idf_idx = full_lut ? nullptr : ctx->present.as<uint32_t>();   /* null: idf indexed by df */
    a.idf = ctx->idf_vals.as<double>();
    a.idf_rank = ctx->idf_rank.as<double>();
    /* large V: 4-byte df gathers + the small idf-by-df table instead of 8-byte idf gathers;
     * only with ranks over 21 bits (the score kernels' wide instance: k5_radix and the
     * common instance read idf by rank) */
    a.idf_by_df = (full_lut && V > (1u << 21)) ? 1u : 0u;
    a.large_list = ctx->large_list.as<uint32_t>() + 1;
    a.large_count = ctx->large_list.as<uint32_t>();
    a.cls_nblk = (N + 255) / 256;
    a.cls_list = ctx->large_list.as<uint32_t>() + N + 2;
    ENSURE(ctx->cls_off, ((size_t)3 * a.cls_nblk + 8) * 4);
    a.cls_off = ctx->cls_off.as<uint32_t>();
    {   /* presorted documents over 4096 pairs are emitted in 4096-pair chunks: <= 2 R / 4096 tasks */
        const uint64_t cap_t = 2 * R_total / 4096 + 64;
        ENSURE(ctx->split_tasks, cap_t * 8 + 8);
        a.split_count = ctx->split_tasks.as<uint32_t>();
        a.split_tasks = ctx->split_tasks.as<uint2>() + 1;
        a.split_cap = (uint32_t)(cap_t < 0xFFFFFFFFull ? cap_t : 0xFFFFFFFFull);
    }
    a.ndocs = N;
    a.nterms = V;
    a.rank_bits = V > 1 ? 32u - (uint32_t)__builtin_clz(V - 1) : 1u;
    a.rec_total = R_total;
    a.slot_cap = cap;
    a.status = (uint32_t*)(cnt + 3);
    a.out_term = ctx->out_term.as<uint32_t>();
    a.out_cnt = ctx->out_cnt.as<uint32_t>();
    a.out_score = ctx->out_score.as<double>();
    XCHK(launch_score_order(a, ar, s, ctx->stream2, ctx->ev_fork, ctx->ev_order));
    mark(ctx, S_NSTAGES);
    {   /* the final status, the pair total and (with a transport) global V: one launch */
        WordList wl{};
        wl.src[0] = cnt + 3;
        wl.bytes[0] = 4;
        wl.src[1] = ctx->out_off.as<uint64_t>() + N;
        wl.bytes[1] = 8;
        wl.src[2] = cnt + 12;
        wl.bytes[2] = 4;
        wl.n = ctx->xp ? 3 : 2;
        if (ctx->xp) {
            XCHK(launch_words_to_host(wl, ctx->hpin_dev + 24, s));
            XSYNC(s);
        } else {
            HIPCHK(words_wait(ctx, wl, 24, s));
        }
    }
    ctx->idf_pin_busy = false;   /* the stream has drained */
    const uint32_t st_end = (uint32_t)ctx->hpin[24];
    const uint64_t P = ctx->hpin[25];
    ctx->npairs = P;
    if (ctx->xp) ctx->Vg = (uint32_t)ctx->hpin[26];
    if (st_end & ST_BOUNDS) {
        fprintf(stderr, "tfidf: internal bounds check tripped (status 0x%x)\n", st_end);
        return TFIDF_E_STATE;
    }
    return 0;
}

/* One attempt of the pipeline: local stages, the DF exchange (with an attached
 * transport every rank enters it, whatever its local status, see exchange_df), the
 * stages after it.  Returns 0 on success, 1 to retry with grown capacities (with a
 * transport: decided by all ranks together), <0 on error. */
static int run_once(tfidf_ctx* ctx, const CorpusDev& c, const uint32_t* dev_ids, uint64_t Nt) {
    int rc = run_local(ctx, c, dev_ids, Nt);
    mark(ctx, S_EXCHANGE);
    if (ctx->xp) {
        rc = exchange_df(ctx, rc, ctx->run_V, c.bytes);
        if (rc) return rc;
    } else {
        if (rc) return rc;
        ctx->Vg = ctx->run_V;   /* one rank: the global df is the local one (df_of_run) */
    }
    return run_post(ctx, Nt);
}

/* Host-side preparation of a run: argument checks, the host corpus copied to HBM. */
static int run_prepare(tfidf_ctx* ctx, const tfidf_corpus* in, CorpusDev& c, const uint32_t*& dev_ids, uint64_t& Nt) {
    if (in->ndocs && !in->doc_off) return TFIDF_E_INVAL;
    if (in->nbytes && !in->bytes) return TFIDF_E_INVAL;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint32_t N = in->ndocs;
    const bool dev = (in->flags & TFIDF_CORPUS_DEVICE) != 0;
    dev_ids = nullptr;
    uint64_t lo = 0, hi = 0;
    if (dev) {
        c.bytes = in->bytes;
        c.doc_off = in->doc_off;
        dev_ids = in->doc_ids;
        uint64_t e[2] = {0, 0};
        if (N) {   /* one round trip on the run's stream (after any work already queued on it) */
            HIPCHK(hipMemcpyAsync(ctx->hpin + 12, in->doc_off, 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(ctx->hpin + 13, in->doc_off + N, 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            e[0] = ctx->hpin[12];
            e[1] = ctx->hpin[13];
        }
        lo = e[0]; hi = e[1];
    } else {
        ENSURE(ctx->in_bytes, in->nbytes + 64);
        ENSURE(ctx->in_off, ((size_t)N + 1) * 8);
        if (in->nbytes) HIPCHK(hipMemcpyAsync(ctx->in_bytes.p, in->bytes, in->nbytes, hipMemcpyHostToDevice, s));
        if (N || in->doc_off) HIPCHK(hipMemcpyAsync(ctx->in_off.p, in->doc_off, ((size_t)N + 1) * 8, hipMemcpyHostToDevice, s));
        if (in->doc_ids) {
            ENSURE(ctx->in_ids, (size_t)N * 4 + 4);
            HIPCHK(hipMemcpyAsync(ctx->in_ids.p, in->doc_ids, (size_t)N * 4, hipMemcpyHostToDevice, s));
            dev_ids = ctx->in_ids.as<uint32_t>();
        }
        c.bytes = ctx->in_bytes.as<uint8_t>();
        c.doc_off = ctx->in_off.as<uint64_t>();
        if (N) { lo = in->doc_off[0]; hi = in->doc_off[N]; }
        HIPCHK(hipStreamSynchronize(s));
    }
    if (hi > in->nbytes || lo > hi) return TFIDF_E_INVAL;
    c.nbytes = in->nbytes;
    c.ndocs = N;
    c.lo = lo;
    c.hi = hi;
    Nt = in->ndocs_total ? in->ndocs_total : N;
    if (Nt < N || Nt > 0xFFFFFFFFull) return TFIDF_E_INVAL;
    return TFIDF_OK;
}

extern "C" int tfidf_run(tfidf_ctx* ctx, const tfidf_corpus* in) {
    if (!ctx) return TFIDF_E_INVAL;
    ctx->have_result = false;
    ctx->have_info = false;
    ctx->text_valid = false;
    CorpusDev c{};
    const uint32_t* dev_ids = nullptr;
    uint64_t Nt = 0;
    int rc = in ? run_prepare(ctx, in, c, dev_ids, Nt) : TFIDF_E_INVAL;
    if (rc) {
        /* a rank that fails before its first stage still takes part in the agreement, so
         * its peers return TFIDF_E_PEER instead of waiting for it */
        if (ctx->xp) (void)exchange_agree(ctx, rc, 0, nullptr);
        return rc;
    }
    hipStream_t s = ctx->stream;
    const uint32_t N = in->ndocs;
    IdfJoin idf_guard{ctx};
    rc = idf_start(ctx, Nt);
    if (rc) {
        if (ctx->xp) (void)exchange_agree(ctx, rc, 0, nullptr);
        return rc;
    }
    rc = 1;
    for (int attempt = 0; attempt < 8 && rc == 1; ++attempt) {
        const size_t need = ctx->arena.peak > ctx->arena_buf.cap ? ctx->arena.peak * 2 : ctx->arena_buf.cap;
        const int arc = arena_reset(ctx, need);
        /* with peers, an allocation failure is reported through the agreement as well */
        rc = arc ? arc : run_once(ctx, c, dev_ids, Nt);
        if (arc && ctx->xp) (void)exchange_agree(ctx, arc, 0, nullptr);
        if (rc == 1) {
            HIPCHK(hipStreamSynchronize(s));
            HIPCHK(hipStreamSynchronize(ctx->stream2));
            HIPCHK(hipStreamSynchronize(ctx->stream3));   /* the early idf upload (run_local) */
        }
    }
    if (rc == 1) return TFIDF_E_CAPACITY;
    if (rc) return rc;
    ctx->corpus = *in;
    ctx->run_nbytes = c.hi - c.lo;
    ctx->dev_bytes = c.bytes;
    ctx->dev_ids = dev_ids;
    ctx->ndocs = N;
    ctx->ndocs_total = Nt;
    ctx->have_result = true;
    ctx->have_info = true;
    if (ctx->timing) (void)hipEventSynchronize(ctx->ev[S_NSTAGES]);   /* done on the device; the runtime may not know yet */
    if (ctx->timing == 2) {
        for (int i = 0; i < S_NSTAGES; ++i) ctx->ms_stage[i] = 0;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ctx->ev[S_TOKCOUNT], ctx->ev[S_VOCAB]);
        ctx->ms_stage[S_TOKCOUNT] = ms;
        float tot = 0;
        (void)hipEventElapsedTime(&tot, ctx->ev[S_PREP], ctx->ev[S_NSTAGES]);
        ctx->ms_total = tot;
    } else if (ctx->timing) {
        for (int i = 0; i < S_NSTAGES; ++i) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, ctx->ev[i], ctx->ev[i + 1]);
            ctx->ms_stage[i] = ms;
        }
        float tot = 0;
        (void)hipEventElapsedTime(&tot, ctx->ev[S_PREP], ctx->ev[S_NSTAGES]);
        ctx->ms_total = tot;
    }
    ctx->totals.runs += 1;
    ctx->totals.ms_tokcount += ctx->timing ? ctx->ms_stage[S_TOKCOUNT] : 0.0;
    ctx->totals.ms_total += ctx->timing ? ctx->ms_total : 0.0;
    ctx->totals.idf_logs += ctx->idf_logs;
    ctx->totals.ms_idf_host += ctx->ms_idf_host;
    ctx->totals.ms_idf_wait += ctx->ms_idf_wait;
    return TFIDF_OK;
}

extern "C" int tfidf_run_totals_get(tfidf_ctx* ctx, tfidf_run_totals* out, int reset) {
    if (!ctx || !out) return TFIDF_E_INVAL;
    *out = ctx->totals;
    if (reset) ctx->totals = tfidf_run_totals{};
    return TFIDF_OK;
}

extern "C" int tfidf_debug_k1_stamps(tfidf_ctx* ctx, uint64_t* out, int n) {
    if (!ctx || !out || n <= 0) return TFIDF_E_INVAL;
    if (!ctx->stamps_on || !ctx->stamps.p) return TFIDF_E_STATE;
    int m = n < K1_DEBUG_WORDS ? n : K1_DEBUG_WORDS;
    HIPCHK(hipMemcpy(out, ctx->stamps.p, 8 * (size_t)m, hipMemcpyDeviceToHost));
    return m;
}

/* Measured HBM streaming peaks: `iters` timed passes of a read-only stream
 * over nbytes and of an nbytes copy (counted as 2 x nbytes), after one warm-up pass each;
 * the buffers are allocated for the call and released. */
extern "C" int tfidf_hbm_probe(tfidf_ctx* ctx, uint64_t nbytes, int iters, double* read_gbps, double* copy_gbps) {
    if (!ctx || !read_gbps || !copy_gbps || nbytes < 4096 || iters <= 0) return TFIDF_E_INVAL;
    HIPCHK(hipSetDevice(ctx->device));
    nbytes &= ~(uint64_t)4095;
    hipStream_t s = ctx->stream;
    void *a = nullptr, *b = nullptr;
    uint32_t* sink = nullptr;
    if (tfidf_dev_malloc(&a, nbytes) != hipSuccess) return TFIDF_E_NOMEM;
    if (tfidf_dev_malloc(&b, nbytes) != hipSuccess) { (void)hipFree(a); return TFIDF_E_NOMEM; }
    if (tfidf_dev_malloc((void**)&sink, 256) != hipSuccess) { (void)hipFree(a); (void)hipFree(b); return TFIDF_E_NOMEM; }
    int ncu = 256, dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const unsigned grid = (unsigned)(ncu > 0 ? ncu : 256) * 16u;
    hipEvent_t e0, e1;
    int rc = TFIDF_OK;
    float ms_r = 0.f, ms_c = 0.f;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) rc = TFIDF_E_HIP;
    if (!rc && (hipMemsetAsync(a, 0, nbytes, s) != hipSuccess || hipMemsetAsync(b, 0, nbytes, s) != hipSuccess)) rc = TFIDF_E_HIP;
    if (!rc && (launch_stream_read(a, nbytes, sink, grid, s) || launch_stream_copy(a, b, nbytes, grid, s))) rc = TFIDF_E_HIP;
    if (!rc) {
        bool ok = hipEventRecord(e0, s) == hipSuccess;
        for (int i = 0; ok && i < iters; ++i) ok = launch_stream_read(a, nbytes, sink, grid, s) == 0;
        ok = ok && hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
             hipEventElapsedTime(&ms_r, e0, e1) == hipSuccess;
        ok = ok && hipEventRecord(e0, s) == hipSuccess;
        for (int i = 0; ok && i < iters; ++i) ok = launch_stream_copy(a, b, nbytes, grid, s) == 0;
        ok = ok && hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
             hipEventElapsedTime(&ms_c, e0, e1) == hipSuccess;
        if (!ok) rc = TFIDF_E_HIP;
    }
    if (!rc) {
        *read_gbps = ms_r > 0 ? (double)nbytes * iters / (ms_r * 1e-3) / 1e9 : 0.0;
        *copy_gbps = ms_c > 0 ? 2.0 * (double)nbytes * iters / (ms_c * 1e-3) / 1e9 : 0.0;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamSynchronize(s);
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipFree(sink);
    return rc;
}

extern "C" int tfidf_alloc_stats(uint64_t* allocs, uint64_t* bytes) {
    if (!allocs || !bytes) return TFIDF_E_INVAL;
    *allocs = g_dev_allocs.load(std::memory_order_relaxed);
    *bytes = g_dev_alloc_bytes.load(std::memory_order_relaxed);
    return TFIDF_OK;
}

extern "C" int tfidf_last_run_info(tfidf_ctx* ctx, tfidf_run_info* out) {
    tfidf_run_info* info = out;
    if (!ctx || !info || info->size < 16) return TFIDF_E_INVAL;
    if (!ctx->have_info) return TFIDF_E_STATE;
    const size_t want = info->size < sizeof(tfidf_run_info) ? (size_t)info->size : sizeof(tfidf_run_info);
    tfidf_run_info full;
    memset(&full, 0, sizeof(full));
    info = &full;   /* filled whole here, copied out up to the caller's size below */
    info->nbytes = ctx->run_nbytes;   /* no device round trip: the run read the bounds */
    info->ntokens = ctx->ntokens;
    info->npairs = ctx->npairs;
    info->nterms = ctx->V;
    info->nterms_global = ctx->Vg;
    info->nchunks = ctx->nchunks;
    info->partial_records = ctx->nrec_part;
    info->ndocs = ctx->ndocs;
    info->vocab_capacity = (uint32_t)ctx->vcap;
    info->ms_total = ctx->ms_total;
    info->ms_tokcount = ctx->ms_stage[S_TOKCOUNT];
    for (int i = 0; i < S_NSTAGES; ++i) info->ms_stage[i] = ctx->ms_stage[i];
    info->nstages = S_NSTAGES;
    info->flags = (ctx->k1_vs ? TFIDF_RUN_K1_VS : 0u) | (ctx->k1_sl ? TFIDF_RUN_K1_SL : 0u) |
                  (ctx->xp && ctx->last_dense ? TFIDF_RUN_XCHG_DENSE : 0u);
    info->device_allocs = g_dev_allocs.load(std::memory_order_relaxed);
    info->device_alloc_bytes = g_dev_alloc_bytes.load(std::memory_order_relaxed);
    info->idf_logs = ctx->idf_logs;
    info->ms_idf_host = ctx->ms_idf_host;
    info->ms_idf_wait = ctx->ms_idf_wait;
    full.size = want;
    memcpy(out, &full, want);
    return TFIDF_OK;
}

/* ------------------------------------------------------------------- fetch -- */

extern "C" void tfidf_result_free(tfidf_result* r) {
    if (!r) return;
    free(r->pair_doc); free(r->pair_term); free(r->pair_count); free(r->pair_docsize); free(r->pair_df);
    free(r->pair_score); free(r->doc_id); free(r->doc_size); free(r->term_off); free(r->term_bytes);
    free(r->term_df);
    memset(r, 0, sizeof(*r));
}

extern "C" int tfidf_fetch(tfidf_ctx* ctx, tfidf_result* r) {
    if (!ctx || !r) return TFIDF_E_INVAL;
    if (!ctx->have_result) return TFIDF_E_STATE;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    memset(r, 0, sizeof(*r));
    const uint64_t P = ctx->npairs;
    const uint32_t N = ctx->ndocs, V = ctx->V;
    r->npairs = P;
    r->ndocs = N;
    r->nterms = V;
    r->ndocs_total = ctx->ndocs_total;
    size_t p4 = (size_t)P * 4 + 4;
    r->pair_doc = (uint32_t*)malloc(p4);
    r->pair_term = (uint32_t*)malloc(p4);
    r->pair_count = (uint32_t*)malloc(p4);
    r->pair_docsize = (uint32_t*)malloc(p4);
    r->pair_df = (uint32_t*)malloc(p4);
    r->pair_score = (double*)malloc((size_t)P * 8 + 8);
    r->doc_id = (uint32_t*)malloc((size_t)N * 4 + 4);
    r->doc_size = (uint32_t*)malloc((size_t)N * 4 + 4);
    r->term_df = (uint32_t*)malloc((size_t)V * 4 + 4);
    r->term_off = (uint64_t*)malloc(((size_t)V + 1) * 8);
    if (!r->pair_doc || !r->pair_term || !r->pair_count || !r->pair_docsize || !r->pair_df || !r->pair_score ||
        !r->doc_id || !r->doc_size || !r->term_df || !r->term_off) {
        tfidf_result_free(r);
        return TFIDF_E_NOMEM;
    }
    std::vector<uint32_t> order(N);
    std::vector<uint64_t> ooff((size_t)N + 1);
    if (P) {
        HIPCHK(hipMemcpyAsync(r->pair_term, ctx->out_term.p, P * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(r->pair_count, ctx->out_cnt.p, P * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(r->pair_score, ctx->out_score.p, P * 8, hipMemcpyDeviceToHost, s));
    }
    if (N) {
        HIPCHK(hipMemcpyAsync(r->doc_size, ctx->doc_size.p, (size_t)N * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(order.data(), ctx->order, (size_t)N * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(ooff.data(), ctx->out_off.p, ((size_t)N + 1) * 8, hipMemcpyDeviceToHost, s));
    }
    if (V) HIPCHK(hipMemcpyAsync(r->term_df, df_of_run(ctx), (size_t)V * 4, hipMemcpyDeviceToHost, s));
    /* term strings in rank order */
    std::vector<uint4> keys(V);
    std::vector<uint32_t> sor(V);
    if (V) {
        HIPCHK(hipMemcpyAsync(sor.data(), ctx->slot_of_rank.p, (size_t)V * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        ENSURE(ctx->x_mine, (size_t)V * 16 + 16);
        if (launch_keys_by_rank(ctx->vkeys.as<uint4>(), ctx->slot_of_rank.as<uint32_t>(), V, ctx->x_mine.as<uint4>(), s))
            return TFIDF_E_HIP;
        HIPCHK(hipMemcpyAsync(keys.data(), ctx->x_mine.p, (size_t)V * 16, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    if (ctx->corpus.doc_ids && !(ctx->corpus.flags & TFIDF_CORPUS_DEVICE)) {
        memcpy(r->doc_id, ctx->corpus.doc_ids, (size_t)N * 4);
    } else if (ctx->dev_ids) {
        HIPCHK(hipMemcpy(r->doc_id, ctx->dev_ids, (size_t)N * 4, hipMemcpyDeviceToHost));
    } else {
        for (uint32_t i = 0; i < N; ++i) r->doc_id[i] = i + 1;
    }
    /* per-pair document, docSize and df: expanded from the per-document output order
     * (K5 writes 16 bytes per pair) */
    for (uint32_t j = 0; j < N; ++j) {
        const uint32_t d = order[j];
        const uint32_t id = r->doc_id[d], dsz = r->doc_size[d];
        for (uint64_t q = ooff[j]; q < ooff[j + 1] && q < P; ++q) {
            r->pair_doc[q] = id;
            r->pair_docsize[q] = dsz;
        }
    }
    for (uint64_t q = 0; q < P; ++q) r->pair_df[q] = r->pair_term[q] < V ? r->term_df[r->pair_term[q]] : 0u;
    std::string pool;
    pool.reserve((size_t)V * 8);
    for (uint32_t t = 0; t < V; ++t) {
        r->term_off[t] = pool.size();
        uint64_t lo = ((uint64_t)keys[t].y << 32) | keys[t].x, hi = ((uint64_t)keys[t].w << 32) | keys[t].z;
        if ((hi >> 56) == 0xFFu) {
            uint64_t rep = 0;
            HIPCHK(hipMemcpy(&rep, ctx->vrep.as<uint64_t>() + sor[t], 8, hipMemcpyDeviceToHost));
            uint64_t off = rep & 0xFFFFFFFFFFull, len = rep >> 40;
            std::string w(len, '\0');
            HIPCHK(hipMemcpy(&w[0], ctx->dev_bytes + off, len, hipMemcpyDeviceToHost));
            pool += w;
        } else {
            uint8_t b[16];
            memcpy(b, &lo, 8);
            memcpy(b + 8, &hi, 8);
            int n = 0;
            while (n < 16 && b[n] != 0x09) ++n;
            pool.append((const char*)b, (size_t)n);
        }
    }
    r->term_off[V] = pool.size();
    r->term_bytes = (uint8_t*)malloc(pool.size() + 1);
    if (!r->term_bytes) { tfidf_result_free(r); return TFIDF_E_NOMEM; }
    memcpy(r->term_bytes, pool.data(), pool.size());
    return TFIDF_OK;
}

/* ----------------------------------------------------------------- synthetic -- */

/* ----------------------------------------------------------------- ingest ----
 * ingest.cpp streams input/doc1..N into the context's host-input buffers (§8f row 2). */
int tfidf_ctx_ingest_buffers(tfidf_ctx* ctx, uint64_t nbytes, uint32_t ndocs, uint8_t** dbytes, uint64_t** doff,
                             uint32_t** dids) {
    HIPCHK(hipSetDevice(ctx->device));
    ENSURE(ctx->in_bytes, nbytes + 64);
    ENSURE(ctx->in_off, ((size_t)ndocs + 1) * 8);
    *dbytes = ctx->in_bytes.as<uint8_t>();
    *doff = ctx->in_off.as<uint64_t>();
    if (dids) {
        ENSURE(ctx->in_ids, (size_t)ndocs * 4 + 4);
        *dids = ctx->in_ids.as<uint32_t>();
    }
    return TFIDF_OK;
}

extern "C" int tfidf_synth_device(tfidf_ctx* ctx, uint64_t seed, uint32_t V, uint32_t mode, const double* cdf,
                                  const uint32_t* doc_ids, const uint64_t* ntok, uint32_t ndocs,
                                  uint64_t ndocs_total, tfidf_corpus* out) {
    if (!ctx || !ntok || !out || V == 0 || (mode == SYN_MODE_ZIPF && !cdf)) return TFIDF_E_INVAL;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    std::vector<uint64_t> bf((size_t)ndocs + 1);
    uint64_t nb = 0;
    for (uint32_t i = 0; i < ndocs; ++i) { bf[i] = nb; nb += (ntok[i] + SYN_BLOCK_TOKENS - 1) / SYN_BLOCK_TOKENS; }
    bf[ndocs] = nb;
    ENSURE(ctx->syn_blkfirst, bf.size() * 8);
    ENSURE(ctx->syn_ntok, (size_t)ndocs * 8 + 8);
    ENSURE(ctx->syn_blkbytes, (nb + 1) * 8);
    ENSURE(ctx->syn_off, ((size_t)ndocs + 1) * 8);
    HIPCHK(hipMemcpyAsync(ctx->syn_blkfirst.p, bf.data(), bf.size() * 8, hipMemcpyHostToDevice, s));
    if (ndocs) HIPCHK(hipMemcpyAsync(ctx->syn_ntok.p, ntok, (size_t)ndocs * 8, hipMemcpyHostToDevice, s));
    const uint32_t* dids = nullptr;
    if (doc_ids) {
        ENSURE(ctx->syn_ids, (size_t)ndocs * 4 + 4);
        HIPCHK(hipMemcpyAsync(ctx->syn_ids.p, doc_ids, (size_t)ndocs * 4, hipMemcpyHostToDevice, s));
        dids = ctx->syn_ids.as<uint32_t>();
    }
    const double* dcdf = nullptr;
    if (mode == SYN_MODE_ZIPF) {
        ENSURE(ctx->syn_cdf, (size_t)V * 8);
        HIPCHK(hipMemcpyAsync(ctx->syn_cdf.p, cdf, (size_t)V * 8, hipMemcpyHostToDevice, s));
        dcdf = ctx->syn_cdf.as<double>();
    }
    syn_spec sp;
    tfidf_synth_spec(&sp, seed, V, mode, dcdf);
    if (arena_reset(ctx, ctx->arena_buf.cap) != 0) return TFIDF_E_NOMEM;
    if (launch_synth_bytes(&sp, dids, ctx->syn_ntok.as<uint64_t>(), ctx->syn_blkfirst.as<uint64_t>(), nb, ndocs,
                           ctx->syn_blkbytes.as<uint64_t>(), s))
        return TFIDF_E_HIP;
    if (scan_excl_u64(ctx->syn_blkbytes.as<uint64_t>(), ctx->syn_blkbytes.as<uint64_t>(), nb, ctx->arena, s))
        return TFIDF_E_HIP;
    uint64_t total = 0;
    HIPCHK(hipMemcpyAsync(&total, ctx->syn_blkbytes.as<uint64_t>() + nb, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    ENSURE(ctx->syn_bytes, total + 64);
    if (launch_synth_fill(&sp, dids, ctx->syn_ntok.as<uint64_t>(), ctx->syn_blkfirst.as<uint64_t>(), nb, ndocs,
                          ctx->syn_blkbytes.as<uint64_t>(), ctx->syn_bytes.as<uint8_t>(), ctx->syn_off.as<uint64_t>(), s))
        return TFIDF_E_HIP;
    HIPCHK(hipStreamSynchronize(s));
    memset(out, 0, sizeof(*out));
    out->bytes = ctx->syn_bytes.as<uint8_t>();
    out->nbytes = total;
    out->doc_off = ctx->syn_off.as<uint64_t>();
    out->doc_ids = dids;
    out->ndocs = ndocs;
    out->flags = TFIDF_CORPUS_DEVICE;
    out->ndocs_total = ndocs_total ? ndocs_total : ndocs;
    return TFIDF_OK;
}

/* ------------------------------------------------------------ emission (GPU) ----
 * the "docN@word\t%.16f\n" lines (TFIDF.c:245,281) formatted in HBM
 * by emit.hip (exact round-half-even %.16f), then copied out / written to output.txt
 * (TFIDF.c:274-282). */
/* the length pass: term metadata, bytes per output position, their scan (doc_toff) and
 * the text buffer sized to the total (one synchronisation for the total) */
static int format_prepare(tfidf_ctx* ctx, EmitLaunch& e, uint64_t& total) {
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint32_t N = ctx->ndocs, V = ctx->V;
    unsigned long long* cnt = ctx->counters.as<unsigned long long>();
    uint32_t* status = (uint32_t*)(cnt + 3);
    HIPCHK(hipMemsetAsync(status, 0, 4, s));
    ENSURE(ctx->t_key, (size_t)V * 16 + 16);
    ENSURE(ctx->t_len, (size_t)V * 4 + 4);
    ENSURE(ctx->doc_tbytes, ((size_t)N + 1) * 8);
    ENSURE(ctx->doc_toff, ((size_t)N + 1) * 8);
    if (launch_term_meta(ctx->vkeys.as<uint4>(), ctx->vrep.as<uint64_t>(), ctx->slot_of_rank.as<uint32_t>(), V,
                         ctx->t_key.as<uint4>(), ctx->t_len.as<uint32_t>(), s))
        return TFIDF_E_HIP;
    e = EmitLaunch{ctx->order, ctx->dev_ids, ctx->out_off.as<uint64_t>(), ctx->out_term.as<uint32_t>(),
                   ctx->out_score.as<double>(), ctx->t_key.as<uint4>(), ctx->t_len.as<uint32_t>(), ctx->dev_bytes, N,
                   status};
    total = 0;
    if (N) {
        if (launch_emit_bytes(e, ctx->doc_tbytes.as<uint64_t>(), s)) return TFIDF_E_HIP;
        ctx->arena.used = 0;
        if (scan_excl_u64(ctx->doc_tbytes.as<uint64_t>(), ctx->doc_toff.as<uint64_t>(), N, ctx->arena, s))
            return TFIDF_E_HIP;
        HIPCHK(hipMemcpyAsync(&ctx->hpin[20], ctx->doc_toff.as<uint64_t>() + N, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        total = ctx->hpin[20];
    }
    ENSURE(ctx->text, total + 64);
    return TFIDF_OK;
}

/* the formatter's status after its launches (the stream is synchronised by the caller) */
static int format_finish(tfidf_ctx* ctx, uint64_t total) {
    uint32_t* status = (uint32_t*)(ctx->counters.as<unsigned long long>() + 3);
    ctx->hpin[21] = 0;
    HIPCHK(hipMemcpyAsync(&ctx->hpin[21], status, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if ((uint32_t)ctx->hpin[21] & ST_BOUNDS) {
        fprintf(stderr, "tfidf: score outside the %%.16f formatter's range\n");
        return TFIDF_E_STATE;
    }
    ctx->text_bytes = total;
    ctx->text_valid = true;
    return TFIDF_OK;
}

extern "C" int tfidf_format(tfidf_ctx* ctx, uint64_t* nbytes) {
    if (!ctx || !nbytes) return TFIDF_E_INVAL;
    if (!ctx->have_result) return TFIDF_E_STATE;
    if (ctx->text_valid) { *nbytes = ctx->text_bytes; return TFIDF_OK; }
    EmitLaunch e{};
    uint64_t total = 0;
    int rc = format_prepare(ctx, e, total);
    if (rc) return rc;
    if (total && launch_emit_write(e, ctx->doc_toff.as<uint64_t>(), ctx->text.as<uint8_t>(), ctx->stream))
        return TFIDF_E_HIP;
    rc = format_finish(ctx, total);
    if (!rc) *nbytes = total;
    return rc;
}

extern "C" int tfidf_copy_text(tfidf_ctx* ctx, uint64_t off, void* dst, uint64_t n) {
    if (!ctx || (n && !dst)) return TFIDF_E_INVAL;
    if (!ctx->text_valid) return TFIDF_E_STATE;
    if (off > ctx->text_bytes || n > ctx->text_bytes - off) return TFIDF_E_INVAL;
    if (!n) return TFIDF_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemcpy(dst, ctx->text.as<uint8_t>() + off, n, hipMemcpyDeviceToHost));
    return TFIDF_OK;
}

/* output.txt (TFIDF.c:274-282): the text leaves HBM through a ring of WR_NBUF pinned
 * 16 MB staging buffers owned by the context (allocated on first use and kept: pinning
 * 128 MB costs ~20 ms per call).  The copies run on stream2 while the host writes the
 * buffers already copied; when the text is not yet formatted, the formatter runs in
 * WR_GROUPS document groups on the main stream and each copy waits only for the group
 * that holds its last byte, so formatting of group g+1 overlaps the copy of group g. */
static int wr_ring_init(tfidf_ctx* ctx) {
    if (ctx->wr_buf[0]) return TFIDF_OK;
    for (int i = 0; i < WR_NBUF; ++i) {
        if (hipHostMalloc((void**)&ctx->wr_buf[i], WR_BUF, hipHostMallocDefault) != hipSuccess) {
            ctx->wr_buf[i] = nullptr;
            for (int j = 0; j < i; ++j) { (void)hipHostFree(ctx->wr_buf[j]); ctx->wr_buf[j] = nullptr; }
            return TFIDF_E_NOMEM;
        }
    }
    for (int i = 0; i < WR_NBUF; ++i) HIPCHK(hipEventCreateWithFlags(&ctx->wr_ev[i], hipEventDisableTiming));
    for (int i = 0; i < WR_GROUPS; ++i) HIPCHK(hipEventCreateWithFlags(&ctx->wr_fmt[i], hipEventDisableTiming));
    return TFIDF_OK;
}

static double now_ms() {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

extern "C" int tfidf_write_output_gpu(tfidf_ctx* ctx, const char* path, int append) {
    if (!ctx || !path) return TFIDF_E_INVAL;
    if (!ctx->have_result) return TFIDF_E_STATE;
    const double t0 = now_ms();
    tfidf_output_info oi{};
    oi.size = sizeof(oi);
    HIPCHK(hipSetDevice(ctx->device));
    int rc = wr_ring_init(ctx);
    if (rc) return rc;
    hipStream_t s = ctx->stream, cs = ctx->stream2;
    const uint32_t N = ctx->ndocs;
    uint64_t total = ctx->text_bytes;
    /* group g covers output positions [N g / ng, N (g+1) / ng) and text bytes [gb[g], gb[g+1]) */
    uint64_t gb[WR_GROUPS + 1];
    int ng = 0;
    const bool fmt = !ctx->text_valid;
    if (fmt) {
        EmitLaunch e{};
        rc = format_prepare(ctx, e, total);
        if (rc) return rc;
        ng = N ? (N < WR_GROUPS ? (int)N : WR_GROUPS) : 0;
        std::vector<uint64_t> toff((size_t)N + 1);
        if (N) HIPCHK(hipMemcpy(toff.data(), ctx->doc_toff.p, ((size_t)N + 1) * 8, hipMemcpyDeviceToHost));
        for (int g = 0; g < ng; ++g) {
            const uint32_t d0 = (uint32_t)((uint64_t)N * g / ng), d1 = (uint32_t)((uint64_t)N * (g + 1) / ng);
            gb[g] = toff[d0];
            gb[g + 1] = toff[d1];
            if (launch_emit_write(e, ctx->doc_toff.as<uint64_t>(), ctx->text.as<uint8_t>(), s, d0, d1))
                return TFIDF_E_HIP;
            HIPCHK(hipEventRecord(ctx->wr_fmt[g], s));
        }
        oi.formatted = 1;
    }
    const double t_prep = now_ms();
    oi.ms_prepare = fmt ? t_prep - t0 : 0.0;
    const int fd = open(path, O_WRONLY | O_CREAT | (append ? 0 : O_TRUNC), 0644);
    if (fd < 0) { (void)hipStreamSynchronize(s); return TFIDF_E_OUTPUT; }
    struct stat fst;
    const bool regular = fstat(fd, &fst) == 0 && S_ISREG(fst.st_mode);
    /* a regular file: blocks written at their offsets by WR_WRITERS threads (page-cache
     * copies in parallel); anything else (a pipe, /dev/null): one thread, in order */
    const uint64_t base = append && regular ? (uint64_t)fst.st_size : 0;
    if (!regular && append) (void)lseek(fd, 0, SEEK_END);
    const uint8_t* src = ctx->text.as<uint8_t>();
    const uint64_t nblk = (total + WR_BUF - 1) / WR_BUF;
    const int nw = regular ? (nblk < (uint64_t)WR_WRITERS ? (int)(nblk ? nblk : 1) : WR_WRITERS) : 1;
    oi.writers = (uint32_t)nw;
    std::mutex mu;
    std::condition_variable cv;
    uint64_t issued = 0;             /* blocks whose copies were sent */
    uint64_t freed[WR_NBUF] = {0};   /* per ring buffer: blocks it has finished (written) */
    bool failed = false;
    int wrc = TFIDF_OK;
    double t_last_copy = t_prep, write_ms = 0.0;
    auto blk_n = [&](uint64_t k) { return (k + 1) * WR_BUF <= total ? WR_BUF : total - k * WR_BUF; };
    /* writer w takes blocks k = w, w + nw, ...: waits for the copy, writes, frees the buffer */
    auto writer = [&](int w) {
        double my_write = 0.0, my_last = 0.0;
        for (uint64_t k = (uint64_t)w; k < nblk; k += (uint64_t)nw) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return issued > k || failed; });
                if (failed) break;
            }
            const int b = (int)(k % WR_NBUF);
            bool ok = hipEventSynchronize(ctx->wr_ev[b]) == hipSuccess;
            const double tc = now_ms();
            my_last = tc > my_last ? tc : my_last;
            const uint64_t n = blk_n(k);
            uint64_t done = 0;
            while (ok && done < n) {
                const ssize_t r = regular ? pwrite(fd, ctx->wr_buf[b] + done, n - done, (off_t)(base + k * WR_BUF + done))
                                          : write(fd, ctx->wr_buf[b] + done, n - done);
                if (r <= 0) { ok = false; break; }
                done += (uint64_t)r;
            }
            my_write += now_ms() - tc;
            std::lock_guard<std::mutex> lk(mu);
            if (!ok) {
                failed = true;
                if (!wrc) wrc = done < n ? TFIDF_E_OUTPUT : TFIDF_E_HIP;
            }
            freed[b] = k + 1;
            cv.notify_all();
            if (failed) break;
        }
        std::lock_guard<std::mutex> lk(mu);
        write_ms += my_write;
        if (my_last > t_last_copy) t_last_copy = my_last;
    };
    std::vector<std::thread> th;
    for (int w = 1; w < nw; ++w) th.emplace_back(writer, w);
    /* issue: block k reuses ring buffer k % WR_NBUF once block k - WR_NBUF is written; its
     * copy waits (on the copy stream) for every format group holding one of its bytes */
    std::thread issuer([&] {
        (void)hipSetDevice(ctx->device);
        int gwait = 0;
        for (uint64_t k = 0; k < nblk; ++k) {
            const int b = (int)(k % WR_NBUF);
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return k < WR_NBUF || freed[b] >= k - WR_NBUF + 1 || failed; });
                if (failed) return;
            }
            const uint64_t b0 = k * WR_BUF, n = blk_n(k);
            bool ok = true;
            while (fmt && gwait < ng && gb[gwait] < b0 + n) {
                if (hipStreamWaitEvent(cs, ctx->wr_fmt[gwait], 0) != hipSuccess) ok = false;
                ++gwait;
            }
            if (ok && (hipMemcpyAsync(ctx->wr_buf[b], src + b0, n, hipMemcpyDeviceToHost, cs) != hipSuccess ||
                       hipEventRecord(ctx->wr_ev[b], cs) != hipSuccess))
                ok = false;
            std::lock_guard<std::mutex> lk(mu);
            if (!ok) { failed = true; if (!wrc) wrc = TFIDF_E_HIP; }
            else issued = k + 1;
            cv.notify_all();
            if (failed) return;
        }
    });
    (void)hipSetDevice(ctx->device);
    writer(0);
    issuer.join();
    for (auto& t : th) t.join();
    (void)hipStreamSynchronize(cs);
    rc = wrc;
    if (fmt) {
        const int r2 = format_finish(ctx, total);   /* synchronises the main stream */
        if (!rc) rc = r2;
        /* a formatting error (a score outside the %.16f range: ST_BOUNDS) found after the
         * blocks were written: no complete-looking file is left behind — the file (or the
         * appended shard) is cut back to where this call started */
        if (r2 && regular) (void)!ftruncate(fd, (off_t)base);
    }
    if (close(fd) != 0 && !rc) rc = TFIDF_E_OUTPUT;
    oi.text_bytes = total;
    oi.ms_d2h_busy = nblk ? t_last_copy - t_prep : 0.0;
    oi.ms_write = write_ms;
    oi.ms_total = now_ms() - t0;
    ctx->out_info = oi;
    return rc;
}

extern "C" int tfidf_last_output_info(const tfidf_ctx* ctx, tfidf_output_info* info) {
    if (!ctx || !info || info->size < sizeof(uint64_t)) return TFIDF_E_INVAL;
    const uint64_t n = info->size < sizeof(tfidf_output_info) ? info->size : sizeof(tfidf_output_info);
    tfidf_output_info o = ctx->out_info;
    o.size = n;
    memcpy(info, &o, (size_t)n);
    return TFIDF_OK;
}

extern "C" int tfidf_format_f64(tfidf_ctx* ctx, const double* vals, uint64_t n, char* out) {
    if (!ctx || (n && (!vals || !out))) return TFIDF_E_INVAL;
    if (!n) return TFIDF_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    DevBuf v, o;
    if (v.ensure(n * 8) || o.ensure(n * 32)) { v.release(); o.release(); return TFIDF_E_NOMEM; }
    unsigned long long* cnt = ctx->counters.as<unsigned long long>();
    uint32_t* status = (uint32_t*)(cnt + 3);
    uint32_t st = 0;
    int rc = TFIDF_OK;
    if (hipMemsetAsync(status, 0, 4, s) != hipSuccess ||
        hipMemcpyAsync(v.p, vals, n * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        launch_format_f64(v.as<double>(), n, o.as<uint8_t>(), status, s) ||
        hipMemcpyAsync(out, o.p, n * 32, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(&st, status, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        rc = TFIDF_E_HIP;
    v.release();
    o.release();
    if (!rc && (st & ST_BOUNDS)) rc = TFIDF_E_INVAL;
    return rc;
}
