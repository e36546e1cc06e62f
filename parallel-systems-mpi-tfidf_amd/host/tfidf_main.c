/*
 * tfidf_main.c — `tfidf`, the drop-in for the reference program's process contract.
 *
 * Run with no arguments in a directory holding input/doc1..docN: writes ./output.txt with
 * one "docN@word\t%.16f" line per (document, word) in strcmp order, exactly as
 * `mpirun -np P ./TFIDF` does (TFIDF.c:52-287).  Messages and exit codes follow the
 * reference: "Directory failed to open" -> 1 (TFIDF.c:100-103), "Error Opening File: ..."
 * -> 0 (TFIDF.c:134-138, 274-278), an empty input/ -> "More workers than input files!
 * Exiting." (TFIDF.c:120-123, as with -np 2).  --debug-jobs prints the TF Job / IDF Job
 * blocks (TFIDF.c:199-205, 236-239), one pair of blocks per shard (the reference prints
 * one per rank); --stats prints one JSON line of ingest / run / output times to stderr.
 *
 * Parallelism (the reference's `mpirun -np P`, TFIDF.c:82-92,125-130):
 *   --gpus N     GPUs to use (default 1; capped at the visible GPUs), one shard each;
 *   --shards K   shards (default: N), dealt to the GPUs round-robin — more shards than
 *                GPUs run through the in-process transport (tests on one GPU).
 * Shards are byte-balanced contiguous ranges of the "docN@" order (tfidf_plan_dir), never
 * more than N documents; their outputs are concatenated in shard order.  One shard
 * streams input/ straight into HBM (tfidf_ingest_dir_device).  The work runs on the GPU
 * through libtfidf_hip.so; there is no CPU path.
 */
#include <dirent.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/tfidf.h"

static double wall_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

static int fail(int rc) {
    fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc));
    return 3;
}

/* TFIDF.c:134-138 */
static int missing_doc(const char* indir, uint32_t bad, uint32_t ndocs) {
    printf("Error Opening File: %s/doc%u, rank = %d, i=%u, numDocs= %u\n", indir, bad, 1, bad, ndocs);
    return 0;
}

/* --debug-jobs: the TF Job / IDF Job blocks of one shard (TFIDF.c:199-205,236-239) */
static int debug_jobs(tfidf_ctx* ctx) {
    tfidf_result r;
    int rc = tfidf_fetch(ctx, &r);
    if (rc) return rc;
    tfidf_print_jobs(&r);
    tfidf_result_free(&r);
    return TFIDF_OK;
}

/* ------------------------------------------------------------- one shard -- */

static int run_single(int device, const char* indir, const char* outpath, int debug, int stats) {
    tfidf_ctx* ctx = NULL;
    int rc = tfidf_open(device, &ctx);
    if (rc) return fail(rc);
    /* input/doc1..N streamed into HBM through pinned segments (TFIDF.c:98-110,130-147) */
    tfidf_corpus c;
    tfidf_ingest_info ii;
    uint32_t bad = 0;
    rc = tfidf_ingest_dir_device(ctx, indir, 0, &c, &bad, &ii);
    if (rc == TFIDF_E_NOINPUT) { printf("Directory failed to open\n"); tfidf_close(ctx); return 1; }
    if (rc == TFIDF_E_NODOC) { tfidf_close(ctx); return missing_doc(indir, bad, c.ndocs); }
    if (rc) { tfidf_close(ctx); return fail(rc); }
    if (c.ndocs == 0) { printf("More workers than input files! Exiting.\n"); tfidf_close(ctx); return 0; }
    rc = tfidf_run(ctx, &c);
    if (!rc && debug) rc = debug_jobs(ctx);
    if (rc) { tfidf_close(ctx); return fail(rc); }
    tfidf_run_info ri;
    ri.size = sizeof(ri);
    double t_out = 0;
    if (stats) { tfidf_last_run_info(ctx, &ri); t_out = wall_ms(); }
    /* lines formatted on the GPU, copied out through pinned buffers (TFIDF.c:245,274-282) */
    rc = tfidf_write_output_gpu(ctx, outpath, 0);
    if (rc == TFIDF_E_OUTPUT) printf("Error Opening File: %s\n", outpath);
    else if (rc) { tfidf_close(ctx); return fail(rc); }
    if (stats) {
        const double out_ms = wall_ms() - t_out;
        tfidf_output_info oi;
        memset(&oi, 0, sizeof(oi));
        oi.size = sizeof(oi);
        (void)tfidf_last_output_info(ctx, &oi);
        fprintf(stderr,
                "{\"docs\": %u, \"corpus_bytes\": %llu, \"shards\": 1, \"ingest_threads\": %u, \"ingest_scan_ms\": %.3f, "
                "\"ingest_read_h2d_ms\": %.3f, \"ingest_GBps\": %.3f, \"run_device_ms\": %.3f, \"pairs\": %llu, "
                "\"output_ms\": %.3f, \"output_bytes\": %llu, \"output_format_prepare_ms\": %.3f, "
                "\"output_d2h_busy_ms\": %.3f, \"output_write_thread_ms\": %.3f, \"output_writers\": %u}\n",
                ii.ndocs, (unsigned long long)ii.nbytes, ii.threads, ii.ms_scan, ii.ms_read,
                ii.ms_total > 0 ? ii.nbytes / ii.ms_total / 1e6 : 0.0, ri.ms_total, (unsigned long long)ri.npairs,
                out_ms, (unsigned long long)oi.text_bytes, oi.ms_prepare, oi.ms_d2h_busy, oi.ms_write, oi.writers);
    }
    tfidf_close(ctx);
    return 0;
}

/* ------------------------------------------------------------ K shards -- */

struct shard_job {
    tfidf_group* g;
    const tfidf_dir_plan* plan;
    const char* indir;
    uint32_t shard;
    tfidf_corpus corpus;
    uint32_t bad;
    int rc;
};

static void* ingest_job(void* arg) {
    struct shard_job* j = (struct shard_job*)arg;
    j->bad = 0;
    /* each rank's reader pool gets a share of the host threads */
    const int threads = 4;
    j->rc = tfidf_ingest_shard_device(tfidf_group_ctx(j->g, (int)j->shard), j->indir, j->plan, j->shard, threads,
                                      &j->corpus, &j->bad, NULL);
    return NULL;
}

static int run_sharded(int ngpus, int nshards, const char* indir, const char* outpath, int debug, int stats) {
    const double t0 = wall_ms();
    tfidf_dir_plan plan;
    uint32_t bad = 0;
    int rc = tfidf_plan_dir(indir, (uint32_t)nshards, 0, &plan, &bad);
    if (rc == TFIDF_E_NOINPUT) { printf("Directory failed to open\n"); return 1; }
    if (rc == TFIDF_E_NODOC) return missing_doc(indir, bad, plan.ndocs);
    if (rc) return fail(rc);
    if (plan.ndocs == 0) { printf("More workers than input files! Exiting.\n"); tfidf_plan_free(&plan); return 0; }
    if (plan.ndocs < (uint32_t)nshards) {   /* idle GPUs are simply not used */
        nshards = (int)plan.ndocs;
        tfidf_plan_free(&plan);
        rc = tfidf_plan_dir(indir, (uint32_t)nshards, 0, &plan, &bad);
        if (rc == TFIDF_E_NODOC) return missing_doc(indir, bad, plan.ndocs);
        if (rc) return fail(rc);
    }
    int* dev = (int*)malloc(sizeof(int) * (size_t)nshards);
    struct shard_job* jobs = (struct shard_job*)calloc((size_t)nshards, sizeof(struct shard_job));
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nshards);
    tfidf_corpus* cs = (tfidf_corpus*)calloc((size_t)nshards, sizeof(tfidf_corpus));
    if (!dev || !jobs || !th || !cs) { tfidf_plan_free(&plan); return fail(TFIDF_E_NOMEM); }
    for (int r = 0; r < nshards; ++r) dev[r] = r % ngpus;
    tfidf_group* g = NULL;
    rc = tfidf_group_open(nshards, dev, 0, &g);
    if (rc) { tfidf_plan_free(&plan); return fail(rc); }
    const double t_open = wall_ms();
    /* every shard streams its documents into its GPU at once */
    for (int r = 0; r < nshards; ++r) {
        jobs[r].g = g;
        jobs[r].plan = &plan;
        jobs[r].indir = indir;
        jobs[r].shard = (uint32_t)r;
        pthread_create(&th[r], NULL, ingest_job, &jobs[r]);
    }
    for (int r = 0; r < nshards; ++r) pthread_join(th[r], NULL);
    uint32_t worst_bad = 0;
    for (int r = 0; r < nshards; ++r) {
        if (jobs[r].rc == TFIDF_E_NODOC && (worst_bad == 0 || jobs[r].bad < worst_bad)) worst_bad = jobs[r].bad;
        else if (jobs[r].rc && !rc) rc = jobs[r].rc;
        cs[r] = jobs[r].corpus;
    }
    if (worst_bad) {
        const uint32_t n = plan.ndocs;
        tfidf_group_close(g);
        tfidf_plan_free(&plan);
        return missing_doc(indir, worst_bad, n);
    }
    const double t_ingest = wall_ms();
    if (!rc) rc = tfidf_group_run(g, cs);
    for (int r = 0; r < nshards && !rc && debug; ++r) rc = debug_jobs(tfidf_group_ctx(g, r));
    if (rc) { tfidf_group_close(g); tfidf_plan_free(&plan); return fail(rc); }
    const double t_run = wall_ms();
    /* each GPU formats its shard; the texts are written in shard order (TFIDF.c:253-282) */
    rc = tfidf_group_write_output(g, outpath);
    if (rc == TFIDF_E_OUTPUT) printf("Error Opening File: %s\n", outpath);
    else if (rc) { tfidf_group_close(g); tfidf_plan_free(&plan); return fail(rc); }
    if (stats) {
        uint64_t pairs = 0, bytes = 0;
        for (int r = 0; r < nshards; ++r) {
            tfidf_run_info ri;
            ri.size = sizeof(ri);
            if (tfidf_last_run_info(tfidf_group_ctx(g, r), &ri) == 0) pairs += ri.npairs;
            bytes += plan.shard_bytes[r];
        }
        fprintf(stderr,
                "{\"docs\": %u, \"corpus_bytes\": %llu, \"shards\": %d, \"gpus\": %d, \"plan_open_ms\": %.3f, "
                "\"ingest_ms\": %.3f, \"run_ms\": %.3f, \"pairs\": %llu, \"output_ms\": %.3f}\n",
                plan.ndocs, (unsigned long long)bytes, nshards, ngpus, t_open - t0, t_ingest - t_open, t_run - t_ingest,
                (unsigned long long)pairs, wall_ms() - t_run);
    }
    tfidf_group_close(g);
    tfidf_plan_free(&plan);
    free(dev);
    free(jobs);
    free(th);
    free(cs);
    return 0;
}

int main(int argc, char** argv) {
    int debug = 0, stats = 0, device = -1, ngpus = 0, nshards = 0;
    const char* indir = "input";
    const char* outpath = "output.txt";
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--debug-jobs")) debug = 1;
        else if (!strcmp(argv[i], "--stats")) stats = 1;
        else if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--gpus") && i + 1 < argc) ngpus = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--shards") && i + 1 < argc) nshards = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--input") && i + 1 < argc) indir = argv[++i];
        else if (!strcmp(argv[i], "--output") && i + 1 < argc) outpath = argv[++i];
        else {
            fprintf(stderr, "usage: tfidf [--debug-jobs] [--stats] [--gpus N] [--shards K] [--device D] "
                            "[--input DIR] [--output FILE]\n");
            return 2;
        }
    }
    /* TFIDF.c:100-103 before anything touches the GPU */
    DIR* d = opendir(indir);
    if (!d) { printf("Directory failed to open\n"); return 1; }
    closedir(d);
    const int visible = tfidf_device_count();
    if (visible <= 0) return fail(TFIDF_E_NODEV);
    if (device >= 0) ngpus = 1;                 /* --device D: one GPU, that one */
    /* default: ONE GPU.  Several GPUs (an RCCL clique over xGMI) only when asked for with
     * --gpus N: the multi-GPU path is validated on the driver's 8-GPU node, not here */
    if (ngpus <= 0) ngpus = 1;
    if (ngpus > visible) ngpus = visible;
    if (nshards <= 0) nshards = ngpus;
    if (nshards == 1) return run_single(device >= 0 ? device : 0, indir, outpath, debug, stats);
    if (device > 0) return fail(TFIDF_E_INVAL);   /* several shards use devices 0..N-1 */
    return run_sharded(ngpus, nshards, indir, outpath, debug, stats);
}
