/*
 * tfidf_main.c — `tfidf`, the drop-in for the reference program's process contract.
 *
 * Run with no arguments in a directory holding input/doc1..docN: writes ./output.txt with
 * one "docN@word\t%.16f" line per (document, word) in strcmp order, exactly as
 * `mpirun -np P ./TFIDF` does (TFIDF.c:52-287).  Messages and exit codes follow the
 * reference: "Directory failed to open" -> 1 (TFIDF.c:100-103), "Error Opening File: ..."
 * -> 0 (TFIDF.c:134-138, 274-278), an empty input/ -> "More workers than input files!
 * Exiting." (TFIDF.c:120-123, as with -np 2).  --debug-jobs prints the TF Job / IDF Job
 * blocks (TFIDF.c:199-205, 236-239); --stats prints one JSON line of ingest / run / output
 * times to stderr.  input/ is streamed into HBM by tfidf_ingest_dir_device (host reads
 * overlapped with the H2D copies).  The work runs on the GPU through libtfidf_hip.so;
 * there is no CPU path.
 */
#include <dirent.h>
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

int main(int argc, char** argv) {
    int debug = 0, stats = 0, device = 0;
    const char* indir = "input";
    const char* outpath = "output.txt";
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--debug-jobs")) debug = 1;
        else if (!strcmp(argv[i], "--stats")) stats = 1;
        else if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--input") && i + 1 < argc) indir = argv[++i];
        else if (!strcmp(argv[i], "--output") && i + 1 < argc) outpath = argv[++i];
        else {
            fprintf(stderr, "usage: tfidf [--debug-jobs] [--stats] [--device D] [--input DIR] [--output FILE]\n");
            return 2;
        }
    }
    /* TFIDF.c:100-103 before anything touches the GPU */
    DIR* d = opendir(indir);
    if (!d) { printf("Directory failed to open\n"); return 1; }
    closedir(d);
    tfidf_ctx* ctx = NULL;
    int rc = tfidf_open(device, &ctx);
    if (rc) { fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc)); return 3; }
    /* input/doc1..N streamed into HBM through pinned segments (TFIDF.c:98-110,130-147) */
    tfidf_corpus c;
    tfidf_ingest_info ii;
    uint32_t bad = 0;
    rc = tfidf_ingest_dir_device(ctx, indir, 0, &c, &bad, &ii);
    if (rc == TFIDF_E_NOINPUT) { printf("Directory failed to open\n"); tfidf_close(ctx); return 1; }
    if (rc == TFIDF_E_NODOC) {
        printf("Error Opening File: %s/doc%u, rank = %d, i=%u, numDocs= %u\n", indir, bad, 1, bad, c.ndocs);
        tfidf_close(ctx);
        return 0;
    }
    if (rc) { fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc)); tfidf_close(ctx); return 3; }
    if (c.ndocs == 0) { printf("More workers than input files! Exiting.\n"); tfidf_close(ctx); return 0; }
    rc = tfidf_run(ctx, &c);
    if (rc) { fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc)); tfidf_close(ctx); return 3; }
    if (debug) {
        tfidf_result r;
        rc = tfidf_fetch(ctx, &r);
        if (rc) { fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc)); tfidf_close(ctx); return 3; }
        tfidf_print_jobs(&r);
        tfidf_result_free(&r);
    }
    tfidf_run_info ri;
    double t_out = 0;
    if (stats) { tfidf_last_run_info(ctx, &ri); t_out = wall_ms(); }
    /* lines formatted on the GPU, copied out through pinned buffers (TFIDF.c:245,274-282) */
    rc = tfidf_write_output_gpu(ctx, outpath, 0);
    if (rc == TFIDF_E_OUTPUT) printf("Error Opening File: %s\n", outpath);
    else if (rc) { fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc)); tfidf_close(ctx); return 3; }
    if (stats)
        fprintf(stderr,
                "{\"docs\": %u, \"corpus_bytes\": %llu, \"ingest_threads\": %u, \"ingest_scan_ms\": %.3f, "
                "\"ingest_read_h2d_ms\": %.3f, \"ingest_GBps\": %.3f, \"run_device_ms\": %.3f, \"pairs\": %llu, "
                "\"output_ms\": %.3f}\n",
                ii.ndocs, (unsigned long long)ii.nbytes, ii.threads, ii.ms_scan, ii.ms_read,
                ii.ms_total > 0 ? ii.nbytes / ii.ms_total / 1e6 : 0.0, ri.ms_total, (unsigned long long)ri.npairs,
                wall_ms() - t_out);
    tfidf_close(ctx);
    return 0;
}
