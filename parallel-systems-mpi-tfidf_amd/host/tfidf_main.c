/*
 * tfidf_main.c — `tfidf`, the drop-in for the reference program's process contract.
 *
 * Run with no arguments in a directory holding input/doc1..docN: writes ./output.txt with
 * one "docN@word\t%.16f" line per (document, word) in strcmp order, exactly as
 * `mpirun -np P ./TFIDF` does (TFIDF.c:52-287).  Messages and exit codes follow the
 * reference: "Directory failed to open" -> 1 (TFIDF.c:100-103), "Error Opening File: ..."
 * -> 0 (TFIDF.c:134-138, 274-278), an empty input/ -> "More workers than input files!
 * Exiting." (TFIDF.c:120-123, as with -np 2).  --debug-jobs prints the TF Job / IDF Job
 * blocks (TFIDF.c:199-205, 236-239).  The work runs on the GPU through libtfidf_hip.so;
 * there is no CPU path.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/tfidf.h"

int main(int argc, char** argv) {
    int debug = 0, device = 0;
    const char* indir = "input";
    const char* outpath = "output.txt";
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--debug-jobs")) debug = 1;
        else if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--input") && i + 1 < argc) indir = argv[++i];
        else if (!strcmp(argv[i], "--output") && i + 1 < argc) outpath = argv[++i];
        else {
            fprintf(stderr, "usage: tfidf [--debug-jobs] [--device D] [--input DIR] [--output FILE]\n");
            return 2;
        }
    }
    uint8_t* bytes = NULL;
    uint64_t nbytes = 0, *doc_off = NULL;
    uint32_t ndocs = 0, bad = 0;
    int rc = tfidf_ingest_dir(indir, &bytes, &nbytes, &doc_off, &ndocs, &bad);
    if (rc == TFIDF_E_NOINPUT) { printf("Directory failed to open\n"); return 1; }
    if (rc == TFIDF_E_NODOC) {
        printf("Error Opening File: %s/doc%u, rank = %d, i=%u, numDocs= %u\n", indir, bad, 1, bad, ndocs);
        return 0;
    }
    if (rc) { fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc)); return 3; }
    if (ndocs == 0) { printf("More workers than input files! Exiting.\n"); return 0; }
    tfidf_ctx* ctx = NULL;
    rc = tfidf_open(device, &ctx);
    if (rc) { fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc)); return 3; }
    tfidf_corpus c;
    memset(&c, 0, sizeof c);
    c.bytes = bytes;
    c.nbytes = nbytes;
    c.doc_off = doc_off;
    c.ndocs = ndocs;
    c.ndocs_total = ndocs;
    rc = tfidf_run(ctx, &c);
    if (rc) { fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc)); tfidf_close(ctx); return 3; }
    if (debug) {
        tfidf_result r;
        rc = tfidf_fetch(ctx, &r);
        if (rc) { fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc)); tfidf_close(ctx); return 3; }
        tfidf_print_jobs(&r);
        tfidf_result_free(&r);
    }
    /* lines formatted on the GPU, copied out through pinned buffers (TFIDF.c:245,274-282) */
    rc = tfidf_write_output_gpu(ctx, outpath, 0);
    if (rc == TFIDF_E_OUTPUT) printf("Error Opening File: %s\n", outpath);
    else if (rc) { fprintf(stderr, "tfidf: %s\n", tfidf_strerror(rc)); tfidf_close(ctx); return 3; }
    tfidf_close(ctx);
    tfidf_free(bytes);
    tfidf_free(doc_off);
    return 0;
}
