/*
 * tfidf.h — C-ABI of the MI355X-native TF-IDF engine (libtfidf_hip.so).
 *
 * The reference (ndas7/Parallel-Systems-MPI-TFIDF, TFIDF.c) has no library API: the
 * whole path is one monolithic main() (TFIDF.c:52-287) whose seams are
 *   ingest      input/docN bytes            TFIDF.c:98-110, 130-147
 *   count       wordCount / docSize / df    TFIDF.c:141-196, 291-326
 *   score       tf * log(N/df)              TFIDF.c:202, 243-244
 *   emit        "docN@word\t%.16f", qsort   TFIDF.c:245, 273-282
 * Every entry point below names the reference lines it replaces.  Plain C types only:
 * pointers + sizes, no torch or HIP types.  Every function returns 0 or a negative
 * TFIDF_E* code (never exit()s, unlike TFIDF.c:102,122,137,277).  A context is used
 * by one host thread at a time.
 */
#ifndef TFIDF_H
#define TFIDF_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: tfidf_run_info starts with its own size (set by the caller), the experimental K1 run
 *    flags are gone */
#define TFIDF_ABI_VERSION 2

enum tfidf_status {
    TFIDF_OK = 0,
    TFIDF_E_INVAL = -1,     /* bad argument */
    TFIDF_E_NOMEM = -2,     /* host or device allocation failed */
    TFIDF_E_HIP = -3,       /* HIP runtime error */
    TFIDF_E_RCCL = -4,      /* RCCL error */
    TFIDF_E_NODEV = -5,     /* no usable gfx950 device */
    TFIDF_E_NOINPUT = -6,   /* ./input cannot be opened        (TFIDF.c:100-103) */
    TFIDF_E_NODOC = -7,     /* input/docN cannot be opened     (TFIDF.c:134-138) */
    TFIDF_E_OUTPUT = -8,    /* output.txt cannot be written    (TFIDF.c:274-278) */
    TFIDF_E_CAPACITY = -9,  /* an internal table could not be grown, or a term (a token's bytes
                               up to its first NUL) is 16 MiB or longer: its offset/length
                               word holds 24 length bits, or two distinct terms of 16 bytes or
                               more share their 120-bit identity key (compared byte by byte on
                               every key match: reported, never merged) */
    TFIDF_E_STATE = -10,    /* call out of order (e.g. fetch before run) */
    TFIDF_E_PEER = -11      /* another rank of the DF exchange failed (this rank did not) */
};

/* ---------------------------------------------------------------- corpus ---- */

#define TFIDF_CORPUS_DEVICE 1u   /* bytes/doc_off/doc_ids are device pointers on the ctx's GPU */

/* One shard of documents.  Replaces the reference's per-rank fopen/fscanf ingest
 * (TFIDF.c:130-147): document i (0-based, local) is bytes[doc_off[i], doc_off[i+1]).
 * Document boundaries are token boundaries.  Tokens follow fscanf("%s") in the C
 * locale: maximal runs of bytes not in {0x20,0x09..0x0D}; a term is the token's bytes
 * up to its first NUL (strcmp semantics, TFIDF.c:152,172). */
typedef struct tfidf_corpus {
    const uint8_t*  bytes;
    uint64_t        nbytes;
    const uint64_t* doc_off;      /* ndocs + 1 entries, non-decreasing, doc_off[ndocs] <= nbytes */
    const uint32_t* doc_ids;      /* global 1-based ids ("docN"); NULL means 1..ndocs */
    uint32_t        ndocs;        /* documents in this shard */
    uint32_t        flags;        /* TFIDF_CORPUS_* */
    uint64_t        ndocs_total;  /* N of log(N/df) (TFIDF.c:98-115,243); 0 means ndocs */
} tfidf_corpus;

/* ---------------------------------------------------------------- result ---- */

/* Host-side result, pairs in output order: the strcmp order of the reference's
 * "docN@word\t%.16f" lines (TFIDF.c:245,273).  Arrays are owned by the library and
 * released by tfidf_result_free(). */
typedef struct tfidf_result {
    uint64_t  npairs;       /* unique (doc, term) pairs in this shard = output lines */
    uint32_t  ndocs;        /* documents in this shard */
    uint32_t  nterms;       /* distinct terms in this shard */
    uint64_t  ndocs_total;  /* N used for idf */
    /* per pair (output order) */
    uint32_t* pair_doc;     /* global doc id (TFIDF.c:132 "doc%d") */
    uint32_t* pair_term;    /* index into the term table below */
    uint32_t* pair_count;   /* wordCount     (TFIDF.c:154,163) */
    uint32_t* pair_docsize; /* docSize       (TFIDF.c:141-143) */
    uint32_t* pair_df;      /* numDocsWithWord over ALL shards (TFIDF.c:169-188,215-234) */
    double*   pair_score;   /* tf * log(N/df) (TFIDF.c:202,243-244) */
    /* per local document, input order */
    uint32_t* doc_id;
    uint32_t* doc_size;
    /* term table: this shard's terms in strcmp("word\t") order */
    uint64_t* term_off;     /* nterms + 1 */
    uint8_t*  term_bytes;
    uint32_t* term_df;      /* global df of each term */
} tfidf_result;

/* ---------------------------------------------------------------- context --- */

typedef struct tfidf_ctx tfidf_ctx;

/* Opens device `device` (HIP ordinal).  Fails with TFIDF_E_NODEV unless it is gfx950. */
int tfidf_open(int device, tfidf_ctx** out);
/* Number of visible HIP devices (0 when there is none). */
int tfidf_device_count(void);
void tfidf_close(tfidf_ctx* ctx);
const char* tfidf_strerror(int status);
int tfidf_abi_version(void);

/* ---- multi-GPU: one process per GPU; replaces MPI_Init/Comm_size/Comm_rank
 *      (TFIDF.c:82,91-92) and the DF combine MPI_Reduce(CustomReduce)+MPI_Bcast
 *      (TFIDF.c:209-222,291-326) with RCCL collectives over xGMI, in one of two forms
 *      chosen alike by every rank from the agreed per-rank term counts:
 *        dense (every rank's V <= 2^17, the default for c2/c3/c5-size shards): the ranks'
 *          term keys are all-gathered, numbered identically on every rank, and ONE
 *          ncclAllReduce (sum) of a u32 df vector over those numbers gives the global df;
 *        hash-owner (larger V, e.g. 10^7 terms): each term's df is summed by an owner rank
 *          (a hash of the term) after an all-to-all of (term, df) and returned by a second
 *          all-to-all (grouped ncclSend / ncclRecv).
 *      TFIDF_XCHG=dense|owner|dense_table forces a form. */
#define TFIDF_UNIQUE_ID_BYTES 128
int tfidf_comm_unique_id(uint8_t id[TFIDF_UNIQUE_ID_BYTES]);
/* Attaches an RCCL communicator rank (ncclCommInitRankConfig).  From then on every tfidf_run
 * of this context is collective: all ranks call it, each on its own shard (contiguous
 * ranges of the "docN@" order, ndocs_total = N of the whole corpus).  Capacity retries
 * are agreed between the ranks (all repeat or none does); a rank whose run fails makes
 * the others return TFIDF_E_PEER instead of waiting.
 * Abort contract: the communicator is created non-blocking (a peer that never joins makes
 * this call return TFIDF_E_PEER after TFIDF_COMM_TIMEOUT_S seconds, default 600, 0 = no
 * limit), and every RCCL call and every wait for a collective's kernels is polled.  A
 * failure agreed before the exchange's collectives (a local error, a capacity retry) needs
 * nothing from the caller.  A rank-local failure AFTER the agreement aborts this rank's
 * communicator; a peer process waiting for it gives up at the same deadline (or when RCCL
 * reports the peer's failure) and aborts its own.  A context whose communicator was aborted
 * returns TFIDF_E_PEER from then on: close and reopen it. */
int tfidf_comm_init(tfidf_ctx* ctx, const uint8_t id[TFIDF_UNIQUE_ID_BYTES], int rank, int nranks);   /* nranks <= 1024 */

/* ---- one process, several shards: the drop-in for `mpirun -np P ./TFIDF`
 *      (TFIDF.c:82-92 process group, :125-130 document -> rank assignment, :253-273
 *      gather + sort).  Rank r runs on devices[r] (NULL: device r).  When every rank has
 *      its own GPU the ranks are one RCCL clique (non-blocking communicators created in one
 *      ncclGroupStart/End); when a device is listed more than once (or TFIDF_GROUP_LOCAL is
 *      set) they exchange through device copies in this process — same engine code, same
 *      results.  An error on one rank inside the exchange sets the clique's abort flag: every
 *      rank, wherever it waits (inside an RCCL call, for a collective's kernels, or at its
 *      next call), aborts its own communicator at its next poll, so no peer stays blocked; the
 *      other ranks return TFIDF_E_PEER.  An RCCL group is unusable after such an abort (close
 *      and reopen it); an in-process group starts its next tfidf_group_run afresh. */
#define TFIDF_GROUP_LOCAL 1u
typedef struct tfidf_group tfidf_group;
int tfidf_group_open(int nranks, const int* devices, uint32_t flags, tfidf_group** out);
int tfidf_group_size(const tfidf_group* g);
tfidf_ctx* tfidf_group_ctx(tfidf_group* g, int rank);
/* tfidf_run on every rank at once (one host thread per rank); shards[nranks].  Returns
 * the lowest rank's own error, else TFIDF_E_PEER, else 0. */
int tfidf_group_run(tfidf_group* g, const tfidf_corpus* shards);
/* every rank formats its lines on its GPU, then output.txt = the texts in rank order */
int tfidf_group_write_output(tfidf_group* g, const char* path);
void tfidf_group_close(tfidf_group* g);

/* Runs the whole hot path on this shard: tokenize -> per-document TF counts ->
 * vocabulary -> DF (all-reduced across ranks when a communicator is attached) ->
 * tf*log(N/df) -> output order.  Replaces TFIDF.c:130-273.  Results stay in HBM
 * until tfidf_fetch().  Host-pointer corpora are copied to HBM first. */
int tfidf_run(tfidf_ctx* ctx, const tfidf_corpus* corpus);

/* Copies the last run's results to host memory. */
int tfidf_fetch(tfidf_ctx* ctx, tfidf_result* out);
void tfidf_result_free(tfidf_result* r);

/* Counters of the last run (sizes, for roofline accounting).  The caller sets `size` to
 * sizeof(tfidf_run_info) as it was compiled; the library writes no byte past it (a
 * caller built against an older, shorter struct gets its prefix), and sets `size` to the
 * bytes it wrote.  TFIDF_E_INVAL when size < 16. */
typedef struct tfidf_run_info {
    uint64_t size;            /* in: sizeof(tfidf_run_info) of the caller; out: bytes written */
    uint64_t nbytes;          /* C */
    uint64_t ntokens;         /* T */
    uint64_t npairs;          /* P */
    uint32_t nterms;          /* V (this shard) */
    uint32_t nterms_global;   /* V over all ranks */
    uint64_t nchunks;         /* tokenize+count work units */
    uint64_t partial_records; /* (doc, term) records of documents split across work units */
    uint32_t ndocs;
    uint32_t vocab_capacity;
    double   ms_total;        /* device time of the whole run (HIP events) */
    double   ms_tokcount;     /* device time of the tokenize+count kernels (HIP events) */
    double   ms_stage[16];    /* per-stage device times, see tfidf_stage_name() */
    uint32_t nstages;
    uint32_t flags;           /* TFIDF_RUN_* */
    /* device (re)allocations made by this library in this process since it was loaded
     * (hipMalloc of the engine's buffers, cumulative, all contexts): a caller timing
     * steady-state runs reads them before and after and expects no change */
    uint64_t device_allocs;
    uint64_t device_alloc_bytes;
    /* the run's idf table, log(N/df) on the host's libm (TFIDF.c:243): up to 2^18 documents
     * every df = 1..N is tabulated by the context's host worker threads while the device runs
     * the stages before the score; beyond that only the run's distinct df values, after the DF
     * stage (one host round trip) */
    uint64_t idf_logs;        /* libm log() calls made for this run's table (every run builds its own) */
    double   ms_idf_host;     /* wall time of those calls (host threads) */
    double   ms_idf_wait;     /* time the run waited for them before the score stage */
} tfidf_run_info;
#define TFIDF_RUN_K1_VS   2u  /* slot-keyed tokenize+count kernel (the default path; the general
                                 kernel of TFIDF_K1=general or an unaligned corpus leaves it clear) */
#define TFIDF_RUN_K1_ST   4u  /* retired: round 3's k_tokcount_st (removed in round 5), never set */
#define TFIDF_RUN_K1_SL   8u  /* ... run as k_tokcount_sl (the default, vocabulary table <= 32M slots);
                                 neither ST nor SL with VS set: k_tokcount_vs (larger tables) */
#define TFIDF_RUN_XCHG_DENSE 16u  /* multi-rank: the DF exchange used the dense all-reduce form
                                     (else the hash-owner all-to-all; single rank: no exchange) */
int tfidf_last_run_info(tfidf_ctx* ctx, tfidf_run_info* info);
/* Sums over the successful runs since the last reset (a caller timing many runs reads them
 * once instead of querying every run): runs, K1 ms, whole-run ms (HIP events: 0 while
 * timing is off), idf logs, idf host ms, idf wait ms.  reset != 0 zeroes them after the read. */
typedef struct tfidf_run_totals {
    uint64_t runs;
    double ms_tokcount, ms_total;
    uint64_t idf_logs;
    double ms_idf_host, ms_idf_wait;
} tfidf_run_totals;
int tfidf_run_totals_get(tfidf_ctx* ctx, tfidf_run_totals* out, int reset);
/* The same device-allocation counters without a run (process-wide, cumulative). */
int tfidf_alloc_stats(uint64_t* allocs, uint64_t* bytes);
const char* tfidf_stage_name(int stage);
/* HIP event timing of a run's stages (tfidf_run_info.ms_stage / ms_tokcount / ms_total):
 * enable 0 none, 1 every stage (the default; ten event records per run), 2 the tokenize+count
 * kernel and the whole run only (four records; each record costs the stream ~5 us). */
int tfidf_set_timing(tfidf_ctx* ctx, int enable);
/* Diagnostics: per-phase cycle sums of the fast tokenize+count kernel, available only
 * from the diagnostic build lib/libtfidf_hip_stamps.so with TFIDF_STAMPS=1 set before
 * tfidf_open.  Returns the number of values written (phases + workgroup count). */
int tfidf_debug_k1_stamps(tfidf_ctx* ctx, uint64_t* out, int n);

/* Diagnostics: measured HBM streaming peaks on this device (SURVEY §8d's "fraction of a
 * measured copy-kernel peak"): GB/s of a read-only stream over nbytes and of an nbytes
 * copy (2 x nbytes moved), each averaged over `iters` passes after a warm-up. */
int tfidf_hbm_probe(tfidf_ctx* ctx, uint64_t nbytes, int iters, double* read_gbps, double* copy_gbps);

/* ---------------------------------------------------------------- emission -- */

/* GPU emission (the default output path): formats the last run's lines
 * "docN@word\t%.16f\n" (TFIDF.c:245,281) in output order into one text in HBM.  %.16f
 * is computed exactly (integer significand x 10^16, 128-bit, ties to even: glibc
 * printf's result).  The corpus of the run must still be valid (long terms' bytes are
 * read from it).  *nbytes = the text's size. */
int tfidf_format(tfidf_ctx* ctx, uint64_t* nbytes);
/* Copies bytes [off, off + n) of the formatted text to host memory. */
int tfidf_copy_text(tfidf_ctx* ctx, uint64_t off, void* dst, uint64_t n);
/* tfidf_format + D2H + write to `path` (TFIDF.c:274-282); append != 0 appends (a shard
 * after the previous ones).  An unformatted result is formatted in document groups whose
 * D2H copies overlap the next group's formatting; the copies go through the context's
 * ring of pinned 16 MB buffers (kept across calls) and a regular file is written by
 * several threads at their blocks' offsets (pwrite).  TFIDF_E_OUTPUT when the file
 * cannot be opened or written. */
int tfidf_write_output_gpu(tfidf_ctx* ctx, const char* path, int append);
/* Timings of the last tfidf_write_output_gpu (the caller sets `size` = sizeof). */
typedef struct tfidf_output_info {
    uint64_t size;
    uint64_t text_bytes;      /* bytes written */
    uint32_t writers;         /* host writer threads (1: not a regular file) */
    uint32_t formatted;       /* 1: this call formatted the text (0: it was already) */
    double   ms_prepare;      /* length pass + text size (0 when already formatted) */
    double   ms_d2h_busy;     /* host wall time from the first copy issued to the last copy done */
    double   ms_write;        /* summed host time inside write/pwrite (over writer threads) */
    double   ms_total;        /* the whole call */
} tfidf_output_info;
int tfidf_last_output_info(const tfidf_ctx* ctx, tfidf_output_info* info);
/* The device %.16f formatter on n host doubles: out = n 32-byte slots, NUL-padded.
 * TFIDF_E_INVAL for values outside [0, 2^63/10^16) (scores are < 23). */
int tfidf_format_f64(tfidf_ctx* ctx, const double* vals, uint64_t n, char* out);

/* Host emission from a fetched result (glibc snprintf; kept for callers that already
 * hold a tfidf_result): writes the same lines to `path`. */
int tfidf_write_output(const tfidf_result* r, const char* path);
/* Prints the debug TF Job / IDF Job blocks (TFIDF.c:199-205,236-239) to stdout,
 * one block pair for this shard, pairs in output order. */
int tfidf_print_jobs(const tfidf_result* r);

/* ---------------------------------------------------------------- ingest ---- */

/* Reference input contract (TFIDF.c:98-110,130-147): N = number of entries of `dir`
 * other than "." and ".."; documents are dir/doc1 .. dir/docN.  Reads them into one
 * malloc'd buffer with doc_off[N+1].  Returns TFIDF_E_NOINPUT / TFIDF_E_NODOC
 * (with *bad_doc set) like the reference's error exits. */
int tfidf_ingest_dir(const char* dir, uint8_t** bytes, uint64_t* nbytes,
                     uint64_t** doc_off, uint32_t* ndocs, uint32_t* bad_doc);
void tfidf_free(void* p);

/* Streaming ingest into HBM (replaces TFIDF.c:98-110,130-147): the
 * same contract as tfidf_ingest_dir (N = entries of `dir` other than "." and "..";
 * documents dir/doc1..docN; TFIDF_E_NOINPUT / TFIDF_E_NODOC with *bad_doc = the smallest
 * document that cannot be read), but the files are pread() by `nthreads` host threads
 * (0: OMP_NUM_THREADS, at most 16) into a ring of pinned 8 MiB segments whose H2D copies
 * overlap the reads.  *out is a device corpus (TFIDF_CORPUS_DEVICE, doc ids 1..N) owned
 * by the context, valid until the next ingest, host-corpus tfidf_run or tfidf_close.
 * `info` (optional) receives sizes and host wall times. */
typedef struct tfidf_ingest_info {
    uint64_t nbytes;      /* corpus bytes */
    uint64_t segments;    /* 8 MiB staging segments copied */
    uint32_t ndocs;       /* N */
    uint32_t threads;     /* reader threads used */
    double   ms_scan;     /* directory count + open/fstat of every document */
    double   ms_read;     /* reads + overlapped H2D, until the last copy completed */
    double   ms_total;
} tfidf_ingest_info;
int tfidf_ingest_dir_device(tfidf_ctx* ctx, const char* dir, int nthreads, tfidf_corpus* out,
                            uint32_t* bad_doc, tfidf_ingest_info* info);

/* Byte-balanced shard plan of an input directory (replaces the round-robin
 * document -> rank deal of TFIDF.c:125-130).  One scan gives N (every entry but "." and
 * "..", TFIDF.c:98-110) and the sizes of doc1..docN (TFIDF.c:130-138 error contract:
 * TFIDF_E_NOINPUT, TFIDF_E_NODOC with *bad_doc = the smallest missing id).  Documents are
 * ordered by "docN@" (the output's strcmp order, TFIDF.c:49,273) and cut into nshards
 * contiguous ranges at the cuts nearest to r * total / nshards, so every shard holds at
 * most total / nshards + the largest document and the shards' outputs concatenate in
 * shard order.  Release with tfidf_plan_free. */
typedef struct tfidf_dir_plan {
    uint32_t  ndocs;         /* N */
    uint32_t  nshards;
    uint32_t* doc_ids;       /* N document ids in "docN@" order */
    uint64_t* doc_bytes;     /* their sizes */
    uint32_t* shard_first;   /* nshards + 1: shard r = doc_ids[shard_first[r] .. shard_first[r + 1]) */
    uint64_t* shard_bytes;   /* nshards */
} tfidf_dir_plan;
int tfidf_plan_dir(const char* dir, uint32_t nshards, int nthreads, tfidf_dir_plan* plan, uint32_t* bad_doc);
void tfidf_plan_free(tfidf_dir_plan* plan);
/* Streams shard `shard` of the plan into the context's HBM like tfidf_ingest_dir_device;
 * the corpus carries the documents' global ids (device) and ndocs_total = N. */
int tfidf_ingest_shard_device(tfidf_ctx* ctx, const char* dir, const tfidf_dir_plan* plan, uint32_t shard,
                              int nthreads, tfidf_corpus* out, uint32_t* bad_doc, tfidf_ingest_info* info);
/* The plan's pieces on their own (host only): ids 1..n in "docN@" order, and the
 * byte-balanced cut of a sequence of sizes (first[nshards + 1]). */
int tfidf_doc_name_order(uint32_t n, uint32_t* ids);
int tfidf_shard_split(const uint64_t* bytes, uint32_t n, uint32_t nshards, uint32_t* first);

/* ---------------------------------------------------------------- synthetic - */

/* Synthetic Zipfian corpus (generator in csrc/synth.h).  ntok[i] tokens
 * in local document i whose global id is doc_ids[i]; cdf = Zipf CDF over V ranks
 * (zipf mode) or NULL (mode 1: config-1 "4 words per doc").  Host version fills
 * caller-provided buffers (query the size first with bytes == NULL). */
int tfidf_synth_host(uint64_t seed, uint32_t V, uint32_t mode, const double* cdf,
                     const uint32_t* doc_ids, const uint64_t* ntok, uint32_t ndocs,
                     uint8_t* bytes, uint64_t* nbytes, uint64_t* doc_off);
/* Device version: generates straight into HBM buffers owned by the ctx and returns a
 * device corpus (flags = TFIDF_CORPUS_DEVICE) valid until the next synth call or
 * tfidf_close. */
int tfidf_synth_device(tfidf_ctx* ctx, uint64_t seed, uint32_t V, uint32_t mode,
                       const double* cdf, const uint32_t* doc_ids, const uint64_t* ntok,
                       uint32_t ndocs, uint64_t ndocs_total, tfidf_corpus* out);

#ifdef __cplusplus
}
#endif
#endif /* TFIDF_H */
