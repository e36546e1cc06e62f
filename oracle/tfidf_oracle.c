/*
 * tfidf_oracle.c — CPU restatement of the reference TF-IDF path (TFIDF.c).
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product
 * path (libtfidf_hip.so) never links, calls or falls back to it.
 *
 * Parity pinning: this restatement is checked byte-for-byte against golden outputs of
 * the reference program itself (oracle/_ref/TFIDF, built from /root/reference/TFIDF.c
 * by oracle/Makefile and run under MPICH mpirun by tests/golden/make_golden.py); see
 * tests/test_oracle_golden.py.
 *
 * What it restates (file:line in /root/reference/TFIDF.c):
 *   N            = entries of input/ except "." and ".."            :98-110
 *   tokens       = fscanf(fp,"%s") runs of non-isspace bytes (C locale) :141-147
 *   docSize      = tokens in the document                            :141-143
 *   term         = token bytes up to the first NUL (strcmp/strcpy)   :152,161,172,184
 *   wordCount    = occurrences of (term, doc)                        :151-167
 *   df           = documents containing term (currDoc dedupe, summed
 *                  over ranks by CustomReduce)                       :169-188,291-319
 *   tf           = 1.0 * wordCount / docSize                         :202
 *   idf          = log(1.0 * N / df)  (glibc libm)                   :243
 *   score        = tf * idf                                          :244
 *   line         = sprintf("%s@%s\t%.16f", "doc<i>", word, score)    :132,245
 *   order        = qsort(strcmp) over the lines                      :47-50,273
 *   output.txt   = lines + '\n'                                      :274-282
 *   debug jobs   = "word@docN\twc/ds" and "word@docN\tN/df"          :199-205,236-239
 * The reference's linear searches (O(P) strcmp per token) are restated with hash
 * tables; the function computed is the same.  Capacity defects of the reference
 * (32-entry stack arrays, 16-byte word buffer: SURVEY Appendix B) are not reproduced.
 */
#include <dirent.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct oracle_out {
    uint64_t npairs;
    uint32_t nterms;
    uint32_t ndocs;
    /* per pair, output (strcmp) order */
    uint32_t* doc_id;
    uint32_t* term;     /* index into term table */
    uint32_t* count;
    uint32_t* docsize;
    uint32_t* df;
    double* score;
    /* term table, intern (first occurrence) order */
    uint64_t* term_off; /* nterms + 1 */
    char* term_pool;
    /* output.txt content */
    char* lines;
    uint64_t lines_len;
    /* debug job lines, per document in input order, first-occurrence order inside */
    char* tf_jobs;
    uint64_t tf_len;
    char* idf_jobs;
    uint64_t idf_len;
} oracle_out;

/* isspace() in the C locale: the set fscanf("%s") stops at (TFIDF.c:142,147) */
static inline int o_ws(uint8_t c) { return c == 0x20 || (c >= 0x09 && c <= 0x0D); }

static uint64_t o_hash(const uint8_t* p, uint64_t n, uint64_t salt) {
    uint64_t h = 0xcbf29ce484222325ull ^ salt;
    for (uint64_t i = 0; i < n; ++i) { h ^= p[i]; h *= 0x100000001b3ull; }
    h ^= h >> 29; h *= 0xbf58476d1ce4e5b9ull; h ^= h >> 32;
    return h;
}

/* ---- growable byte buffer ---- */
typedef struct { char* p; uint64_t n, cap; } o_buf;
static void ob_need(o_buf* b, uint64_t extra) {
    if (b->n + extra + 1 <= b->cap) return;
    uint64_t c = b->cap ? b->cap : 4096;
    while (c < b->n + extra + 1) c *= 2;
    b->p = (char*)realloc(b->p, c);
    if (!b->p) { fprintf(stderr, "oracle: out of memory\n"); exit(3); }
    b->cap = c;
}

/* ---- term intern table: term bytes -> term index ---- */
typedef struct {
    uint32_t* slot;       /* term index + 1, 0 = empty */
    uint64_t cap;         /* power of two */
    uint32_t n;
    uint64_t* off;        /* term k = pool[off[k], off[k+1]) */
    uint64_t off_cap;
    o_buf pool;
    uint32_t* df;         /* numDocsWithWord */
    uint32_t* last_doc;   /* currDoc (TFIDF.c:174-177) */
} o_vocab;

static void ov_init(o_vocab* v) {
    memset(v, 0, sizeof(*v));
    v->cap = 1024;
    v->slot = (uint32_t*)calloc(v->cap, sizeof(uint32_t));
    v->off_cap = 1024;
    v->off = (uint64_t*)malloc(v->off_cap * sizeof(uint64_t));
    v->df = (uint32_t*)malloc(v->off_cap * sizeof(uint32_t));
    v->last_doc = (uint32_t*)malloc(v->off_cap * sizeof(uint32_t));
    v->off[0] = 0;
}

static void ov_grow(o_vocab* v) {
    uint64_t ncap = v->cap * 2;
    uint32_t* ns = (uint32_t*)calloc(ncap, sizeof(uint32_t));
    for (uint64_t i = 0; i < v->cap; ++i) {
        uint32_t e = v->slot[i];
        if (!e) continue;
        uint32_t k = e - 1;
        uint64_t h = o_hash((const uint8_t*)v->pool.p + v->off[k], v->off[k + 1] - v->off[k], 0) & (ncap - 1);
        while (ns[h]) h = (h + 1) & (ncap - 1);
        ns[h] = e;
    }
    free(v->slot);
    v->slot = ns;
    v->cap = ncap;
}

static uint32_t ov_intern(o_vocab* v, const uint8_t* w, uint64_t n) {
    if ((uint64_t)(v->n + 1) * 2 > v->cap) ov_grow(v);
    uint64_t h = o_hash(w, n, 0) & (v->cap - 1);
    for (;;) {
        uint32_t e = v->slot[h];
        if (!e) break;
        uint32_t k = e - 1;
        if (v->off[k + 1] - v->off[k] == n && memcmp(v->pool.p + v->off[k], w, n) == 0) return k;
        h = (h + 1) & (v->cap - 1);
    }
    uint32_t k = v->n++;
    if ((uint64_t)v->n + 1 > v->off_cap) {
        v->off_cap *= 2;
        v->off = (uint64_t*)realloc(v->off, v->off_cap * sizeof(uint64_t));
        v->df = (uint32_t*)realloc(v->df, v->off_cap * sizeof(uint32_t));
        v->last_doc = (uint32_t*)realloc(v->last_doc, v->off_cap * sizeof(uint32_t));
    }
    ob_need(&v->pool, n);
    memcpy(v->pool.p + v->pool.n, w, n);
    v->pool.n += n;
    v->off[k + 1] = v->pool.n;
    v->df[k] = 0;
    v->last_doc[k] = UINT32_MAX;
    v->slot[h] = k + 1;
    return k;
}

/* ---- per-document pair list (TFIDF[] records, TFIDF.c:26-35,151-167) ---- */
typedef struct { uint32_t doc_idx, term, count; } o_pair;

typedef struct { const char* s; uint64_t i; } o_line;
static int o_line_cmp(const void* a, const void* b) {
    return strcmp(((const o_line*)a)->s, ((const o_line*)b)->s);
}

int oracle_run(const uint8_t* bytes, const uint64_t* doc_off, uint32_t ndocs,
               const uint32_t* doc_ids, uint64_t n_total, oracle_out* out) {
    memset(out, 0, sizeof(*out));
    if (n_total == 0) n_total = ndocs;
    o_vocab v;
    ov_init(&v);
    o_pair* pairs = NULL;
    uint64_t np = 0, np_cap = 0;
    uint32_t* docsize = (uint32_t*)calloc(ndocs ? ndocs : 1, sizeof(uint32_t));
    uint64_t* doc_first_pair = (uint64_t*)calloc((uint64_t)ndocs + 1, sizeof(uint64_t));
    /* per-document term -> pair index map, cleared per document */
    uint64_t dcap = 256;
    uint32_t* dmap = (uint32_t*)malloc(dcap * 2 * sizeof(uint32_t)); /* (term+1, pair idx) */
    for (uint32_t d = 0; d < ndocs; ++d) {
        const uint8_t* p = bytes + doc_off[d];
        const uint8_t* e = bytes + doc_off[d + 1];
        doc_first_pair[d] = np;
        /* pass 1: docSize (TFIDF.c:141-143) */
        uint32_t ds = 0;
        for (const uint8_t* q = p; q < e;) {
            while (q < e && o_ws(*q)) ++q;
            if (q >= e) break;
            ++ds;
            while (q < e && !o_ws(*q)) ++q;
        }
        docsize[d] = ds;
        /* per-document map sized for ds tokens */
        uint64_t need = 16;
        while (need < (uint64_t)ds * 2) need *= 2;
        if (need > dcap) { dcap = need; dmap = (uint32_t*)realloc(dmap, dcap * 2 * sizeof(uint32_t)); }
        memset(dmap, 0, need * 2 * sizeof(uint32_t));
        /* pass 2: counts (TFIDF.c:147-189) */
        for (const uint8_t* q = p; q < e;) {
            while (q < e && o_ws(*q)) ++q;
            if (q >= e) break;
            const uint8_t* s = q;
            while (q < e && !o_ws(*q)) ++q;
            uint64_t n = (uint64_t)(q - s);
            const uint8_t* z = (const uint8_t*)memchr(s, 0, n); /* strcmp/strcpy stop at NUL */
            if (z) n = (uint64_t)(z - s);
            uint32_t t = ov_intern(&v, s, n);
            uint64_t h = ((uint64_t)t * 0x9E3779B97F4A7C15ull >> 17) & (need - 1);
            for (;;) {
                if (dmap[2 * h] == 0) {
                    if (np == np_cap) {
                        np_cap = np_cap ? np_cap * 2 : 4096;
                        pairs = (o_pair*)realloc(pairs, np_cap * sizeof(o_pair));
                    }
                    pairs[np].doc_idx = d; pairs[np].term = t; pairs[np].count = 1;
                    dmap[2 * h] = t + 1; dmap[2 * h + 1] = (uint32_t)(np - doc_first_pair[d]);
                    ++np;
                    break;
                }
                if (dmap[2 * h] == t + 1) { pairs[doc_first_pair[d] + dmap[2 * h + 1]].count++; break; }
                h = (h + 1) & (need - 1);
            }
            if (v.last_doc[t] != d) { v.df[t]++; v.last_doc[t] = d; } /* TFIDF.c:174-177 */
        }
    }
    doc_first_pair[ndocs] = np;

    /* lines (TFIDF.c:202,243-245) */
    o_buf lines = {0}, tfj = {0}, idfj = {0};
    uint64_t* line_off = (uint64_t*)malloc((np + 1) * sizeof(uint64_t));
    double* score = (double*)malloc((np ? np : 1) * sizeof(double));
    char num[64];
    for (uint64_t i = 0; i < np; ++i) {
        const o_pair* pr = &pairs[i];
        uint32_t id = doc_ids ? doc_ids[pr->doc_idx] : pr->doc_idx + 1;
        const char* w = v.pool.p + v.off[pr->term];
        int wl = (int)(v.off[pr->term + 1] - v.off[pr->term]);
        double tf = 1.0 * pr->count / docsize[pr->doc_idx];
        double idf = log(1.0 * (double)n_total / v.df[pr->term]);
        double sc = tf * idf;
        score[i] = sc;
        line_off[i] = lines.n;
        int nn = snprintf(num, sizeof num, "doc%u@", id);
        ob_need(&lines, (uint64_t)nn + (uint64_t)wl + 64);
        memcpy(lines.p + lines.n, num, (size_t)nn); lines.n += (uint64_t)nn;
        memcpy(lines.p + lines.n, w, (size_t)wl); lines.n += (uint64_t)wl;
        lines.n += (uint64_t)snprintf(lines.p + lines.n, 64, "\t%.16f", sc);
        lines.p[lines.n++] = 0;
        ob_need(&tfj, (uint64_t)wl + 64);
        memcpy(tfj.p + tfj.n, w, (size_t)wl); tfj.n += (uint64_t)wl;
        tfj.n += (uint64_t)snprintf(tfj.p + tfj.n, 64, "@doc%u\t%u/%u\n", id, pr->count, docsize[pr->doc_idx]);
        ob_need(&idfj, (uint64_t)wl + 64);
        memcpy(idfj.p + idfj.n, w, (size_t)wl); idfj.n += (uint64_t)wl;
        idfj.n += (uint64_t)snprintf(idfj.p + idfj.n, 64, "@doc%u\t%llu/%u\n", id,
                                     (unsigned long long)n_total, v.df[pr->term]);
    }
    line_off[np] = lines.n;

    /* qsort(strcmp) (TFIDF.c:47-50,273) over line starts; carry the pair index */
    o_line* ord = (o_line*)malloc((np ? np : 1) * sizeof(o_line));
    for (uint64_t i = 0; i < np; ++i) { ord[i].s = lines.p + line_off[i]; ord[i].i = i; }
    qsort(ord, np, sizeof(o_line), o_line_cmp);

    out->npairs = np;
    out->ndocs = ndocs;
    out->nterms = v.n;
    out->doc_id = (uint32_t*)malloc((np ? np : 1) * sizeof(uint32_t));
    out->term = (uint32_t*)malloc((np ? np : 1) * sizeof(uint32_t));
    out->count = (uint32_t*)malloc((np ? np : 1) * sizeof(uint32_t));
    out->docsize = (uint32_t*)malloc((np ? np : 1) * sizeof(uint32_t));
    out->df = (uint32_t*)malloc((np ? np : 1) * sizeof(uint32_t));
    out->score = (double*)malloc((np ? np : 1) * sizeof(double));
    o_buf txt = {0};
    ob_need(&txt, lines.n + np);
    for (uint64_t r = 0; r < np; ++r) {
        uint64_t i = ord[r].i;
        const o_pair* pr = &pairs[i];
        out->doc_id[r] = doc_ids ? doc_ids[pr->doc_idx] : pr->doc_idx + 1;
        out->term[r] = pr->term;
        out->count[r] = pr->count;
        out->docsize[r] = docsize[pr->doc_idx];
        out->df[r] = v.df[pr->term];
        out->score[r] = score[i];
        uint64_t l = line_off[i + 1] - line_off[i] - 1;
        memcpy(txt.p + txt.n, lines.p + line_off[i], l);
        txt.n += l;
        txt.p[txt.n++] = '\n';
    }
    out->lines = txt.p ? txt.p : (char*)calloc(1, 1);
    out->lines_len = txt.n;
    out->term_off = (uint64_t*)malloc(((uint64_t)v.n + 1) * sizeof(uint64_t));
    memcpy(out->term_off, v.off, ((uint64_t)v.n + 1) * sizeof(uint64_t));
    out->term_pool = v.pool.p ? v.pool.p : (char*)calloc(1, 1);
    out->tf_jobs = tfj.p ? tfj.p : (char*)calloc(1, 1);
    out->tf_len = tfj.n;
    out->idf_jobs = idfj.p ? idfj.p : (char*)calloc(1, 1);
    out->idf_len = idfj.n;

    free(ord); free(line_off); free(score); free(lines.p);
    free(pairs); free(docsize); free(doc_first_pair); free(dmap);
    free(v.slot); free(v.off); free(v.df); free(v.last_doc);
    return 0;
}

void oracle_free(oracle_out* o) {
    free(o->doc_id); free(o->term); free(o->count); free(o->docsize); free(o->df); free(o->score);
    free(o->term_off); free(o->term_pool); free(o->lines); free(o->tf_jobs); free(o->idf_jobs);
    memset(o, 0, sizeof(*o));
}

/* ------------------------------------------------------------------------------
 * CPU baseline of the whole multi-worker path (bench.py cpu_baseline only): the
 * reference's rank structure on host threads.  Shard s = documents order[first[s] ..
 * first[s+1]) (contiguous "docN@" ranges, so shard outputs concatenate in order):
 *   1. every thread tokenizes and counts its shard (TFIDF.c:130-196, as oracle_run);
 *   2. the DF combine: shard vocabularies merged, df summed (CustomReduce + Bcast,
 *      TFIDF.c:209-222,291-326);
 *   3. every thread scores and formats its lines with the global df and sorts them
 *      (TFIDF.c:202,243-245,273);
 *   4. the shard texts are concatenated in shard order (the gather, TFIDF.c:253-270).
 * All four phases are inside the caller's timed region. */
#include <pthread.h>

typedef struct {
    const uint8_t* bytes;
    const uint64_t* doc_off;
    const uint32_t* doc_ids;
    const uint32_t* order;
    uint32_t a, b;            /* order[a .. b) */
    uint64_t n_total;
    o_vocab v;
    o_pair* pairs;
    uint64_t np;
    uint32_t* docsize;        /* by position in [a, b) */
    uint32_t* gdf;            /* global df of each shard term (phase 2) */
    o_buf text;
} o_shard;

static void* o_shard_count(void* arg) {
    o_shard* s = (o_shard*)arg;
    o_vocab* v = &s->v;
    ov_init(v);
    const uint32_t nd = s->b - s->a;
    s->docsize = (uint32_t*)calloc(nd ? nd : 1, sizeof(uint32_t));
    uint64_t np_cap = 0, dcap = 256;
    uint32_t* dmap = (uint32_t*)malloc(dcap * 2 * sizeof(uint32_t));
    for (uint32_t j = 0; j < nd; ++j) {
        const uint32_t d = s->order[s->a + j];
        const uint8_t* p = s->bytes + s->doc_off[d];
        const uint8_t* e = s->bytes + s->doc_off[d + 1];
        const uint64_t first = s->np;
        uint32_t ds = 0;
        for (const uint8_t* q = p; q < e;) {
            while (q < e && o_ws(*q)) ++q;
            if (q >= e) break;
            ++ds;
            while (q < e && !o_ws(*q)) ++q;
        }
        s->docsize[j] = ds;
        uint64_t need = 16;
        while (need < (uint64_t)ds * 2) need *= 2;
        if (need > dcap) { dcap = need; dmap = (uint32_t*)realloc(dmap, dcap * 2 * sizeof(uint32_t)); }
        memset(dmap, 0, need * 2 * sizeof(uint32_t));
        for (const uint8_t* q = p; q < e;) {
            while (q < e && o_ws(*q)) ++q;
            if (q >= e) break;
            const uint8_t* w = q;
            while (q < e && !o_ws(*q)) ++q;
            uint64_t n = (uint64_t)(q - w);
            const uint8_t* z = (const uint8_t*)memchr(w, 0, n);
            if (z) n = (uint64_t)(z - w);
            const uint32_t t = ov_intern(v, w, n);
            uint64_t h = ((uint64_t)t * 0x9E3779B97F4A7C15ull >> 17) & (need - 1);
            for (;;) {
                if (dmap[2 * h] == 0) {
                    if (s->np == np_cap) {
                        np_cap = np_cap ? np_cap * 2 : 4096;
                        s->pairs = (o_pair*)realloc(s->pairs, np_cap * sizeof(o_pair));
                    }
                    s->pairs[s->np].doc_idx = j; s->pairs[s->np].term = t; s->pairs[s->np].count = 1;
                    dmap[2 * h] = t + 1; dmap[2 * h + 1] = (uint32_t)(s->np - first);
                    ++s->np;
                    break;
                }
                if (dmap[2 * h] == t + 1) { s->pairs[first + dmap[2 * h + 1]].count++; break; }
                h = (h + 1) & (need - 1);
            }
            if (v->last_doc[t] != j) { v->df[t]++; v->last_doc[t] = j; }
        }
    }
    free(dmap);
    return NULL;
}

static void* o_shard_emit(void* arg) {
    o_shard* s = (o_shard*)arg;
    o_buf lines = {0};
    uint64_t* line_off = (uint64_t*)malloc((s->np + 1) * sizeof(uint64_t));
    char num[64];
    for (uint64_t i = 0; i < s->np; ++i) {
        const o_pair* pr = &s->pairs[i];
        const uint32_t d = s->order[s->a + pr->doc_idx];
        const uint32_t id = s->doc_ids ? s->doc_ids[d] : d + 1;
        const char* w = s->v.pool.p + s->v.off[pr->term];
        const int wl = (int)(s->v.off[pr->term + 1] - s->v.off[pr->term]);
        const double sc = (1.0 * pr->count / s->docsize[pr->doc_idx]) * log(1.0 * (double)s->n_total / s->gdf[pr->term]);
        line_off[i] = lines.n;
        const int nn = snprintf(num, sizeof num, "doc%u@", id);
        ob_need(&lines, (uint64_t)nn + (uint64_t)wl + 64);
        memcpy(lines.p + lines.n, num, (size_t)nn); lines.n += (uint64_t)nn;
        memcpy(lines.p + lines.n, w, (size_t)wl); lines.n += (uint64_t)wl;
        lines.n += (uint64_t)snprintf(lines.p + lines.n, 64, "\t%.16f", sc);
        lines.p[lines.n++] = 0;
    }
    o_line* ord = (o_line*)malloc((s->np ? s->np : 1) * sizeof(o_line));
    for (uint64_t i = 0; i < s->np; ++i) { ord[i].s = lines.p + line_off[i]; ord[i].i = i; }
    qsort(ord, s->np, sizeof(o_line), o_line_cmp);
    ob_need(&s->text, lines.n + 1);
    for (uint64_t r = 0; r < s->np; ++r) {
        const uint64_t l = strlen(ord[r].s);
        memcpy(s->text.p + s->text.n, ord[r].s, l);
        s->text.n += l;
        s->text.p[s->text.n++] = '\n';
    }
    free(ord); free(line_off); free(lines.p);
    return NULL;
}

int oracle_run_sharded(const uint8_t* bytes, const uint64_t* doc_off, const uint32_t* doc_ids, uint64_t n_total,
                       const uint32_t* order, const uint32_t* first, uint32_t nshards, char** text, uint64_t* len,
                       uint64_t* npairs) {
    o_shard* sh = (o_shard*)calloc(nshards, sizeof(o_shard));
    pthread_t* th = (pthread_t*)malloc(nshards * sizeof(pthread_t));
    for (uint32_t k = 0; k < nshards; ++k) {
        sh[k].bytes = bytes; sh[k].doc_off = doc_off; sh[k].doc_ids = doc_ids; sh[k].order = order;
        sh[k].a = first[k]; sh[k].b = first[k + 1]; sh[k].n_total = n_total;
    }
    for (uint32_t k = 0; k < nshards; ++k) pthread_create(&th[k], NULL, o_shard_count, &sh[k]);
    for (uint32_t k = 0; k < nshards; ++k) pthread_join(th[k], NULL);
    /* DF combine: one global term table, df summed over the shards */
    o_vocab g;
    ov_init(&g);
    uint32_t** map = (uint32_t**)malloc(nshards * sizeof(uint32_t*));
    for (uint32_t k = 0; k < nshards; ++k) {
        map[k] = (uint32_t*)malloc((sh[k].v.n + 1) * sizeof(uint32_t));
        for (uint32_t t = 0; t < sh[k].v.n; ++t) {
            const uint32_t gt = ov_intern(&g, (const uint8_t*)sh[k].v.pool.p + sh[k].v.off[t], sh[k].v.off[t + 1] - sh[k].v.off[t]);
            g.df[gt] += sh[k].v.df[t];
            map[k][t] = gt;
        }
    }
    for (uint32_t k = 0; k < nshards; ++k) {   /* the broadcast: each shard's terms get the global df */
        sh[k].gdf = (uint32_t*)malloc((sh[k].v.n + 1) * sizeof(uint32_t));
        for (uint32_t t = 0; t < sh[k].v.n; ++t) sh[k].gdf[t] = g.df[map[k][t]];
    }
    for (uint32_t k = 0; k < nshards; ++k) pthread_create(&th[k], NULL, o_shard_emit, &sh[k]);
    for (uint32_t k = 0; k < nshards; ++k) pthread_join(th[k], NULL);
    /* gather in shard order */
    uint64_t total = 0, np = 0;
    for (uint32_t k = 0; k < nshards; ++k) { total += sh[k].text.n; np += sh[k].np; }
    char* out = (char*)malloc(total + 1);
    uint64_t at = 0;
    for (uint32_t k = 0; k < nshards; ++k) {
        if (sh[k].text.n) memcpy(out + at, sh[k].text.p, sh[k].text.n);
        at += sh[k].text.n;
    }
    *text = out;
    *len = total;
    *npairs = np;
    for (uint32_t k = 0; k < nshards; ++k) {
        free(sh[k].pairs); free(sh[k].docsize); free(sh[k].gdf); free(sh[k].text.p); free(map[k]);
        free(sh[k].v.slot); free(sh[k].v.off); free(sh[k].v.df); free(sh[k].v.last_doc); free(sh[k].v.pool.p);
    }
    free(g.slot); free(g.off); free(g.df); free(g.last_doc); free(g.pool.p);
    free(map); free(sh); free(th);
    return 0;
}

void oracle_free_text(char* p) { free(p); }

/* N semantics (TFIDF.c:98-110): every entry except "." and ".." */
int oracle_count_entries(const char* dir) {
    DIR* d = opendir(dir);
    if (!d) return -1;
    int n = 0;
    struct dirent* e;
    while ((e = readdir(d)) != NULL) {
        if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
        ++n;
    }
    closedir(d);
    return n;
}

#ifdef ORACLE_MAIN
/* Process-contract mirror of `mpirun -np 2 ./TFIDF` (one worker rank). */
int main(void) {
    int n = oracle_count_entries("input");
    if (n < 0) { printf("Directory failed to open\n"); return 1; }       /* TFIDF.c:100-103 */
    uint64_t* off = (uint64_t*)malloc(((uint64_t)n + 1) * sizeof(uint64_t));
    o_buf all = {0};
    off[0] = 0;
    for (int i = 1; i <= n; ++i) {
        char fn[64];
        snprintf(fn, sizeof fn, "input/doc%d", i);
        FILE* fp = fopen(fn, "rb");
        if (!fp) {                                                       /* TFIDF.c:134-138 */
            printf("Error Opening File: %s, rank = %d, i=%d, numDocs= %d\n", fn, 1, i, n);
            return 0;
        }
        char tmp[1 << 16];
        size_t r;
        while ((r = fread(tmp, 1, sizeof tmp, fp)) > 0) { ob_need(&all, r); memcpy(all.p + all.n, tmp, r); all.n += r; }
        fclose(fp);
        off[i] = all.n;
    }
    oracle_out o;
    oracle_run((const uint8_t*)all.p, off, (uint32_t)n, NULL, (uint64_t)n, &o);
    printf("-------------TF Job-------------\n");
    fwrite(o.tf_jobs, 1, o.tf_len, stdout);
    printf("------------IDF Job-------------\n");
    fwrite(o.idf_jobs, 1, o.idf_len, stdout);
    FILE* fo = fopen("output.txt", "w");
    if (!fo) { printf("Error Opening File: output.txt\n"); return 0; }    /* TFIDF.c:274-278 */
    fwrite(o.lines, 1, o.lines_len, fo);
    fclose(fo);
    oracle_free(&o);
    free(off); free(all.p);
    return 0;
}
#endif
