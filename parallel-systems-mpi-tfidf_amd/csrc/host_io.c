/*
 * host_io.c — host-side pieces of libtfidf_hip.so: reference input contract (ingest),
 * output emission and host synthetic generation.  Plain C.
 *
 *   tfidf_ingest_dir    TFIDF.c:98-110 (N = entries of input/ minus "." and ".."),
 *                       TFIDF.c:130-139 (documents input/doc1..docN, error on missing)
 *   tfidf_write_output  TFIDF.c:245 ("%s@%s\t%.16f"), TFIDF.c:274-282 (output.txt)
 *   tfidf_print_jobs    TFIDF.c:199-205 (TF Job), TFIDF.c:236-239 (IDF Job)
 */
#include <dirent.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/tfidf.h"
#include "synth.h"

const char* tfidf_strerror(int s) {
    switch (s) {
    case TFIDF_OK: return "ok";
    case TFIDF_E_INVAL: return "invalid argument";
    case TFIDF_E_NOMEM: return "out of memory";
    case TFIDF_E_HIP: return "HIP runtime error";
    case TFIDF_E_RCCL: return "RCCL error";
    case TFIDF_E_NODEV: return "no gfx950 device";
    case TFIDF_E_NOINPUT: return "Directory failed to open";
    case TFIDF_E_NODOC: return "Error Opening File";
    case TFIDF_E_OUTPUT: return "Error Opening File: output.txt";
    case TFIDF_E_CAPACITY: return "capacity exceeded";
    case TFIDF_E_STATE: return "call out of order";
    case TFIDF_E_PEER: return "another rank failed";
    default: return "unknown error";
    }
}

int tfidf_abi_version(void) { return TFIDF_ABI_VERSION; }

void tfidf_free(void* p) { free(p); }

int tfidf_ingest_dir(const char* dir, uint8_t** bytes, uint64_t* nbytes,
                     uint64_t** doc_off, uint32_t* ndocs, uint32_t* bad_doc) {
    if (!dir || !bytes || !nbytes || !doc_off || !ndocs) return TFIDF_E_INVAL;
    DIR* d = opendir(dir);
    if (!d) return TFIDF_E_NOINPUT;
    uint64_t n = 0;
    struct dirent* e;
    while ((e = readdir(d)) != NULL) {
        if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
        ++n;
    }
    closedir(d);
    uint64_t* off = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    if (!off) return TFIDF_E_NOMEM;
    /* pass 1: sizes */
    size_t plen = strlen(dir) + 32;
    char* path = (char*)malloc(plen);
    off[0] = 0;
    for (uint64_t i = 1; i <= n; ++i) {
        snprintf(path, plen, "%s/doc%llu", dir, (unsigned long long)i);
        FILE* fp = fopen(path, "rb");
        if (!fp) {
            if (bad_doc) *bad_doc = (uint32_t)i;
            *ndocs = (uint32_t)n;
            free(off); free(path);
            return TFIDF_E_NODOC;
        }
        fseek(fp, 0, SEEK_END);
        long sz = ftell(fp);
        fclose(fp);
        off[i] = off[i - 1] + (uint64_t)(sz > 0 ? sz : 0);
    }
    uint8_t* buf = (uint8_t*)malloc(off[n] ? off[n] : 1);
    if (!buf) { free(off); free(path); return TFIDF_E_NOMEM; }
    for (uint64_t i = 1; i <= n; ++i) {
        snprintf(path, plen, "%s/doc%llu", dir, (unsigned long long)i);
        FILE* fp = fopen(path, "rb");
        if (!fp) {
            if (bad_doc) *bad_doc = (uint32_t)i;
            *ndocs = (uint32_t)n;
            free(off); free(path); free(buf);
            return TFIDF_E_NODOC;
        }
        uint64_t want = off[i] - off[i - 1];
        size_t got = fread(buf + off[i - 1], 1, (size_t)want, fp);
        fclose(fp);
        if (got != want) { free(off); free(path); free(buf); return TFIDF_E_NODOC; }
    }
    free(path);
    *bytes = buf;
    *nbytes = off[n];
    *doc_off = off;
    *ndocs = (uint32_t)n;
    return TFIDF_OK;
}

/* "doc%u@<word>\t%.16f\n" — the %.16f conversion is glibc's (exact binary->decimal,
 * round-half-even), identical to the reference's sprintf (TFIDF.c:245). */
int tfidf_write_output(const tfidf_result* r, const char* path) {
    if (!r || !path) return TFIDF_E_INVAL;
    FILE* fp = fopen(path, "w");
    if (!fp) return TFIDF_E_OUTPUT;
    static char buf[1 << 20];
    setvbuf(fp, NULL, _IOFBF, 1 << 22);
    size_t n = 0;
    for (uint64_t i = 0; i < r->npairs; ++i) {
        uint32_t t = r->pair_term[i];
        uint64_t wo = r->term_off[t], wl = r->term_off[t + 1] - wo;
        if (n + wl + 96 > sizeof buf) { fwrite(buf, 1, n, fp); n = 0; }
        if (wl + 96 > sizeof buf) { fclose(fp); return TFIDF_E_INVAL; }
        n += (size_t)snprintf(buf + n, 32, "doc%u@", r->pair_doc[i]);
        memcpy(buf + n, r->term_bytes + wo, (size_t)wl);
        n += (size_t)wl;
        n += (size_t)snprintf(buf + n, 64, "\t%.16f\n", r->pair_score[i]);
    }
    fwrite(buf, 1, n, fp);
    fclose(fp);
    return TFIDF_OK;
}

int tfidf_print_jobs(const tfidf_result* r) {
    if (!r) return TFIDF_E_INVAL;
    for (int pass = 0; pass < 2; ++pass) {
        fputs(pass == 0 ? "-------------TF Job-------------\n" : "------------IDF Job-------------\n", stdout);
        for (uint64_t i = 0; i < r->npairs; ++i) {
            uint32_t t = r->pair_term[i];
            uint64_t wo = r->term_off[t], wl = r->term_off[t + 1] - wo;
            fwrite(r->term_bytes + wo, 1, (size_t)wl, stdout);
            if (pass == 0)
                printf("@doc%u\t%u/%u\n", r->pair_doc[i], r->pair_count[i], r->pair_docsize[i]);
            else
                printf("@doc%u\t%llu/%u\n", r->pair_doc[i], (unsigned long long)r->ndocs_total, r->pair_df[i]);
        }
    }
    return TFIDF_OK;
}

static uint64_t syn_gcd(uint64_t a, uint64_t b) { while (b) { uint64_t t = a % b; a = b; b = t; } return a; }

/* shared by host and device generation: fills the spec (perm_a chosen coprime to V) */
void tfidf_synth_spec(syn_spec* s, uint64_t seed, uint32_t V, uint32_t mode, const double* cdf) {
    memset(s, 0, sizeof(*s));
    s->seed = seed;
    s->V = V;
    s->m = syn_digits26(V);
    s->mode = mode;
    s->cdf = cdf;
    uint64_t a = (syn_mix64(seed ^ 0xA11CEull) % (V ? V : 1)) | 1u;
    if (a < 2) a = 1;
    while (V > 1 && syn_gcd(a, V) != 1) ++a;
    s->perm_a = V > 1 ? a : 1;
    s->perm_b = V ? syn_mix64(seed ^ 0xB0Bull) % V : 0;
}

int tfidf_synth_host(uint64_t seed, uint32_t V, uint32_t mode, const double* cdf,
                     const uint32_t* doc_ids, const uint64_t* ntok, uint32_t ndocs,
                     uint8_t* bytes, uint64_t* nbytes, uint64_t* doc_off) {
    if (!ntok || !nbytes || V == 0 || (mode == SYN_MODE_ZIPF && !cdf)) return TFIDF_E_INVAL;
    syn_spec s;
    tfidf_synth_spec(&s, seed, V, mode, cdf);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < ndocs; ++i) {
        uint64_t id = doc_ids ? doc_ids[i] : (uint64_t)i + 1;
        uint64_t nb = (ntok[i] + SYN_BLOCK_TOKENS - 1) / SYN_BLOCK_TOKENS;
        if (doc_off) doc_off[i] = pos;
        for (uint64_t b = 0; b < nb; ++b) {
            pos += bytes ? syn_block_fill(&s, id, ntok[i], b, bytes + pos)
                         : syn_block_bytes(&s, id, ntok[i], b);
        }
    }
    if (doc_off) doc_off[ndocs] = pos;
    *nbytes = pos;
    return TFIDF_OK;
}
