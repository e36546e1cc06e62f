/* kernels.h — parameter blocks and host launchers of the TF-IDF path kernels. */
#ifndef TFIDF_KERNELS_H
#define TFIDF_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "prims.h"

/* chunking (K0/K1) */
#define K1_NT        256                 /* threads per tokenize+count workgroup */
#define K1_WIN       (K1_NT * 16)        /* bytes per window: one 16-byte group per thread */
#ifndef CHUNK_BYTES
#define CHUNK_BYTES  12288u              /* nominal chunk (work unit) size: tokcount_vs / general
                                            (c4: 16 -> 12 KiB snapped to document starts keeps more
                                            chunks under the LDS table's fill limit: 8.2 M -> fewer
                                            partial records, merge 0.92 -> 0.68 ms, K1 +0.04 ms) */
#endif
#ifndef CHUNK_BYTES_ST
#define CHUNK_BYTES_ST 24576u            /* ... and tokcount_sl/st's: their per-chunk set-up, flush and
                                            barrier wait over 1.5x the bytes (c2 K1 -3 %, c5 -5 %) */
#endif
#ifndef DENSE_DOC
#define DENSE_DOC    (4ull << 20)        /* documents longer than this: dense merge of their partial records */
#endif
#define BIG_LIST_CAP 4096u               /* dense-merge candidates K0 lists */
#define DENSE_REP    16u                 /* copies of each dense per-document array (spreads hot-term atomics) */
#ifndef BIG_DOC
#define BIG_DOC      49152u              /* documents longer than this are split across chunks */
#endif
#ifndef K5_MAX_PAIRS
#define K5_MAX_PAIRS 4096                /* largest complete (unmerged) document K5 sorts in LDS */
#endif

/* status bits (device word) */
#define ST_VOCAB_FULL  1u
#define ST_VOCAB_SPIN  2u
#define ST_REC_FULL    4u
#define ST_PART_FULL   8u
#define ST_BOUNDS      16u   /* internal consistency guard tripped (a bug, reported as an error) */
#define ST_HAS_LONG    64u   /* the vocabulary holds terms of >= 16 bytes (their order needs vocab_long_fixup) */
#define ST_TERM_LONG   32u   /* a term of >= 16 MiB: beyond the 24-bit length of a long key's rep */
#define ST_LONG_COLLIDE 128u /* two distinct terms of >= 16 bytes share their 120-bit key (dev_vocab.h) */

/* doc flags */
#define DF_PARTIAL     1u
#define DF_PRESORTED   2u

#define INVALID_SLOT   0xFFFFFFFFu

struct CorpusDev {
    const uint8_t* bytes;
    uint64_t nbytes;
    const uint64_t* doc_off;   /* ndocs + 1 */
    uint32_t ndocs;
    uint64_t lo, hi;           /* doc_off[0], doc_off[ndocs] (host-known) */
};

struct VocabDev {
    uint4* keys;               /* cap identity keys (see dev_common.h) */
    uint64_t* rep;             /* long terms: (len << 40) | byte offset */
    uint64_t mask;             /* cap - 1 */
};

struct K1Out {
    uint32_t* rec_slot;        /* complete documents' (term slot, count) records */
    uint32_t* rec_cnt;
    unsigned long long* rec_alloc;
    uint64_t rec_cap;
    uint32_t* part_doc;        /* records of documents split across flushes/chunks */
    uint32_t* part_slot;
    uint32_t* part_cnt;
    unsigned long long* part_alloc;
    uint64_t part_cap;
    uint64_t* doc_recoff;
    uint32_t* doc_npairs;
    uint32_t* doc_size;
    uint8_t* doc_flags;
    uint32_t* status;
    unsigned long long* ntokens;
    unsigned long long* chunk_ctr;   /* K1 dynamic chunk schedule (zeroed per run) */
    unsigned long long* chunk_shard; /* tokcount_st: 8 sharded chunk counters (zeroed per run) */
    unsigned long long* stamps;  /* diagnostic build only: K1_NSTAMP phase cycle sums, WG count,
                                    then K1_NCOUNT event counters */
};
#define K1_NSTAMP 17
#define K1_NCOUNT 4   /* segments, flushes, tokens taking the full probe, probe iterations */
#define K1_STAMP_WORDS (K1_NSTAMP + 1 + K1_NCOUNT)
#define K1_DEBUG_WORDS 16384   /* diagnostic builds: the stamps buffer's size in u64 words */

/* K0: chunk boundaries; chunk_start has nchunks+1 entries, chunk_doc nchunks */
int launch_plan_chunks(const CorpusDev& c, uint64_t nchunks, uint32_t chunk_bytes, uint64_t* chunk_start,
                       uint32_t* chunk_doc, uint32_t* big_list, unsigned long long* big_ctr, hipStream_t s);
/* K1: tokenize + per-document term counts for chunks [c0, c1) */
int launch_tokcount(const CorpusDev& c, const uint64_t* chunk_start, const uint32_t* chunk_doc,
                    uint64_t c0, uint64_t c1, const VocabDev& v, const K1Out& o, hipStream_t s);

/* K1 round-1 path (tokcount_vs.hip): 16-byte aligned corpus base; returns -3 when the
 * vocabulary capacity exceeds the LDS entry's slot field */
int launch_tokcount_vs(const CorpusDev& c, const uint64_t* chunk_start, const uint32_t* chunk_doc, uint64_t c0,
                       uint64_t c1, const VocabDev& v, const K1Out& o, hipStream_t s);
#define K1_VS_MAX_CAP (1ull << 28)

#define K1_ST_MAX_CAP (1ull << 22)   /* tokcount_sl past this vocabulary capacity: half-size chunks */
#define K1_SL_MAX_CAP (1ull << 25)   /* the largest table tokcount_sl addresses (the default limit;
                                        TFIDF_SL_MAXCAP lowers it), tokcount_vs beyond */
/* K1 default (tokcount_sl.hip): one workgroup per chunk, straight-line rounds; the output
 * block is read from device memory (o_dev: a K1Out the engine copies there per run).
 * 16-byte aligned corpus base; -3 when the vocabulary exceeds K1_SL_MAX_CAP slots */
int launch_tokcount_sl(const CorpusDev& c, const uint64_t* chunk_start, const uint32_t* chunk_doc, uint64_t c0,
                       uint64_t c1, const VocabDev& v, const K1Out* o_dev, hipStream_t s);


/* vocabulary finalisation */
int launch_vocab_flags(const VocabDev& v, uint64_t cap, uint32_t* flags, hipStream_t s);
int launch_vocab_compact(const VocabDev& v, uint64_t cap, const uint32_t* dense_of_slot, const CorpusDev& c,
                         uint32_t* vslot, uint4* sortkey, uint32_t* seq, hipStream_t s);
/* large-V vocabulary sort as two u64 sorts: key halves (in seq order when seq != null) and
 * the sorted keys gathered back (long-term fix-up only) */
int launch_sortkey_half(const uint4* k, uint64_t n, const uint32_t* seq, int hi, uint64_t* out, hipStream_t s);
int launch_gather_u128(const uint4* k, const uint32_t* seq, uint64_t n, uint4* out, hipStream_t s);
/* several byte fills in one launch (a run's clears: one kernel instead of one per buffer);
 * each segment's base 16-byte aligned (device allocations are) */
constexpr int FILL_MAX = 8;
struct FillList {
    void* p[FILL_MAX];
    uint64_t bytes[FILL_MAX];
    uint32_t val[FILL_MAX];   /* the byte value, replicated */
    uint32_t n;
};
int launch_fill_multi(const FillList& l, hipStream_t s);
/* a few device words (4 or 8 bytes each) into pinned host memory in one launch (the run's
 * status reads: one small kernel instead of one copy per word) */
constexpr int WORDS_MAX = 16;
struct WordList {
    const void* src[WORDS_MAX];
    uint32_t bytes[WORDS_MAX];   /* 4 or 8 */
    uint32_t n;
    uint64_t token;              /* nonzero: written to dst[n] after the words (system-scope fence
                                    between): the host polls it instead of waiting on the stream */
};
int launch_words_to_host(const WordList& l, uint64_t* host_dst, hipStream_t s);
int launch_vocab_rank(const uint32_t* sorted_dense, const uint32_t* vslot, uint32_t V, uint32_t* rank_of_slot,
                      uint32_t* slot_of_rank, uint16_t* rank16, hipStream_t s);
/* long terms tied on their first 16 bytes: ordered by iterated segmented sorts (host loop,
 * one sync per 16 bytes of common prefix); -2 when the arena is too small */
/* the large-V sort's tie fix-up (finalize.hip): runs of equal first 8 bytes in the
 * prefix-sorted order re-ordered by the low halves (low_mask: their varying bytes) */
int launch_vocab_prefix_ties(const uint64_t* sorted_hi, uint32_t* sorted_dense, const uint4* skey, uint32_t V,
                             uint32_t low_mask, Arena& ar, hipStream_t s);
int launch_vocab_long_fixup(const uint4* sorted_keys, uint32_t* sorted_dense, const uint32_t* vslot,
                            const VocabDev& v, const CorpusDev& c, uint32_t V, Arena& ar, hipStream_t s);

/* partial documents: sort key (doc << 32 | rank) and merge */
int launch_part_keys(const uint32_t* part_doc, const uint32_t* part_slot, const uint32_t* rank_of_slot, uint64_t n,
                     uint64_t* keys, uint32_t* seq, hipStream_t s);
int launch_part_heads(const uint64_t* keys, uint64_t n, uint32_t* head, hipStream_t s);
int launch_part_merge(const uint64_t* keys, const uint32_t* seq, const uint32_t* part_cnt, const uint32_t* head_pos,
                      uint64_t n, const uint32_t* slot_of_rank, uint64_t rec_base, uint32_t* rec_slot,
                      uint32_t* rec_cnt, uint64_t* doc_recoff, uint32_t* doc_npairs, uint8_t* doc_flags,
                      hipStream_t s);
/* dense merge of the partial records of long documents (finalize.hip) */
int launch_part_dense(const uint32_t* part_doc, const uint32_t* part_slot, const uint32_t* part_cnt, uint64_t q,
                      const uint32_t* big_idx, const uint32_t* rank_of_slot, uint32_t V, uint32_t* dense,
                      uint64_t* keys, uint32_t* seq, uint32_t* cnt_out, uint32_t* nkeep, hipStream_t s);
int launch_set_big_idx(const uint32_t* big_list, uint32_t nb, uint32_t* big_idx, hipStream_t s);
int launch_dense_emit(const uint32_t* dense, uint32_t nb, uint32_t V, const uint32_t* big_list,
                      const uint32_t* slot_of_rank, uint64_t rec_base, uint32_t* merged_count, uint32_t* tile_cnt,
                      uint32_t* rec_slot, uint32_t* rec_cnt, uint64_t* doc_recoff, uint32_t* doc_npairs,
                      uint8_t* doc_flags, Arena& ar, hipStream_t s);

/* DF.  accumulate: add into df instead of overwriting it (the split DF of a run with
 * partial records, whose main records are counted beside the merge stage) */
int launch_df_hist(uint32_t* rec_slot, uint64_t nrec, const uint32_t* nrec_extra, uint64_t nrec_max,
                   const uint32_t* rank_of_slot, const uint16_t* rank16, uint32_t V, uint64_t slot_cap,
                   uint32_t* status, uint32_t* df, Arena& ar, hipStream_t s, bool accumulate = false);
/* device scratch launch_df_hist takes from its arena (an upper bound) */
size_t df_hist_scratch(uint64_t nrec_max, uint32_t V);
int launch_df_mark(const uint32_t* df, uint32_t V, uint32_t* present, hipStream_t s);
int launch_df_list(const uint32_t* present_scan, uint64_t nvals, uint32_t* vals, hipStream_t s);

/* documents: name order key and output */
int launch_doc_keys(const uint32_t* doc_ids, uint32_t ndocs, uint64_t* keys, uint32_t* seq, hipStream_t s);
int launch_gather_meta(const uint32_t* order, const uint32_t* doc_npairs, const uint64_t* doc_recoff,
                       const uint32_t* doc_size, const uint8_t* doc_flags, uint32_t ndocs, uint64_t* npairs_ord,
                       uint4* meta, hipStream_t s);
struct K5Args {
    const uint32_t* order;       /* docs in output order */
    const uint4* meta;           /* per output position: {recoff lo, hi, npairs | flags << 30, docSize} */
    const uint64_t* out_off;     /* per output position */
    const uint64_t* doc_recoff;
    const uint32_t* doc_npairs;
    const uint32_t* doc_size;
    const uint8_t* doc_flags;
    const uint32_t* rec_slot;
    const uint32_t* rec_cnt;
    const uint32_t* rank_of_slot;
    const uint32_t* df_of_rank;  /* global df */
    const uint32_t* idf_idx;     /* df value -> index into idf */
    const double* idf;
    double* idf_rank;            /* [nterms] scratch: idf of each term rank */
    uint32_t* large_list;        /* [ndocs] scratch: output positions left to k_score_large */
    uint32_t* large_count;
    uint32_t* cls_list;          /* [ndocs] scratch: output positions by kernel class — small documents
                                    (k_score_small), then the wave kernel's, then k_score_large's;
                                    null (wide ranks): the wave kernel takes every position */
    uint32_t* cls_off;           /* [3 * cls_nblk + 1] scratch: per-block class counts, scanned: the
                                    segments start at 0, [cls_nblk], [2 cls_nblk], end at [3 cls_nblk] */
    uint32_t cls_nblk;
    uint2* split_tasks;          /* (output position, chunk) of presorted documents over K5_PS_SPLIT pairs */
    uint32_t* split_count;       /*   null: k_score_large emits them whole */
    uint32_t split_cap;
    uint32_t ndocs;
    uint32_t nterms;
    uint32_t rank_bits;          /* bits of the largest term rank (radix passes) */
    uint32_t idf_by_df;          /* 1: the score kernels read idf[df_of_rank[r]] (large V with a full idf
                                    table: a 4-byte gather into V words + an L2-resident table instead of
                                    an 8-byte gather into V doubles; idf_rank is not built) */
    uint64_t rec_total;          /* bounds guard: records in rec_slot/rec_cnt */
    uint64_t slot_cap;           /* bounds guard: vocabulary capacity */
    uint32_t* status;            /* ST_BOUNDS set instead of faulting */
    uint32_t* out_term;          /* output order: term rank */
    uint32_t* out_cnt;           /*               wordCount */
    double* out_score;           /*               tf * idf */
};
int launch_score_order(const K5Args& a, Arena& ar, hipStream_t s, hipStream_t s2, hipEvent_t ev_fork,
                       hipEvent_t ev_join);

/* multi-GPU vocabulary agreement */
int launch_keys_by_rank(const uint4* vkeys, const uint32_t* slot_of_rank, uint32_t V, uint4* out, hipStream_t s);
/* hash-owner DF exchange: partition this rank's terms by owner into 20-byte (key, df)
 * records (cnt[R] = terms per owner, cur[R] scratch); the send/receive segment offsets from
 * the all-gathered count matrix m (R rows of R counts + 1 status word); aggregate the
 * received records on the owner (table of tcap = 2^k >= 1.5 n slots; *used = distinct keys)
 * and reply per sender (segment + one trailer word = *used); write the returned global df at
 * the term ranks and global V (the trailers summed) to *vg */
/* where the partition reads this rank's term keys: the vocabulary sort's own keys in rank
 * order (skey[r] = the strcmp sort key of term rank r), not a gather through the slot table.
 * A short term's sort key is its identity key byte-swapped; a long term's identity key is
 * read from vkeys at its slot */
struct OwnerKeySrc {
    const uint4* skey;
    const uint32_t* slot_of_rank;   /* long terms */
    const uint4* vkeys;
};
int launch_owner_partition(const OwnerKeySrc& ks, const uint32_t* df, uint32_t V, uint32_t R, uint32_t* cnt, uint32_t* cur,
                           uint32_t* srec, uint32_t* sidx, hipStream_t s);
int launch_owner_offsets(const uint32_t* m, uint32_t R, uint32_t me, uint32_t* soff, uint32_t* roff, hipStream_t s);
int launch_owner_aggregate(const uint32_t* rrec, uint64_t n, const uint32_t* roff, uint32_t R, uint4* tkey, uint64_t tcap,
                           uint32_t* tdf, uint32_t* rslot, uint32_t* reply, unsigned long long* used, uint32_t* status,
                           hipStream_t s);
/* the same, bucketed: records grouped by key hash into buckets of <= 512 on average (a radix sort of
 * (bucket, record index) pairs), each bucket aggregated in LDS; scratch of
 * owner_bucket_scratch(n) bytes */
size_t owner_bucket_scratch(uint64_t n);
int launch_owner_aggregate_buckets(const uint32_t* rrec, uint64_t n, const uint32_t* roff, uint32_t R, void* scratch,
                                   size_t scratch_bytes, uint32_t* reply, unsigned long long* used, uint32_t* status,
                                   uint32_t stage_max, hipStream_t s);
int launch_owner_back(const uint32_t* back, const uint32_t* soff, uint32_t R, const uint32_t* sidx, uint32_t V,
                      uint32_t* df_global, uint32_t* vg, hipStream_t s);
/* out[i] = sum of rows[r * n + i] over r < nrows (the in-process transport's all-reduce) */
int launch_sum_rows_u32(const uint32_t* rows, uint32_t nrows, uint64_t n, uint32_t* out, hipStream_t s);
/* the in-process transport's collectives between contexts on one device, one launch each:
 * XCOPY_MAX segments of 4-byte words copied src[i] -> dst[i] (words[i] each) */
#define XCOPY_MAX 64
struct XCopyList {
    const uint32_t* src[XCOPY_MAX];
    uint32_t* dst[XCOPY_MAX];
    uint64_t off[XCOPY_MAX + 1];   /* prefix sums of the segments' word counts */
    uint32_t n;
};
int launch_xcopy(const XCopyList& l, hipStream_t s);
/* out[i] = sum over r < n of src[r][lo + i], i < len (a reduce-scatter slice) */
int launch_xsum_slice(const XCopyList& l, uint64_t lo, uint64_t len, uint32_t* out, hipStream_t s);
/* dense DF exchange (small vocabularies): gathered keys -> shared positions (tpos[slot] =
 * smallest gathered position of the key, *used = distinct keys), this rank's df scattered
 * over them (pos[r] = position of term rank r), and read back after the all-reduce */
int launch_dense_ids(const uint4* gkeys, uint64_t n, uint4* tkey, uint32_t* tpos, uint64_t tcap,
                     unsigned long long* used, uint32_t* status, hipStream_t s);
int launch_dense_scatter(const uint4* mine, const uint32_t* df, uint32_t V, const uint4* tkey, uint64_t tcap,
                         const uint32_t* tpos, uint32_t* pos, uint32_t* dense, uint32_t* status, hipStream_t s);
int launch_dense_gather(const uint32_t* dense, const uint32_t* pos, uint32_t V, uint32_t* df_global, hipStream_t s);
/* the same with merge numbering when no rank holds long terms (lists in term order, padded
 * with all-ones keys): pos = the keys below each term over all lists; lbm: R x V words;
 * dense[sumv] accumulates the keys first held by each rank (global V after the sum) */
int launch_dense_merge_ids(const uint4* gkeys, uint64_t maxv, uint32_t R, uint32_t me, uint32_t V, uint32_t* lbm,
                           const uint32_t* df, uint64_t sumv, uint32_t* pos, uint32_t* dense, hipStream_t s);

/* Cross-rank identity of terms of >= 16 bytes (engine.cpp exchange_long_check; TFIDF.c:229's
 * strcmp): a long term's identity key is a 120-bit hash, so the ranks all-gather their long
 * terms (key, length, bytes) and every rank checks each key two ranks share byte by byte. */
struct LongEnt {
    uint4 key;
    uint32_t len, pad;
    uint64_t boff;             /* its bytes in the rank's blob */
};
/* this rank's long terms: ents[0, cnt[0]) (blob offsets from an atomic byte counter cnt[1]),
 * src[e] = the corpus offset of one occurrence (the vocabulary's rep) */
int launch_long_list(const uint4* vkeys, const uint64_t* vrep, const uint32_t* slot_of_rank, uint32_t V, LongEnt* ents,
                     uint64_t* src, unsigned long long* cnt, hipStream_t s);
int launch_long_bytes(const LongEnt* ents, const uint64_t* src, uint32_t n, const uint8_t* bytes, uint8_t* blob,
                      hipStream_t s);
/* every gathered entry (R blocks of lcap, blobs of bcap bytes each; padding keys EMPTY)
 * compared with the first entry of its key: a different length or byte sets ST_LONG_COLLIDE */
int launch_long_verify(const LongEnt* g, uint64_t n, uint64_t lcap, const uint8_t* gblob, uint64_t bcap, uint4* tkey,
                       uint32_t* tpos, uint64_t tcap, uint32_t* status, hipStream_t s);

/* synthetic corpus generation on the device */
struct SynSpecDev;
int launch_synth_bytes(const void* spec, const uint32_t* doc_ids, const uint64_t* ntok, const uint64_t* blk_first,
                       uint64_t nblocks, uint32_t ndocs, uint64_t* blk_bytes, hipStream_t s);
int launch_synth_fill(const void* spec, const uint32_t* doc_ids, const uint64_t* ntok, const uint64_t* blk_first,
                      uint64_t nblocks, uint32_t ndocs, const uint64_t* blk_off, uint8_t* bytes, uint64_t* doc_off,
                      hipStream_t s);

/* ---- output emission (emit.hip) ---- */
struct EmitLaunch {
    const uint32_t* order;
    const uint32_t* doc_ids;
    const uint64_t* out_off;
    const uint32_t* term;
    const double* score;
    const uint4* tkey;
    const uint32_t* tlen;
    const uint8_t* corpus;
    uint32_t ndocs;
    uint32_t* status;
};
int launch_term_meta(const uint4* vkeys, const uint64_t* vrep, const uint32_t* slot_of_rank, uint32_t V,
                     uint4* tkey, uint32_t* tlen, hipStream_t s);
int launch_emit_bytes(const EmitLaunch& e, uint64_t* doc_bytes, hipStream_t s);
/* formats the output positions [d0, d1) (default: all) */
int launch_emit_write(const EmitLaunch& e, const uint64_t* doc_text, uint8_t* text, hipStream_t s, uint32_t d0 = 0,
                      uint32_t d1 = 0xFFFFFFFFu);
int launch_format_f64(const double* v, uint64_t n, uint8_t* out, uint32_t* status, hipStream_t s);

#endif
