/*
 * xport.h — the collectives of the DF exchange, behind one small interface.
 *
 * The reference combines per-rank DF with MPI_Reduce(CustomReduce) + MPI_Bcast
 * (TFIDF.c:209-222,291-326) between OS processes.  Here a context (one GPU shard) talks
 * to its peers through an Xport:
 *
 *   RcclXport   ncclAllGather / ncclAllReduce / grouped ncclSend-ncclRecv over xGMI: one
 *               communicator rank per GPU,
 *               either one process per GPU (tfidf_comm_init, torch.distributed launch) or
 *               one process driving every GPU (tfidf_group_open, ncclCommInitAll).
 *   LocalXport  contexts of one process that share a device (tfidf_group_open with a
 *               device listed twice, e.g. K shards on the 1-GPU test box): the same
 *               operations as device-to-device copies between the contexts' buffers, with
 *               host barriers.  The engine code above the interface is identical, so the
 *               owner partition / aggregate / reply kernels and the status agreement run
 *               unchanged with K > 1 ranks on one GPU.
 *
 * Every operation is collective: all ranks call it in the same order.  `words` is the
 * host-level agreement step (status + sizes), the device operations are stream-ordered.
 */
#ifndef TFIDF_XPORT_H
#define TFIDF_XPORT_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

struct tfidf_ctx;

struct Xport {
    int rank = 0, nranks = 1;
    virtual ~Xport() {}
    /* host all-gather of two u64 per rank: all[2 * r + k] = rank r's mine[k] */
    virtual int words(const uint64_t mine[2], uint64_t* all, hipStream_t s) = 0;
    /* device all-gather: recv[r * bytes ...] = rank r's send[0 .. bytes) */
    virtual int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
    /* device all-to-all with per-peer counts of `eb`-byte elements (host arrays of nranks):
     * this rank's elements for peer p are send[so[p] .. so[p] + scnt[p]) and peer p's for
     * this rank land at recv[ro[p] ..), so, ro the exclusive prefix sums of scnt, rcnt
     * (rcnt[p] must equal peer p's scnt[rank]) */
    virtual int alltoallv(const void* send, const uint64_t* scnt, void* recv, const uint64_t* rcnt, size_t eb,
                          hipStream_t s) = 0;
    /* device all-reduce (sum) of n u32 in place: the dense DF exchange's one collective */
    virtual int allreduce_u32(uint32_t* buf, size_t n, hipStream_t s) = 0;
    /* waits for the stream's work, collectives among it.  RcclXport polls, so that an abort
     * of the clique releases a rank waiting for a failed peer's part (TFIDF_E_PEER) */
    virtual int wait(hipStream_t s) { return hipStreamSynchronize(s) == hipSuccess ? 0 : -3 /* TFIDF_E_HIP */; }
    /* a rank failed between collectives: release the peers (they return errors) */
    virtual void abort() = 0;
    virtual const char* name() const = 0;
};

/* engine.cpp: attach (and take ownership of) an Xport; nullptr detaches */
int tfidf_ctx_attach_xport(tfidf_ctx* ctx, Xport* xp);
int tfidf_ctx_device(const tfidf_ctx* ctx);
hipStream_t tfidf_ctx_stream(const tfidf_ctx* ctx);

/* engine.cpp: hipMalloc counted in tfidf_run_info.device_allocs / device_alloc_bytes */
hipError_t tfidf_dev_malloc(void** p, size_t bytes);

/* group.cpp */
/* a process-per-GPU rank: non-blocking ncclCommInitRankConfig with the job's unique id */
int rccl_init_rank(const void* unique_id, int rank, int nranks, int device, Xport** out);

#endif
