/*
 * impc_comm.h -- multi-GPU plumbing of the batched solver: an RCCL communicator
 * over xGMI for the one exchange the path has (every rank's per-QP cost records to every rank,
 * for hypothesis selection), and device-side step timing.
 *
 * The reference has no multi-process path: mpcPlanner::makePlanWithPred solves its candidates
 * serially in one thread (mpcPlanner.cpp:609-628).  The batched replacement shards planning
 * instances across GPUs (one process per GPU, no data-path collective); afterwards each rank's
 * impc_info records (64 bytes per QP: iterations, status, objective, residuals) are all-gathered
 * so every rank holds every hypothesis' cost.
 *
 * The communicator lives in this library, on the same HIP runtime as the solver (the launching
 * framework's own GPU runtime is never touched in a solver process); the 128-byte unique id is
 * exchanged by the caller over any host transport (torch.distributed gloo in bench.py).
 * Handles are not thread-safe; one communicator per context.
 */
#ifndef IMPC_COMM_H
#define IMPC_COMM_H

#include <stdint.h>

#include "impc_qp.h"

#ifdef __cplusplus
extern "C" {
#endif

#define IMPC_COMM_ID_BYTES 128

typedef struct impc_comm_s *impc_comm;

/* ncclGetUniqueId: called by rank 0, the bytes handed to every rank. */
int impc_comm_unique_id(unsigned char id[IMPC_COMM_ID_BYTES]);

/* ncclCommInitRank on the context's device (collective over all ranks). */
int impc_comm_create(impc_ctx ctx, const unsigned char id[IMPC_COMM_ID_BYTES], int rank, int world, impc_comm *out);

int impc_comm_destroy(impc_comm comm);

/* ncclAllGather of `bytes` bytes per rank: rank r's block lands at recv + r * bytes (device
 * pointers), enqueued on `stream` (the context stream when null), ordered after the solver's
 * launches on that stream. */
int impc_comm_allgather(impc_comm comm, const void *send, void *recv, int64_t bytes, void *stream);

/* The cost records of this rank's QPs to every rank: the impc_info arrays of `count` batches
 * (in order) are packed on the device into one block of `max_qps` records (zero padded), and one
 * ncclAllGather places rank r's block at recv + r * max_qps (recv: device, world * max_qps
 * records).  Ranks may hold different QP counts (max_qps >= every rank's sum of batch sizes). */
int impc_comm_gather_info(impc_comm comm, impc_batch *batches, int count, int64_t max_qps, impc_info *recv,
                          void *stream);

/* Max over ranks of a host double (ncclAllReduce, synchronous): the timed region's end. */
int impc_comm_max(impc_comm comm, double *value);

/* Step timing with HIP events on the launch stream (the context stream when null): each call
 * records one event; impc_ctx_timer_read synchronises and returns the elapsed ms between marks
 * 2k and 2k+1 (k < *pairs), then clears the marks. */
int impc_ctx_timer_mark(impc_ctx ctx, void *stream);
int impc_ctx_timer_read(impc_ctx ctx, double *ms, int64_t max_pairs, int64_t *pairs);

#ifdef __cplusplus
}
#endif

#endif
