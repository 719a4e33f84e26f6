// comm.hpp -- RCCL communicator and step timer of the C-ABI (include/impc_comm.h), included by
// impc_qp.hip (same translation unit: shares the context / batch types and error plumbing).
//
// The only cross-GPU exchange of the path is the all-gather of every QP's cost
// record after the solve.  Records are packed on the device (one D2D copy per batch into a
// staging block, zero padded to the largest rank's QP count) and moved by one ncclAllGather on the
// solver's stream -- tens of MB at most (262,144 x 64 B), latency-bound over xGMI.
#pragma once
#include <rccl/rccl.h>

struct impc_comm_s {
    impc_ctx ctx = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
    void *stage = nullptr;  // packed send block (grow-only)
    size_t stage_bytes = 0;
    double *scalar = nullptr;  // impc_comm_max scratch
};

#define NCCL_OK(expr)                                                                             \
    do {                                                                                          \
        ncclResult_t r_ = (expr);                                                                 \
        if (r_ != ncclSuccess) return fail(IMPC_DEVICE_ERROR, std::string(#expr ": ") + ncclGetErrorString(r_)); \
    } while (0)

extern "C" {

int impc_comm_unique_id(unsigned char id[IMPC_COMM_ID_BYTES]) {
    if (!id) return fail(IMPC_INVALID_ARGUMENT, "null id");
    static_assert(sizeof(ncclUniqueId) == IMPC_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    NCCL_OK(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof u);
    return IMPC_OK;
}

int impc_comm_create(impc_ctx ctx, const unsigned char id[IMPC_COMM_ID_BYTES], int rank, int world, impc_comm *out) {
    if (!ctx || !id || !out || world < 1 || rank < 0 || rank >= world)
        return fail(IMPC_INVALID_ARGUMENT, "invalid communicator arguments");
    *out = nullptr;
    HIP_OK(hipSetDevice(ctx->device));
    std::unique_ptr<impc_comm_s> c(new impc_comm_s());
    c->ctx = ctx;
    c->rank = rank;
    c->world = world;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    NCCL_OK(ncclCommInitRank(&c->comm, world, u, rank));
    HIP_OK(hipMalloc((void **)&c->scalar, 2 * sizeof(double)));
    *out = c.release();
    return IMPC_OK;
}

int impc_comm_destroy(impc_comm c) {
    if (!c) return IMPC_OK;
    (void)hipSetDevice(c->ctx->device);
    (void)ctx_quiesce(c->ctx);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->stage) (void)hipFree(c->stage);
    if (c->scalar) (void)hipFree(c->scalar);
    delete c;
    return IMPC_OK;
}

int impc_comm_allgather(impc_comm c, const void *send, void *recv, int64_t bytes, void *stream) {
    if (!c || bytes < 0 || (bytes && (!send || !recv))) return fail(IMPC_INVALID_ARGUMENT, "invalid all-gather");
    HIP_OK(hipSetDevice(c->ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->ctx->stream;
    IMPC_TRY(ctx_order_launch(c->ctx, st));
    NCCL_OK(ncclAllGather(send, recv, (size_t)bytes, ncclChar, c->comm, st));
    return ctx_note_launch(c->ctx, st);
}

int impc_comm_gather_info(impc_comm c, impc_batch *bs, int count, int64_t max_qps, impc_info *recv, void *stream) {
    if (!c || (count && !bs) || count < 0 || max_qps < 0 || !recv) return fail(IMPC_INVALID_ARGUMENT, "invalid gather");
    int64_t total = 0;
    for (int k = 0; k < count; k++) {
        if (!bs[k] || bs[k]->ctx != c->ctx) return fail(IMPC_INVALID_ARGUMENT, "batch of another context");
        total += bs[k]->B;
    }
    if (total > max_qps) return fail(IMPC_INVALID_ARGUMENT, "max_qps is smaller than this rank's QP count");
    HIP_OK(hipSetDevice(c->ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->ctx->stream;
    const size_t bytes = sizeof(impc_info) * (size_t)std::max<int64_t>(max_qps, 1);
    if (bytes > c->stage_bytes) {
        IMPC_TRY(ctx_quiesce(c->ctx));  // no gather in flight reads the old block
        if (c->stage) HIP_OK(hipFree(c->stage));
        c->stage = nullptr;
        HIP_OK(hipMalloc(&c->stage, bytes));
        c->stage_bytes = bytes;
    }
    // the solves that wrote d_info, and an earlier gather still reading the staging block, may
    // have run on other streams: wait for all of them
    IMPC_TRY(ctx_order_after_all(c->ctx, st));
    char *dst = (char *)c->stage;
    for (int k = 0; k < count; k++) {
        const size_t nb = sizeof(impc_info) * (size_t)bs[k]->B;
        HIP_OK(hipMemcpyAsync(dst, bs[k]->d_info, nb, hipMemcpyDeviceToDevice, st));
        dst += nb;
    }
    if (total < max_qps) HIP_OK(hipMemsetAsync(dst, 0, sizeof(impc_info) * (size_t)(max_qps - total), st));
    NCCL_OK(ncclAllGather(c->stage, recv, sizeof(impc_info) * (size_t)max_qps, ncclChar, c->comm, st));
    return ctx_note_launch(c->ctx, st);
}

int impc_comm_max(impc_comm c, double *value) {
    if (!c || !value) return fail(IMPC_INVALID_ARGUMENT, "invalid argument");
    HIP_OK(hipSetDevice(c->ctx->device));
    hipStream_t st = c->ctx->stream;
    IMPC_TRY(ctx_quiesce(c->ctx));
    HIP_OK(hipMemcpyAsync(c->scalar, value, sizeof(double), hipMemcpyHostToDevice, st));
    NCCL_OK(ncclAllReduce(c->scalar, c->scalar + 1, 1, ncclFloat64, ncclMax, c->comm, st));
    HIP_OK(hipMemcpyAsync(value, c->scalar + 1, sizeof(double), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    return IMPC_OK;
}

int impc_ctx_timer_mark(impc_ctx ctx, void *stream) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    hipEvent_t e = nullptr;
    HIP_OK(hipEventCreate(&e));
    ctx->timer_marks.push_back(e);
    HIP_OK(hipEventRecord(e, st));
    return IMPC_OK;
}

int impc_ctx_timer_read(impc_ctx ctx, double *ms, int64_t max_pairs, int64_t *pairs) {
    if (!ctx || !pairs || (max_pairs > 0 && !ms)) return fail(IMPC_INVALID_ARGUMENT, "invalid argument");
    HIP_OK(hipSetDevice(ctx->device));
    const int64_t np = (int64_t)ctx->timer_marks.size() / 2;
    int rc = IMPC_OK;
    for (int64_t k = 0; k < np && k < max_pairs && rc == IMPC_OK; k++) {
        float t = 0.f;
        hipEvent_t a = ctx->timer_marks[(size_t)(2 * k)], b = ctx->timer_marks[(size_t)(2 * k + 1)];
        hipError_t e = hipEventSynchronize(b);
        if (e == hipSuccess) e = hipEventElapsedTime(&t, a, b);
        if (e != hipSuccess) rc = fail(IMPC_DEVICE_ERROR, std::string("timer: ") + hipGetErrorString(e));
        ms[k] = (double)t;
    }
    for (hipEvent_t e : ctx->timer_marks) (void)hipEventDestroy(e);
    ctx->timer_marks.clear();
    *pairs = std::min(np, max_pairs);
    return rc;
}

}  // extern "C"
