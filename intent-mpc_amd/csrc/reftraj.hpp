// reftraj.hpp -- mpcPlanner::getReferenceTraj / getXRef on the device (include/impc_mpc.h,
// impc_reference_traj_device), included by impc_qp.hip.  One thread per planning instance: a
// nearest-point search over the next 3 s of the instance's path from its last start index, then
// the horizon's points (padded with the path's last point) as the 8-state reference.
#pragma once

namespace impc_reftraj {

// one instance (reference mpcPlanner.cpp:1199-1231, getXRef :968-981)
__global__ void k_reference_traj(int32_t N, double ts, int64_t ni, const int64_t *__restrict__ path_ptr,
                                 const double *__restrict__ path, const double *__restrict__ cur,
                                 int32_t *__restrict__ last_idx, int32_t repeat, double *__restrict__ xref) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ni) return;
    const int64_t p0 = path_ptr[i], len = path_ptr[i + 1] - p0;
    const double *pp = path + 3 * p0;
    const double cx = cur[3 * i], cy = cur[3 * i + 1], cz = cur[3 * i + 2];
    int32_t start = 0;
    if (len > 0) {
        // int maxForwardIdx = maxForwardTime / ts_ (double -> int truncation; 3.0 / 0.1 -> 30)
        const double max_forward_time = 3.0;
        const int32_t max_forward_idx = (int32_t)(max_forward_time / ts);
        const int32_t last = last_idx[i];
        double least = 1.7976931348623157e308;  // std::numeric_limits<double>::max()
        start = last;
        const int64_t end = (int64_t)last + max_forward_idx < len ? (int64_t)last + max_forward_idx : len;
        for (int64_t j = last; j < end; j++) {
            const double dx = cx - pp[3 * j], dy = cy - pp[3 * j + 1], dz = cz - pp[3 * j + 2];
            const double d = sqrt((dx * dx + dy * dy) + dz * dz);  // (currPos_ - inputTraj_[i]).norm()
            if (d < least) {
                least = d;
                start = (int32_t)j;
            }
        }
        last_idx[i] = start;
    }
    for (int32_t r = 0; r < repeat; r++) {
        double *out = xref + ((i * repeat + r) * (int64_t)N) * 8;
        for (int32_t k = 0; k < N; k++) {
            double x = cx, y = cy, z = cz;
            if (len > 0) {
                const int64_t idx = (int64_t)start + k < len ? (int64_t)start + k : len - 1;
                x = pp[3 * idx];
                y = pp[3 * idx + 1];
                z = pp[3 * idx + 2];
            }
            double *o = out + 8 * k;
            o[0] = x;
            o[1] = y;
            o[2] = z;
            o[3] = o[4] = o[5] = o[6] = o[7] = 0.0;
        }
    }
}

}  // namespace impc_reftraj

extern "C" int impc_reference_traj_device(impc_ctx ctx, int32_t horizon, double ts, int64_t ni, const int64_t *path_ptr,
                                          const double *path, const double *curr_pos, int32_t *last_idx,
                                          int32_t repeat, double *xref, void *stream) {
    if (!ctx || horizon < 1 || !(ts > 0.0) || ni < 0 || repeat < 1 ||
        (ni > 0 && (!path_ptr || !curr_pos || !last_idx || !xref)))
        return fail(IMPC_INVALID_ARGUMENT, "invalid reference-trajectory arguments");
    if (ni == 0) return IMPC_OK;
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    IMPC_TRY(ctx_order_launch(ctx, st));
    const unsigned blocks = (unsigned)((ni + 255) / 256);
    hipLaunchKernelGGL(impc_reftraj::k_reference_traj, dim3(blocks), dim3(256), 0, st, horizon, ts, ni, path_ptr, path,
                       curr_pos, last_idx, repeat, xref);
    HIP_OK(hipGetLastError());
    return ctx_note_launch(ctx, st);
}

// ---------------------------------------------------------------- per-candidate row copies
namespace impc_reftraj {
// dst row r * repeat + c = src row r (8-byte words, one thread per word)
__global__ void k_repeat_rows(const double *__restrict__ src, int64_t rows, int64_t words, int32_t repeat,
                              double *__restrict__ dst) {
    const int64_t n = rows * words * repeat;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t w = t % words, rc = t / words, r = rc / repeat;
        dst[t] = src[r * words + w];
    }
}
// dst row r = src row idx[r] (T: 8- or 4-byte words)
template <class T>
__global__ void k_gather_rows(const T *__restrict__ src, int64_t words, const int64_t *__restrict__ idx, int64_t count,
                              T *__restrict__ dst) {
    const int64_t n = count * words;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t w = t % words, r = t / words;
        dst[t] = src[idx[r] * words + w];
    }
}
}  // namespace impc_reftraj

extern "C" int impc_gather_rows_device(impc_ctx ctx, const void *src, int64_t row_bytes, const int64_t *idx,
                                       int64_t count, void *dst, void *stream) {
    if (!ctx || count < 0 || row_bytes < 0 || (row_bytes & 3) || (count && row_bytes && (!src || !dst || !idx)))
        return fail(IMPC_INVALID_ARGUMENT, "invalid row-gather arguments (row_bytes a multiple of 4)");
    if (!count || !row_bytes) return IMPC_OK;
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    IMPC_TRY(ctx_order_launch(ctx, st));
    const bool w8 = (row_bytes & 7) == 0;
    const int64_t words = row_bytes / (w8 ? 8 : 4), n = count * words;
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, (int64_t)ctx->num_cu * 8);
    if (w8)
        hipLaunchKernelGGL(impc_reftraj::k_gather_rows<double>, dim3(blocks), dim3(256), 0, st, (const double *)src,
                           words, idx, count, (double *)dst);
    else
        hipLaunchKernelGGL(impc_reftraj::k_gather_rows<uint32_t>, dim3(blocks), dim3(256), 0, st,
                           (const uint32_t *)src, words, idx, count, (uint32_t *)dst);
    HIP_OK(hipGetLastError());
    return ctx_note_launch(ctx, st);
}

extern "C" int impc_repeat_rows_device(impc_ctx ctx, const void *src, int64_t rows, int64_t row_bytes, int32_t repeat,
                                       void *dst, void *stream) {
    if (!ctx || rows < 0 || row_bytes < 0 || (row_bytes & 7) || repeat < 1 || (rows && row_bytes && (!src || !dst)))
        return fail(IMPC_INVALID_ARGUMENT, "invalid row-repeat arguments (row_bytes a multiple of 8)");
    if (!rows || !row_bytes) return IMPC_OK;
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    IMPC_TRY(ctx_order_launch(ctx, st));
    const int64_t n = rows * (row_bytes / 8) * repeat;
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, (int64_t)ctx->num_cu * 8);
    hipLaunchKernelGGL(impc_reftraj::k_repeat_rows, dim3(blocks), dim3(256), 0, st, (const double *)src, rows,
                       row_bytes / 8, repeat, (double *)dst);
    HIP_OK(hipGetLastError());
    return ctx_note_launch(ctx, st);
}
