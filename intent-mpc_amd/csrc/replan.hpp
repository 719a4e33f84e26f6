// replan.hpp -- the planner state a batched makePlanWithPred carries on the device between replans
// (include/impc_replan.h), included by impc_qp.hip.  One workgroup per committed instance: the
// plan's n values are copied by its lanes into the instance's warm start (plan_x) and states
// (plan_states), lane 0 sets the flags.  Reference: mpcPlanner.cpp:636-639 (fan-out branch) and
// :653-657 (single solve): currentStatesSol_ / currentControlsSol_ = the plan, firstTime_ = false.
#pragma once

namespace impc_replan_k {

__global__ __launch_bounds__(256) void k_commit(int32_t N, int64_t n, int64_t count, const int64_t *__restrict__ inst,
                                                const uint64_t *__restrict__ x_cand, int32_t ncand,
                                                const int32_t *__restrict__ best, const double *__restrict__ x_rows,
                                                const impc_info *__restrict__ info_rows, double *__restrict__ plan_x,
                                                double *__restrict__ plan_states, int32_t *__restrict__ prev_count,
                                                int8_t *__restrict__ first_time, int8_t *__restrict__ valid) {
    for (int64_t r = blockIdx.x; r < count; r += gridDim.x) {
        const int64_t i = inst[r];
        const double *src = nullptr;
        if (x_cand) {
            const int32_t c = best[r];
            if (c >= 0 && c < ncand) src = (const double *)x_cand[r * ncand + c];
        } else if (impc_lib::solve_traj_ok(info_rows[r])) {  // solveTraj's successSolve (:475-478, :513-518)
            src = x_rows + r * n;
        }
        if (src) {
            for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
                const double v = src[k];
                plan_x[i * n + k] = v;
                if (k < 8 * (int64_t)N) plan_states[i * 8 * (int64_t)N + k] = v;
            }
        }
        if (threadIdx.x == 0) {
            valid[i] = src ? 1 : 0;
            if (src) {
                first_time[i] = 0;
                prev_count[i] = N;
            }
        }
    }
}

}  // namespace impc_replan_k

extern "C" int impc_replan_commit_device(impc_ctx ctx, int32_t horizon, int64_t n, int64_t count, const int64_t *inst,
                                         const uint64_t *x_cand, int32_t ncand, const int32_t *best_cand,
                                         const double *x_rows, const impc_info *info_rows, double *plan_x,
                                         double *plan_states, int32_t *prev_count, int8_t *first_time, int8_t *valid,
                                         void *stream) {
    if (!ctx || horizon < 2 || n != 13 * (int64_t)horizon - 5 || count < 0)
        return fail(IMPC_INVALID_ARGUMENT, "replan commit: n must be 13 horizon - 5, count >= 0");
    if (!count) return IMPC_OK;
    if (!inst || !plan_x || !plan_states || !prev_count || !first_time || !valid ||
        (x_cand ? (!best_cand || ncand < 1 || x_rows) : (!x_rows || !info_rows)))
        return fail(IMPC_INVALID_ARGUMENT, "replan commit: one of x_cand (+ best_cand) or x_rows (+ info_rows)");
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    // after the solves and the selection, wherever they ran
    IMPC_TRY(ctx_order_after_all(ctx, st));
    const unsigned blocks = (unsigned)std::min<int64_t>(count, (int64_t)ctx->num_cu * 8);
    hipLaunchKernelGGL(impc_replan_k::k_commit, dim3(blocks), dim3(256), 0, st, horizon, n, count, inst, x_cand, ncand,
                       best_cand, x_rows, info_rows, plan_x, plan_states, prev_count, first_time, valid);
    HIP_OK(hipGetLastError());
    return ctx_note_launch(ctx, st);
}

// ---- a receding window's next initial state from the last solve (impc_batch_follow_plan_device)
namespace impc_replan_k {
// mpcPlanner::getPos / getVel (mpcPlanner.cpp:1257-1290) on QP b's own solution, for the QPs
// whose solve returned one; pos / vel [B][3] updated in place.  Deliberately narrower than
// solveTraj's success (impc_lib::solve_traj_ok, which the replan's commit uses): a receding window
// of raw QPs does not move its x0 to an OSQP_NAN plan (infeasible / diverged QPs), DESIGN.md 2
__global__ void k_follow(int64_t B, int32_t N, int64_t n, double ts, double t, const double *__restrict__ x,
                         const impc_info *__restrict__ info, double *__restrict__ pos, double *__restrict__ vel,
                         double *__restrict__ lin) {
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < B; b += (int64_t)gridDim.x * blockDim.x) {
        const int64_t st = info[b].status_val;
        if (st != IMPC_SOLVED && st != IMPC_SOLVED_INACCURATE && st != IMPC_MAX_ITER_REACHED &&
            st != IMPC_TIME_LIMIT_REACHED)
            continue;
        int idx = (int)floor(t / ts);
        const double dt = t - idx * ts;
        idx = max(0, min(idx, N - 1));
        const int nxt = min(idx + 1, N - 1);
        const double *s = x + b * n + 8 * idx, *e = x + b * n + 8 * nxt;
        for (int c = 0; c < 3; c++) {
            pos[3 * b + c] = s[c] + (e[c] - s[c]) / ts * dt;
            vel[3 * b + c] = s[3 + c] + (e[3 + c] - s[3 + c]) / ts * dt;
        }
        // currentStatesSol_: the next linearisation point (castMPCToQPConstraintMatrix :1042-1051)
        if (lin)
            for (int k = 0; k < 8 * N; k++) lin[b * 8 * (int64_t)N + k] = x[b * n + k];
    }
}
}  // namespace impc_replan_k

extern "C" int impc_batch_follow_plan_device(impc_batch b, int32_t horizon, double ts, double t, double *pos,
                                             double *vel, double *lin_states) {
    if (!b || horizon < 2 || b->n != 13 * (int64_t)horizon - 5 || !(ts > 0.0) || !(t >= 0.0) || !pos || !vel)
        return fail(IMPC_INVALID_ARGUMENT, "follow plan: an mpcPlanner batch (n = 13 horizon - 5), ts > 0, t >= 0");
    HIP_OK(hipSetDevice(b->ctx->device));
    hipStream_t st = b->ctx->stream;
    IMPC_TRY(ctx_order_after_all(b->ctx, st));  // after the solve, wherever it ran
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((b->Bact + 255) / 256, 4096));
    hipLaunchKernelGGL(impc_replan_k::k_follow, dim3(blocks), dim3(256), 0, st, b->Bact, horizon, b->n, ts, t, b->d_xout,
                       b->d_info, pos, vel, lin_states);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

extern "C" int impc_copy_rows_device(impc_ctx ctx, void *dst, int64_t dpitch, const void *src, int64_t spitch,
                                     int64_t width, int64_t rows, void *stream) {
    if (!ctx || rows < 0 || width < 0 || (rows && width && (!dst || !src || dpitch < width || spitch < width)))
        return fail(IMPC_INVALID_ARGUMENT, "copy rows: pitches >= width");
    if (!rows || !width) return IMPC_OK;
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    IMPC_TRY(ctx_order_launch(ctx, st));
    HIP_OK(hipMemcpy2DAsync(dst, (size_t)dpitch, src, (size_t)spitch, (size_t)width, (size_t)rows,
                            hipMemcpyDeviceToDevice, st));
    return ctx_note_launch(ctx, st);
}
