// mpc_build.hpp -- on-device MPC -> QP assembly (include/impc_mpc.h, impc_mpc_build_values_device),
// included by impc_qp.hip.  Restates the instance-dependent part of mpcPlanner's
// castMPCToQPGradient (:952-966), castMPCToQPConstraintMatrix obstacle rows (:1040-1071),
// castMPCToQPConstraintVectors (:1074-1146) and updateObstacleParam (:1148-1197); everything
// else is copied from templates the host builder produced for the shape.
#pragma once

struct impc_mpc_builder_s {
    impc_ctx ctx = nullptr;
    impc_mpc_params p{};
    int32_t S = 0, Kd = 0, K = 0, L = 1, N = 0, W = 0;
    int64_t n = 0, m = 0, nnzP = 0, nnzA = 0, obs_off = 0;
    double *d_tPx = nullptr, *d_tAx = nullptr, *d_tl = nullptr, *d_tu = nullptr;
    int32_t *d_slot = nullptr;
};

namespace impc_build {

struct Args {
    int64_t nb, n, m, nnzP, nnzA, obs_off;
    int32_t N, W, S, Kd, K, L;
    double dsafe, ssafe, qpos, qvel;
    const double *tPx, *tAx, *tl, *tu;
    const int32_t *slot;
    const double *cp, *cv, *xref, *ls, *stc, *sts, *sty, *dp, *ds;
    double *Px, *q, *Ax, *l, *u;
    // replan rows (impc_lib::build_rows, replan_run.hip): the row count in device memory (rows >=
    // *dcount are not built), each row's planning instance (x0, reference, linearisation point
    // and static obstacles are per-instance arrays, indexed by row_inst[b]) and each dynamic obstacle's source:
    // osrc[b][j] = (offset << 1) | held -- held = 0: the trajectory at dp / ds + offset, step
    // stride 3 (a prediction); held = 1: the position at hp / hs + offset for every stage (a
    // current obstacle, updateDynamicObstacles :316-341).  All null: the plain layouts above.
    const int64_t *dcount = nullptr;
    const int32_t *row_inst = nullptr;
    const int64_t *osrc = nullptr;
    const double *hp = nullptr, *hs = nullptr;
};

// ((std::pow(v, 2)) with glibc's correctly rounded pow is exactly the rounded product v * v)
__device__ inline double sq(double v) { return v * v; }

__global__ __launch_bounds__(256) void k_build(Args a) {
#pragma clang fp contract(off)
    const int64_t nb = a.dcount ? (*a.dcount < a.nb ? *a.dcount : a.nb) : a.nb;
    for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const int t0 = (int)threadIdx.x;
        const int64_t ib = a.row_inst ? (int64_t)a.row_inst[b] : b;  // per-instance inputs
        double *Px = a.Px + b * a.nnzP, *Ax = a.Ax + b * a.nnzA, *q = a.q + b * a.n, *l = a.l + b * a.m,
               *u = a.u + b * a.m;
        for (int64_t e = t0; e < a.nnzP; e += blockDim.x) Px[e] = a.tPx[e];
        for (int64_t e = t0; e < a.nnzA; e += blockDim.x) Ax[e] = a.tAx[e];
        for (int64_t r = t0; r < a.m; r += blockDim.x) {
            l[r] = a.tl[r];
            u[r] = a.tu[r];
        }
        // castMPCToQPGradient: q_state = Q * (-xRef), controls 0
        const double *xr = a.xref + ib * (int64_t)a.N * 8;
        for (int64_t k = t0; k < a.n; k += blockDim.x) {
            double v = 0.0;
            if (k < (int64_t)8 * a.N) {
                const int d = (int)(k % 8);
                const double Qd = d < 3 ? a.qpos : d < 6 ? a.qvel : d == 6 ? 100.0 : 1000.0;
                v = Qd * (-xr[k]);
            }
            q[k] = v;
        }
        __syncthreads();
        // x0 rows (:1082-1086): l = u = -x0 on the first 8 rows
        if (t0 < 8) {
            const double x0 = t0 < 3 ? a.cp[3 * ib + t0] : t0 < 6 ? a.cv[3 * ib + t0 - 3] : 0.0;
            l[t0] = -x0;
            u[t0] = -x0;
        }
        // obstacle rows, one (stage i, obstacle j) per thread
        for (int t = t0; t < a.W * a.K; t += blockDim.x) {
            const int i = t / a.K, j = t % a.K;
            double ox, oy, oz, sx, sy, sz, yaw;
            if (j < a.Kd) {  // dynamic first (:1153), prediction clamped to .back()
                const int jj = i < a.L ? i : a.L - 1;
                const double *pp, *ps;
                if (a.osrc) {
                    const int64_t o = a.osrc[b * a.Kd + j], off = o >> 1;
                    pp = (o & 1) ? a.hp + off : a.dp + off + (int64_t)jj * 3;
                    ps = (o & 1) ? a.hs + off : a.ds + off + (int64_t)jj * 3;
                } else {
                    pp = a.dp + (((int64_t)b * a.Kd + j) * a.L + jj) * 3;
                    ps = a.ds + (((int64_t)b * a.Kd + j) * a.L + jj) * 3;
                }
                ox = pp[0], oy = pp[1], oz = pp[2];
                sx = ps[0] / 2 + a.dsafe, sy = ps[1] / 2 + a.dsafe, sz = ps[2] / 2 + a.dsafe;
                yaw = 0.0;
            } else {
                const int js = j - a.Kd;
                const double *c = a.stc + (ib * a.S + js) * 3, *z = a.sts + (ib * a.S + js) * 3;
                ox = c[0], oy = c[1], oz = c[2];
                sx = z[0] / 2 + a.ssafe, sy = z[1] / 2 + a.ssafe, sz = z[2] / 2 + a.ssafe;
                yaw = a.sty[ib * a.S + js];
            }
            double cx, cy, cz;  // linearisation point (:1042-1051)
            if (a.ls) {
                const double *ls = a.ls + (ib * (int64_t)a.N + i) * 8;
                cx = ls[0], cy = ls[1], cz = ls[2];
            } else {
                cx = a.cp[3 * ib], cy = a.cp[3 * ib + 1], cz = a.cp[3 * ib + 2];
            }
            const double cyw = cos(yaw), syw = sin(yaw);
            const double fxx = 2 * ((cx - ox) * cyw + (cy - oy) * syw) / sq(sx) * cyw +
                               2 * (-(cx - ox) * syw + (cy - oy) * cyw) / sq(sy) * (-syw);
            const double fyy = 2 * ((cx - ox) * cyw + (cy - oy) * syw) / sq(sx) * syw +
                               2 * (-(cx - ox) * syw + (cy - oy) * cyw) / sq(sy) * (cyw);
            const double fzz = 2 * ((cz - oz)) / sq(sz);
            const double fxyz = sq((cx - ox) * cyw + (cy - oy) * syw) / sq(sx) +
                                sq(-(cx - ox) * syw + (cy - oy) * cyw) / sq(sy) + sq((cz - oz)) / sq(sz);
            const int32_t *sl = a.slot + 4 * t;
            Ax[sl[0]] = fxx;
            Ax[sl[1]] = fyy;
            Ax[sl[2]] = fzz;
            l[a.obs_off + t] = 1 - fxyz + fxx * cx + fyy * cy + fzz * cz;
        }
        __syncthreads();
    }
}

}  // namespace impc_build

extern "C" int impc_mpc_builder_create(impc_ctx ctx, const impc_mpc_params *p, int32_t num_static, int32_t num_dynamic,
                                       int32_t pred_len, impc_mpc_builder *out) {
    if (!ctx || !p || !out) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (num_dynamic > 0 && pred_len < 1) return fail(IMPC_INVALID_ARGUMENT, "pred_len must be >= 1");
    impc_qp_dims dm;
    if (impc_mpc_dims(p, num_static, num_dynamic, &dm)) return fail(IMPC_INVALID_ARGUMENT, "invalid MPC shape");
    std::unique_ptr<impc_mpc_builder_s> b(new impc_mpc_builder_s());
    b->ctx = ctx;
    b->p = *p;
    b->S = num_static, b->Kd = num_dynamic, b->K = num_static + num_dynamic, b->L = std::max(1, pred_len);
    b->N = p->horizon, b->W = p->horizon - 1;
    b->n = dm.n, b->m = dm.m, b->nnzP = dm.nnzP, b->nnzA = dm.nnzA;
    std::vector<int64_t> slots;
    if (impc_mpc_obstacle_layout(p, num_static, num_dynamic, slots, b->obs_off))
        return fail(IMPC_INVALID_ARGUMENT, "invalid MPC shape");
    // templates: the host builder on one neutral instance (its instance-dependent entries are
    // overwritten by the kernel)
    const int N = b->N, S = b->S, Kd = b->Kd, L = b->L;
    std::vector<double> z3(3, 0.0), xr((size_t)N * 8, 0.0), sc((size_t)S * 3, 0.0), ss((size_t)S * 3, 1.0),
        sy((size_t)S, 0.0), dp((size_t)Kd * L * 3, 0.0), ds((size_t)Kd * L * 3, 1.0);
    std::vector<double> Px((size_t)b->nnzP), q((size_t)b->n), Ax((size_t)b->nnzA), l((size_t)b->m), u((size_t)b->m);
    if (impc_mpc_build_values(p, 1, z3.data(), z3.data(), xr.data(), nullptr, S, sc.data(), ss.data(), sy.data(),
                              Kd, L, dp.data(), ds.data(), Px.data(), q.data(), Ax.data(), l.data(), u.data()))
        return fail(IMPC_INVALID_ARGUMENT, "host builder rejected the shape");
    std::vector<int32_t> sl32(slots.begin(), slots.end());
    HIP_OK(hipSetDevice(ctx->device));
    HIP_OK(hipMalloc((void **)&b->d_tPx, sizeof(double) * std::max<int64_t>(1, b->nnzP)));
    HIP_OK(hipMalloc((void **)&b->d_tAx, sizeof(double) * b->nnzA));
    HIP_OK(hipMalloc((void **)&b->d_tl, sizeof(double) * b->m));
    HIP_OK(hipMalloc((void **)&b->d_tu, sizeof(double) * b->m));
    HIP_OK(hipMalloc((void **)&b->d_slot, sizeof(int32_t) * std::max<size_t>(1, sl32.size())));
    IMPC_TRY(h2d_sync(ctx->stream, b->d_tPx, Px.data(), sizeof(double) * b->nnzP));
    IMPC_TRY(h2d_sync(ctx->stream, b->d_tAx, Ax.data(), sizeof(double) * b->nnzA));
    IMPC_TRY(h2d_sync(ctx->stream, b->d_tl, l.data(), sizeof(double) * b->m));
    IMPC_TRY(h2d_sync(ctx->stream, b->d_tu, u.data(), sizeof(double) * b->m));
    IMPC_TRY(h2d_sync(ctx->stream, b->d_slot, sl32.data(), sizeof(int32_t) * sl32.size()));
    *out = b.release();
    return IMPC_OK;
}

extern "C" int impc_mpc_builder_destroy(impc_mpc_builder b) {
    if (!b) return IMPC_OK;
    if (b->ctx) (void)hipSetDevice(b->ctx->device);
    void *ptrs[] = {b->d_tPx, b->d_tAx, b->d_tl, b->d_tu, b->d_slot};
    for (void *ptr : ptrs)
        if (ptr) (void)hipFree(ptr);
    delete b;
    return IMPC_OK;
}

extern "C" int impc_mpc_build_values_device(impc_mpc_builder b, int64_t nb, const double *curr_pos,
                                            const double *curr_vel, const double *xref, const double *lin_states,
                                            const double *st_centroid, const double *st_size, const double *st_yaw,
                                            const double *dyn_pos, const double *dyn_size, double *Px, double *q,
                                            double *Ax, double *l, double *u, void *stream) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null builder");
    if (nb < 0) return fail(IMPC_INVALID_ARGUMENT, "negative batch");
    if (nb == 0) return IMPC_OK;
    if (!curr_pos || !curr_vel || !xref || !Px || !q || !Ax || !l || !u || (b->S > 0 && (!st_centroid || !st_size || !st_yaw)) ||
        (b->Kd > 0 && (!dyn_pos || !dyn_size)))
        return fail(IMPC_INVALID_ARGUMENT, "null argument");
    HIP_OK(hipSetDevice(b->ctx->device));
    impc_build::Args a{nb, b->n, b->m, b->nnzP, b->nnzA, b->obs_off, b->N, b->W, b->S, b->Kd, b->K, b->L,
                       b->p.dynamic_safety_dist, b->p.static_safety_dist, b->p.position_weight, b->p.velocity_weight,
                       b->d_tPx, b->d_tAx, b->d_tl, b->d_tu, b->d_slot, curr_pos, curr_vel, xref, lin_states,
                       st_centroid, st_size, st_yaw, dyn_pos, dyn_size, Px, q, Ax, l, u};
    hipStream_t st = stream ? (hipStream_t)stream : b->ctx->stream;
    const int64_t groups = std::min<int64_t>(nb, (int64_t)b->ctx->num_cu * 8);
    hipLaunchKernelGGL(impc_build::k_build, dim3((unsigned)groups), dim3(256), 0, st, a);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}
