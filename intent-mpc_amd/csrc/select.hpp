// select.hpp -- device-side candidate scoring and selection (include/impc_select.h), included by
// impc_qp.hip (same translation unit: shares the context type and error plumbing).
//
// Two small kernels on the context stream:
//   k_cand_scores  one thread per (instance, candidate): the three scores of getTrajectoryScore
//                  (mpcPlanner.cpp:771-848) from the candidate's QP solution in device memory
//   k_select       one thread per instance: evaluateTraj (mpcPlanner.cpp:850-887)
// Work per instance is tiny (N x obstacles tanh evaluations); the point is keeping the replan's
// solve -> score -> select on the device, next to the batched solver's outputs.
#pragma once

namespace impc_select {

struct Args {
    int64_t I;
    int N, C, KMAX, L, S, P;
    double dyn_safety, static_safety;
    const double *const *x_cand;
    const int8_t *valid, *first_time;
    const double *prev_states;
    const int32_t *prev_count;
    const double *xref, *st_centroid, *st_size;
    const int32_t *dyn_count;
    const double *dyn_pos, *dyn_size, *prob;
    int32_t *best_cand, *best_pos;
    double *scores, *weighted;
};

__device__ inline double norm3(double a, double b, double c) { return sqrt(a * a + b * b + c * c); }

__global__ __launch_bounds__(64) void k_cand_scores(Args a) {
    const int64_t ic = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ic >= a.I * a.C) return;
    const int64_t inst = ic / a.C;
    double *sc = a.scores + ic * 3;
    if (!a.valid[ic]) {
        sc[0] = sc[1] = sc[2] = (double)NAN;
        return;
    }
    const double *x = a.x_cand[ic];  // state k at x[8k..8k+7]
    // getConsistencyScore (:780-800)
    double cons = 0.0;
    const int pc = a.prev_count[inst];
    if (!a.first_time[inst] && pc > 0 && a.N > 0) {
        const int steps = min(10, min(pc, a.N));
        const double *pv = a.prev_states + inst * (int64_t)a.P * 8;
        double tot = 0.0;
        for (int i = 0; i < steps; i++)
            tot += norm3(pv[8 * i] - x[8 * i], pv[8 * i + 1] - x[8 * i + 1], pv[8 * i + 2] - x[8 * i + 2]);
        tot /= steps;
        cons = fmax(tot, 0.1);
    }
    // getDetourScore (:802-814)
    const double *rf = a.xref + inst * (int64_t)a.N * 8;
    double det = 0.0;
    for (int i = 0; i < a.N; i++)
        det += norm3(rf[8 * i] - x[8 * i], rf[8 * i + 1] - x[8 * i + 1], rf[8 * i + 2] - x[8 * i + 2]);
    det /= a.N;
    det = fmax(det, 0.1);
    // getSafetyScore (:816-848): planar, dynamic full size / static half size in maxSize
    const double catanh = atanh(0.5);
    const int K = a.dyn_count[ic];
    const double *dp = a.dyn_pos + ic * (int64_t)a.KMAX * a.L * 3;
    const double *ds = a.dyn_size + ic * (int64_t)a.KMAX * a.L * 3;
    const double *sp = a.st_centroid + inst * (int64_t)a.S * 3;
    const double *ss = a.st_size + inst * (int64_t)a.S * 3;
    double saf = 0.0;
    for (int i = 0; i < a.N; i++) {
        double dist = 0.0, totw = 0.0;
        const double px = x[8 * i], py = x[8 * i + 1];
        for (int j = 0; j < K; j++) {
            const double *o = dp + ((int64_t)j * a.L + i) * 3, *z = ds + ((int64_t)j * a.L + i) * 3;
            const double maxs = sqrt(z[0] * z[0] + z[1] * z[1]);
            const double d = norm3(px - o[0], py - o[1], 0.0);
            const double w = 1 - tanh(catanh / (a.dyn_safety + maxs) * d);
            dist += d * w;
            totw += w;
        }
        for (int j = 0; j < a.S; j++) {
            const double maxs = sqrt((ss[3 * j] / 2) * (ss[3 * j] / 2) + (ss[3 * j + 1] / 2) * (ss[3 * j + 1] / 2));
            const double d = norm3(px - sp[3 * j], py - sp[3 * j + 1], 0.0);
            const double w = 1 - tanh(catanh / (a.static_safety + maxs) * d);
            dist += d * w;
            totw += w;
        }
        dist /= totw;
        saf += dist;
    }
    saf /= a.N;
    sc[0] = cons;
    sc[1] = det;
    sc[2] = saf;
}

__global__ __launch_bounds__(64) void k_select(Args a) {
    const int64_t inst = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (inst >= a.I) return;
    const int C = a.C;
    const int8_t *val = a.valid + inst * C;
    const double *sc = a.scores + inst * C * 3;
    double *wt = a.weighted + inst * C;
    int n = 0;
    double ca = 0.0, da = 0.0, sa = 0.0;
    for (int c = 0; c < C; c++) {  // std::accumulate in candidate order
        wt[c] = (double)NAN;
        if (!val[c]) continue;
        ca += sc[3 * c];
        da += sc[3 * c + 1];
        sa += sc[3 * c + 2];
        n++;
    }
    if (n == 0) {
        a.best_cand[inst] = -1;
        a.best_pos[inst] = -1;
        return;
    }
    ca /= n;
    da /= n;
    sa /= n;
    const double *pr = a.prob + inst * 4;  // FORWARD, LEFT, RIGHT, STOP
    const double weight[6] = {pr[3], pr[1], pr[2], pr[0], fmax(pr[1], pr[0]), fmax(pr[2], pr[0])};
    int best = -1, bestpos = -1, pos = 0;
    double bestv = 0.0;
    for (int c = 0; c < C; c++) {
        if (!val[c]) continue;
        const double cs = ca / sc[3 * c], ds = da / sc[3 * c + 1], ssc = sc[3 * c + 2] / sa;
        const double v = weight[c] * (1.0 * cs + 1.0 * ds + 1.0 * ssc);  // C <= 6 (checked)
        wt[c] = v;
        if (best < 0 || v > bestv) {  // Eigen maxCoeff: first element, then strictly greater
            best = c;
            bestpos = pos;
            bestv = v;
        }
        pos++;
    }
    a.best_cand[inst] = best;
    a.best_pos[inst] = bestpos;
}

}  // namespace impc_select

extern "C" int impc_select_best_device(impc_ctx ctx, const impc_select_params *p, int64_t instances,
                                       const double *const *x_cand, const int8_t *valid, const int8_t *first_time,
                                       const double *prev_states, const int32_t *prev_count, const double *xref,
                                       const double *st_centroid, const double *st_size, const int32_t *dyn_count,
                                       const double *dyn_pos, const double *dyn_size, const double *prob,
                                       int32_t *best_cand, int32_t *best_pos, double *scores, double *weighted,
                                       void *stream) {
    if (!ctx || !p) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    if (instances < 0 || p->horizon < 1 || p->num_candidates < 1 || p->num_candidates > 6 || p->max_dynamic < 0 ||
        p->pred_len < p->horizon || p->num_static < 0 || p->prev_len < 0)
        return fail(IMPC_INVALID_ARGUMENT, "select: inconsistent sizes (1 <= C <= 6, pred_len >= horizon)");
    if (instances == 0) return IMPC_OK;
    HIP_OK(hipSetDevice(ctx->device));
    impc_select::Args a{instances,   p->horizon,  p->num_candidates, p->max_dynamic, p->pred_len, p->num_static,
                        p->prev_len, p->dynamic_safety_dist, p->static_safety_dist, x_cand, valid, first_time,
                        prev_states, prev_count, xref, st_centroid, st_size, dyn_count, dyn_pos, dyn_size, prob,
                        best_cand, best_pos, scores, weighted};
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    const int64_t ic = instances * p->num_candidates;
    hipLaunchKernelGGL(impc_select::k_cand_scores, dim3((unsigned)((ic + 63) / 64)), dim3(64), 0, st, a);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(impc_select::k_select, dim3((unsigned)((instances + 63) / 64)), dim3(64), 0, st, a);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

extern "C" int impc_select_best(impc_ctx ctx, const impc_select_params *p, int64_t instances,
                                const double *const *x_cand, const int8_t *valid, const int8_t *first_time,
                                const double *prev_states, const int32_t *prev_count, const double *xref,
                                const double *st_centroid, const double *st_size, const int32_t *dyn_count,
                                const double *dyn_pos, const double *dyn_size, const double *prob, int32_t *best_cand,
                                int32_t *best_pos, double *scores, double *weighted) {
    if (!ctx || !p || !x_cand || !valid || !first_time || !prev_count || !xref || !dyn_count || !prob || !best_cand ||
        !best_pos || !scores || !weighted)
        return fail(IMPC_INVALID_ARGUMENT, "null argument");
    if ((p->prev_len > 0 && !prev_states) || (p->num_static > 0 && (!st_centroid || !st_size)) ||
        (p->max_dynamic > 0 && (!dyn_pos || !dyn_size)))
        return fail(IMPC_INVALID_ARGUMENT, "null argument");
    if (instances <= 0) return instances == 0 ? IMPC_OK : fail(IMPC_INVALID_ARGUMENT, "negative instance count");
    HIP_OK(hipSetDevice(ctx->device));
    const int64_t I = instances, C = p->num_candidates, N = p->horizon;
    const size_t szx = sizeof(double *) * I * C, sz8 = I * C, szi = I, szP = sizeof(double) * I * p->prev_len * 8,
                 szpc = sizeof(int32_t) * I, szr = sizeof(double) * I * N * 8,
                 szs = sizeof(double) * I * p->num_static * 3, szdc = sizeof(int32_t) * I * C,
                 szd = sizeof(double) * I * C * (size_t)p->max_dynamic * p->pred_len * 3, szp = sizeof(double) * I * 4,
                 szb = sizeof(int32_t) * I, szsc = sizeof(double) * I * C * 3, szw = sizeof(double) * I * C;
    const size_t parts[] = {szx, sz8, szi, szP, szpc, szr, szs, szs, szdc, szd, szd, szp, szb, szb, szsc, szw};
    size_t off[16], total = 0;
    for (int k = 0; k < 16; k++) {
        off[k] = total;
        total += (parts[k] + 255) & ~(size_t)255;
    }
    char *buf = nullptr;
    HIP_OK(hipMalloc((void **)&buf, total));
    hipStream_t st = ctx->stream;
    auto up = [&](int k, const void *src) {
        return parts[k] ? hipMemcpyAsync(buf + off[k], src, parts[k], hipMemcpyHostToDevice, st) : hipSuccess;
    };
    hipError_t e = hipSuccess;
    const void *srcs[] = {x_cand, valid, first_time, prev_states, prev_count, xref, st_centroid, st_size,
                          dyn_count, dyn_pos, dyn_size, prob};
    for (int k = 0; k < 12 && e == hipSuccess; k++) e = up(k, srcs[k]);
    int rc = IMPC_OK;
    if (e != hipSuccess) {
        rc = fail(IMPC_DEVICE_ERROR, std::string("select upload: ") + hipGetErrorString(e));
    } else {
        rc = impc_select_best_device(
            ctx, p, I, (const double *const *)(buf + off[0]), (const int8_t *)(buf + off[1]),
            (const int8_t *)(buf + off[2]), (const double *)(buf + off[3]), (const int32_t *)(buf + off[4]),
            (const double *)(buf + off[5]), (const double *)(buf + off[6]), (const double *)(buf + off[7]),
            (const int32_t *)(buf + off[8]), (const double *)(buf + off[9]), (const double *)(buf + off[10]),
            (const double *)(buf + off[11]), (int32_t *)(buf + off[12]), (int32_t *)(buf + off[13]),
            (double *)(buf + off[14]), (double *)(buf + off[15]), nullptr);
    }
    if (rc == IMPC_OK) {
        void *dsts[] = {best_cand, best_pos, scores, weighted};
        for (int k = 0; k < 4 && e == hipSuccess; k++)
            e = hipMemcpyAsync(dsts[k], buf + off[12 + k], parts[12 + k], hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = fail(IMPC_DEVICE_ERROR, std::string("select download: ") + hipGetErrorString(e));
    } else {
        (void)hipStreamSynchronize(st);
    }
    (void)hipFree(buf);
    return rc;
}
