// fanout.hpp -- the intent-hypothesis fan-out of a replan (include/impc_fanout.h), included by
// impc_qp.hip (same translation unit: shares the context type and error plumbing).
//
// Two kernels on the context stream:
//   k_fanout_pick  one thread per instance: findClosestObstacle (mpcPlanner.cpp:663-708), the
//                  intent-weight order of getIntentComb (:719-728, std::sort of (weight, index)
//                  pairs, candidates taken from the back, :753-756) and every other obstacle's
//                  most probable intent (:759-768, Eigen maxCoeff = first maximum)
//   k_fanout_copy  one thread per (instance, candidate, obstacle, step): gathers the predicted
//                  position / size rows into the builder's [nb][K'][L][3] layouts -- the bulk of
//                  the bytes, written coalesced
#pragma once

namespace impc_fanout {

constexpr int FORWARD = 0, LEFT = 1, RIGHT = 2, STOP = 3;  // dynamicPredictor's intent enum

struct Args {
    int64_t I;
    int K, L, P;
    const double *curr_pos;
    const int8_t *first_time;
    const double *prev;
    const int32_t *prev_count;
    const double *dyn_cur, *pred_pos, *pred_size, *prob;
    int32_t *ob_idx, *cand_type, *cand_slot;
    double *closest_prob, *single_pos, *single_size, *pair_pos, *pair_size;
};

__device__ inline double norm3(double a, double b, double c) {
#pragma clang fp contract(off)
    return sqrt((a * a + b * b) + c * c);
}

__global__ __launch_bounds__(64) void k_fanout_pick(Args a) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.I) return;
    const int K = a.K;
    const double *cp = a.curr_pos + 3 * i, *dc = a.dyn_cur + i * K * 3;
    // findClosestObstacle (:663-708)
    int ob = -1;
    double minD = INFINITY;
    const int pc = a.prev_count[i];
    if (a.first_time[i] || pc < 2) {  // distance to the current position (:666-684)
        for (int k = 0; k < K; k++) {
            const double d = norm3(cp[0] - dc[3 * k], cp[1] - dc[3 * k + 1], cp[2] - dc[3 * k + 2]);
            if (d < minD) {
                minD = d;
                ob = k;
            }
        }
    } else {  // direction-weighted, every term at states[0] / states[1] as written (:686-706)
        const double *s = a.prev + i * (int64_t)a.P * 8, *ns = s + 8;
        const double traj = atan2(ns[1] - s[1], ns[0] - s[0]);
        for (int k = 0; k < K; k++) {
            const double obs = atan2(dc[3 * k + 1] - s[1], dc[3 * k] - s[0]);
            const double d = norm3(s[0] - dc[3 * k], s[1] - dc[3 * k + 1], s[2] - dc[3 * k + 2]);
            double dist = 0.0;
            for (int j = 0; j < pc / 3; j++) {
                const double w = exp((double)-j);
                dist += w * d * (3.0 - cos(traj - obs));
                if (dist > minD) break;
            }
            if (dist < minD) {
                minD = dist;
                ob = k;
            }
        }
    }
    if (ob < 0) ob = 0;  // only with NaN inputs (the reference would index -1)
    a.ob_idx[i] = ob;
    const double *pr = a.prob + (i * K + ob) * 4;
    // weights of the 6 combinations (:719-725), std::max(x, y) = x < y ? y : x
    const double w[6] = {pr[STOP], pr[LEFT], pr[RIGHT], pr[FORWARD], pr[LEFT] < pr[FORWARD] ? pr[FORWARD] : pr[LEFT],
                         pr[RIGHT] < pr[FORWARD] ? pr[FORWARD] : pr[RIGHT]};
    // candidate position of combination t = number of (weight, index) pairs above it
    int type_at[6];
    for (int t = 0; t < 6; t++) {
        int pos = 0;
        for (int u = 0; u < 6; u++)
            if (w[t] < w[u] || (!(w[u] < w[t]) && t < u)) pos++;
        type_at[pos] = t;
    }
    int ns_ = 0, np_ = 0;
    for (int c = 0; c < 6; c++) {
        const int t = type_at[c];
        a.cand_type[6 * i + c] = t;
        a.cand_slot[6 * i + c] = t < 4 ? ns_++ : 4 + np_++;
    }
    for (int q = 0; q < 4; q++) a.closest_prob[4 * i + q] = pr[q];
}

// maxCoeff (:762): the first most probable intent of obstacle k of instance i
__device__ inline int max_intent(const double *prob, int64_t i, int K, int k) {
    const double *p = prob + (i * K + k) * 4;
    int m = 0;
    for (int q = 1; q < 4; q++)
        if (p[q] > p[m]) m = q;
    return m;
}

__global__ __launch_bounds__(256) void k_fanout_copy(Args a) {
    const int K = a.K, L = a.L;
    const int64_t rs = 4LL * K * L, rp = 2LL * (K + 1) * L, R = rs + rp;
    const int64_t total = a.I * R;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / R;
        int64_t r = e - i * R;
        const bool pair = r >= rs;
        if (pair) r -= rs;
        const int KK = pair ? K + 1 : K;
        const int slot = (int)(r / ((int64_t)KK * L));
        const int o = (int)(r / L % KK), st = (int)(r % L);
        // combination in this slot
        const int want = pair ? 4 + slot : slot;
        int t = 0;
        for (int c = 0; c < 6; c++)
            if (a.cand_slot[6 * i + c] == want) t = a.cand_type[6 * i + c];
        const int ob = a.ob_idx[i];
        const int nfirst = pair ? 2 : 1;  // the closest obstacle's intents come first (:731-750)
        int k, intent;
        if (o < nfirst) {
            k = ob;
            static constexpr int single_intent[4] = {STOP, LEFT, RIGHT, FORWARD};
            intent = t < 4 ? single_intent[t] : (o == 0 ? (t == 4 ? LEFT : RIGHT) : FORWARD);
        } else {  // other obstacles in index order (:759-768)
            const int q = o - nfirst;
            k = q < ob ? q : q + 1;
            intent = max_intent(a.prob, i, K, k);
        }
        const int64_t src = (((i * K + k) * 4 + intent) * (int64_t)L + st) * 3;
        double *dp = pair ? a.pair_pos : a.single_pos, *ds = pair ? a.pair_size : a.single_size;
        const int64_t dst = (((i * (pair ? 2 : 4) + slot) * (int64_t)KK + o) * L + st) * 3;
        for (int d = 0; d < 3; d++) {
            dp[dst + d] = a.pred_pos[src + d];
            ds[dst + d] = a.pred_size[src + d];
        }
    }
}

// candidate -> (solution pointer, obstacle count, padded obstacle sets) for impc_select_best
__global__ __launch_bounds__(256) void k_fanout_candidates(int64_t I, int K, int L, const int32_t *cand_slot,
                                                           const double *spos, const double *ssz, const double *ppos,
                                                           const double *psz, const double *xs, int64_t ns,
                                                           const double *xp, int64_t np, const double **x_cand,
                                                           int32_t *dyn_count, double *dpos, double *dsz) {
    const int64_t rows = (int64_t)(K + 1) * L, total = I * 6 * rows;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t ic = e / rows, i = ic / 6;
        const int r = (int)(e - ic * rows), o = r / L, st = r % L;
        const int s = cand_slot[ic];
        const bool pair = s >= 4;
        if (r == 0) {
            x_cand[ic] = pair ? xp + (2 * i + s - 4) * np : xs + (4 * i + s) * ns;
            dyn_count[ic] = pair ? K + 1 : K;
        }
        const double *sp, *sz;
        if (pair) {
            const int64_t src = (((i * 2 + s - 4) * (int64_t)(K + 1) + o) * L + st) * 3;
            sp = ppos + src;
            sz = psz + src;
        } else {
            const int64_t src = (((i * 4 + s) * (int64_t)K + (o < K ? o : 0)) * L + st) * 3;
            sp = spos + src;
            sz = ssz + src;
        }
        const bool pad = !pair && o == K;
        for (int d = 0; d < 3; d++) {
            dpos[e * 3 + d] = pad ? 0.0 : sp[d];
            dsz[e * 3 + d] = pad ? 0.0 : sz[d];
        }
    }
}

}  // namespace impc_fanout

extern "C" int impc_fanout_candidates_device(impc_ctx ctx, int64_t instances, int32_t num_obstacles,
                                             int32_t pred_len, const int32_t *cand_slot, const double *single_pos,
                                             const double *single_size, const double *pair_pos,
                                             const double *pair_size, const double *x_single, int64_t n_single,
                                             const double *x_pair, int64_t n_pair, const double **x_cand,
                                             int32_t *dyn_count, double *dyn_pos, double *dyn_size, void *stream) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    if (instances < 0 || num_obstacles < 1 || pred_len < 1 || n_single < 1 || n_pair < 1)
        return fail(IMPC_INVALID_ARGUMENT, "fanout candidates: bad sizes");
    if (instances == 0) return IMPC_OK;
    if (!cand_slot || !single_pos || !single_size || !pair_pos || !pair_size || !x_single || !x_pair || !x_cand ||
        !dyn_count || !dyn_pos || !dyn_size)
        return fail(IMPC_INVALID_ARGUMENT, "fanout candidates: null argument");
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    const int64_t total = instances * 6 * (int64_t)(num_obstacles + 1) * pred_len;
    const int64_t blocks = std::min<int64_t>((total + 255) / 256, (int64_t)ctx->num_cu * 16);
    hipLaunchKernelGGL(impc_fanout::k_fanout_candidates, dim3((unsigned)blocks), dim3(256), 0, st, instances,
                       num_obstacles, pred_len, cand_slot, single_pos, single_size, pair_pos, pair_size, x_single,
                       n_single, x_pair, n_pair, x_cand, dyn_count, dyn_pos, dyn_size);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

extern "C" int impc_intent_fanout_device(impc_ctx ctx, int64_t instances, int32_t num_obstacles, int32_t pred_len,
                                         int32_t prev_len, const double *curr_pos, const int8_t *first_time,
                                         const double *prev_states, const int32_t *prev_count, const double *dyn_cur,
                                         const double *pred_pos, const double *pred_size, const double *prob,
                                         int32_t *ob_idx, int32_t *cand_type, int32_t *cand_slot,
                                         double *closest_prob, double *single_pos, double *single_size,
                                         double *pair_pos, double *pair_size, void *stream) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    if (instances < 0 || num_obstacles < 1 || pred_len < 1 || prev_len < 0)
        return fail(IMPC_INVALID_ARGUMENT, "fanout: need instances >= 0, K >= 1, L >= 1, P >= 0");
    if (instances == 0) return IMPC_OK;
    if (!curr_pos || !first_time || !prev_count || (prev_len > 0 && !prev_states) || !dyn_cur || !pred_pos ||
        !pred_size || !prob || !ob_idx || !cand_type || !cand_slot || !closest_prob || !single_pos || !single_size ||
        !pair_pos || !pair_size)
        return fail(IMPC_INVALID_ARGUMENT, "fanout: null argument");
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    // (no scratch: the other obstacles' most probable intents are recomputed where they are used;
    // a stream-ordered hipMallocAsync scratch for them was read back as zeros on some calls)
    impc_fanout::Args a{instances, num_obstacles, pred_len, prev_len, curr_pos, first_time, prev_states,
                        prev_count, dyn_cur, pred_pos, pred_size, prob, ob_idx, cand_type, cand_slot,
                        closest_prob, single_pos, single_size, pair_pos, pair_size};
    hipLaunchKernelGGL(impc_fanout::k_fanout_pick, dim3((unsigned)((instances + 63) / 64)), dim3(64), 0, st, a);
    HIP_OK(hipGetLastError());
    const int64_t rows = instances * (4LL * num_obstacles + 2LL * (num_obstacles + 1)) * pred_len;
    const int64_t blocks = std::min<int64_t>((rows + 255) / 256, (int64_t)ctx->num_cu * 16);
    hipLaunchKernelGGL(impc_fanout::k_fanout_copy, dim3((unsigned)blocks), dim3(256), 0, st, a);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

extern "C" int impc_intent_fanout(impc_ctx ctx, int64_t instances, int32_t num_obstacles, int32_t pred_len,
                                  int32_t prev_len, const double *curr_pos, const int8_t *first_time,
                                  const double *prev_states, const int32_t *prev_count, const double *dyn_cur,
                                  const double *pred_pos, const double *pred_size, const double *prob,
                                  int32_t *ob_idx, int32_t *cand_type, int32_t *cand_slot, double *closest_prob,
                                  double *single_pos, double *single_size, double *pair_pos, double *pair_size) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    if (instances < 0 || num_obstacles < 1 || pred_len < 1 || prev_len < 0)
        return fail(IMPC_INVALID_ARGUMENT, "fanout: need instances >= 0, K >= 1, L >= 1, P >= 0");
    if (instances == 0) return IMPC_OK;
    const size_t I = (size_t)instances, K = (size_t)num_obstacles, L = (size_t)pred_len, P = (size_t)prev_len;
    const size_t parts[] = {8 * I * 3,     I,         8 * I * P * 8,     4 * I,         8 * I * K * 3,
                            8 * I * K * 4 * L * 3, 8 * I * K * 4 * L * 3, 8 * I * K * 4, 4 * I,
                            4 * I * 6,     4 * I * 6, 8 * I * 4,         8 * I * 4 * K * L * 3,
                            8 * I * 4 * K * L * 3, 8 * I * 2 * (K + 1) * L * 3, 8 * I * 2 * (K + 1) * L * 3};
    constexpr int NP = 16, NIN = 8;
    size_t off[NP], total = 0;
    for (int k = 0; k < NP; k++) {
        off[k] = total;
        total += (parts[k] + 255) & ~(size_t)255;
    }
    HIP_OK(hipSetDevice(ctx->device));
    char *buf = nullptr;
    HIP_OK(hipMalloc((void **)&buf, total));
    hipStream_t st = ctx->stream;
    const void *srcs[NIN] = {curr_pos, first_time, prev_states, prev_count, dyn_cur, pred_pos, pred_size, prob};
    void *dsts[NP - NIN] = {ob_idx, cand_type, cand_slot, closest_prob, single_pos, single_size, pair_pos, pair_size};
    hipError_t e = hipSuccess;
    for (int k = 0; k < NIN && e == hipSuccess; k++)
        if (parts[k] && srcs[k]) e = hipMemcpyAsync(buf + off[k], srcs[k], parts[k], hipMemcpyHostToDevice, st);
    int rc = IMPC_OK;
    if (e != hipSuccess) {
        rc = fail(IMPC_DEVICE_ERROR, std::string("fanout upload: ") + hipGetErrorString(e));
    } else {
        auto D = [&](int k) { return (void *)(buf + off[k]); };
        rc = impc_intent_fanout_device(ctx, instances, num_obstacles, pred_len, prev_len, (const double *)D(0),
                                       (const int8_t *)D(1), (const double *)D(2), (const int32_t *)D(3),
                                       (const double *)D(4), (const double *)D(5), (const double *)D(6),
                                       (const double *)D(7), (int32_t *)D(8), (int32_t *)D(9), (int32_t *)D(10),
                                       (double *)D(11), (double *)D(12), (double *)D(13), (double *)D(14),
                                       (double *)D(15), nullptr);
    }
    if (rc == IMPC_OK) {
        for (int k = NIN; k < NP && e == hipSuccess; k++)
            e = hipMemcpyAsync(dsts[k - NIN], buf + off[k], parts[k], hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = fail(IMPC_DEVICE_ERROR, std::string("fanout download: ") + hipGetErrorString(e));
    } else {
        (void)hipStreamSynchronize(st);
    }
    (void)hipFree(buf);
    return rc;
}
