// predict.hpp -- intent probabilities of tracked obstacles (include/impc_predict.h), included by
// impc_qp.hip.  One thread per obstacle walks its history (a 4-state Markov chain with a 4 x 4
// transition matrix per step, dynamicPredictor.cpp:197-281); the work is a few hundred flops per
// history step, so the kernel is latency-bound and tiny next to the solve.
#pragma once

namespace impc_predict {

constexpr int FORWARD = 0, LEFT = 1, RIGHT = 2, STOP = 3;

// genTransitionVector (:257-281) with scale = 1 except scale(si) = pscale
__host__ __device__ inline void transition_vector(const impc_intent_params &p, double theta, double r, int si,
                                                  double out[4]) {
#pragma clang fp contract(off)
    const double s0 = si == 0 ? p.pscale : 1.0, s1 = si == 1 ? p.pscale : 1.0, s2 = si == 2 ? p.pscale : 1.0,
                 s3 = si == 3 ? p.pscale : 1.0;
    const double tf = theta / p.paramf;
    double pf = s0 * (exp(-0.5 * (tf * tf)) + p.paraml);
    double pl = s1 * (p.paraml * (1 + sin(theta)));
    double pr = s2 * (p.paramr * (1 - sin(theta)));
    const double ps = 1 - tanh(p.params / s3 * r);
    const double sum = pr + pl + pf;
    pr = (1 - ps) * pr / sum;
    pl = (1 - ps) * pl / sum;
    pf = (1 - ps) * pf / sum;
    out[FORWARD] = pf;
    out[LEFT] = pl;
    out[RIGHT] = pr;
    out[STOP] = ps;
}

__global__ __launch_bounds__(64) void k_intent_prob(impc_intent_params p, int64_t count, int H, const int32_t *hlen,
                                                    const double *pos, const double *vel, double *prob) {
#pragma clang fp contract(off)
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= count) return;
    const double *ph = pos + o * (int64_t)H * 3, *vh = vel + o * (int64_t)H * 3;
    const int nh = hlen[o];
    double P[4] = {0.25, 0.25, 0.25, 0.25};  // setConstant(1.0 / numIntent_)
    // the reference loops j < numHist (:206), whose last step reads history entry -1 (out of
    // bounds: undefined behaviour); the steps with defined inputs are j <= numHist - 2
    for (int j = 2; j < nh - 1; j++) {
        const double *prevPos = ph + 3 * (nh - j - 1), *currPos = ph + 3 * (nh - j - 2), *pp = ph + 3 * (nh - j);
        const double *currVel = vh + 3 * (nh - j - 2);
        const double prevAngle = atan2(prevPos[1] - pp[1], prevPos[0] - pp[0]);
        const double currAngle = atan2(currPos[1] - prevPos[1], currPos[0] - prevPos[0]);
        double theta = currAngle - prevAngle;
        if (theta > M_PI)
            theta = theta - 2 * M_PI;
        else if (theta <= -M_PI)
            theta = theta + 2 * M_PI;
        const double r = sqrt(currVel[0] * currVel[0] + currVel[1] * currVel[1]);
        double T[4][4];  // column i
        for (int i = 0; i < 4; i++) transition_vector(p, theta, r, i, T[i]);
        double nP[4];
        for (int row = 0; row < 4; row++) {  // (T P)_row, columns accumulated in order
            double acc = 0.0;
            for (int c = 0; c < 4; c++) acc += T[c][row] * P[c];
            nP[row] = acc;
        }
        for (int k = 0; k < 4; k++) P[k] = nP[k];
    }
    for (int k = 0; k < 4; k++) prob[o * 4 + k] = P[k];
}

// ---------------------------------------------------------------- predTraj
// One thread per (obstacle, intent).  The motion-model samples are not stored: each pass over
// them re-simulates (the arithmetic is deterministic), so a thread needs only its output rows,
// which double as the accumulators (mean sums in pred_pos, variance sums in pred_size).
struct TrajArgs {
    impc_traj_params tp;
    impc_occ_map map;
    const uint8_t *occ;
    int64_t count;
    const double *pos, *vel, *size;
    double *ppos, *psize;
};

__device__ inline bool occupied(const TrajArgs &a, double x, double y, double z) {
#pragma clang fp contract(off)
    const int ix = (int)floor((x - a.map.origin[0]) / a.map.resolution);
    const int iy = (int)floor((y - a.map.origin[1]) / a.map.resolution);
    const int iz = (int)floor((z - a.map.origin[2]) / a.map.resolution);
    const int *d = a.map.dims;
    if (ix < 0 || ix >= d[0] || iy < 0 || iy >= d[1] || iz < 0 || iz >= d[2]) return true;
    return a.occ[((int64_t)ix * d[1] + iy) * d[2] + iz] != 0;
}

// A motion-model sample: FORWARD (heading h, speed sp) or turning (speed sp, rate w, end angle e).
struct Sample {
    double h, sp, w, e;
};

// Simulates sample s for num_pred steps, calling cb(k, x, y) for the points k = 1..num_pred;
// returns false at the first point inside the map's occupied space (cb not called for it).
template <class CB>
__device__ bool simulate(const TrajArgs &a, int intent, const double *p0, double a0, const Sample &s, CB cb) {
#pragma clang fp contract(off)
    const double dt = a.tp.dt;
    double x = p0[0], y = p0[1], vx, vy, ang = a0;
    if (intent == FORWARD) {
        vx = s.sp * cos(s.h);
        vy = s.sp * sin(s.h);
    } else {
        vx = s.sp * cos(ang);
        vy = s.sp * sin(ang);
    }
    for (int k = 1; k <= a.tp.num_pred; k++) {
        const double nx = x + dt * vx, ny = y + dt * vy;
        if (occupied(a, nx, ny, p0[2])) return false;
        cb(k, nx, ny);
        x = nx;
        y = ny;
        if (intent != FORWARD) {
            ang += s.w * dt;
            ang = intent == LEFT ? (s.e < ang ? s.e : ang) : (ang < s.e ? s.e : ang);
            const double vv = sqrt(vx * vx + vy * vy);
            vx = vv * cos(ang);
            vy = vv * sin(ang);
        }
    }
    return true;
}

// Calls f(sample) for every valid sample of the model, in the reference's loop order.
template <class F>
__device__ void for_each_sample(const TrajArgs &a, int intent, const double *p0, double v, double a0, F f) {
#pragma clang fp contract(off)
    auto none = [](int, double, double) {};
    const double fa = a.tp.front_angle_deg * M_PI / 180;
    if (intent == FORWARD) {
        for (double i = a0 - fa; i < a0 + fa; i += 0.1)
            for (double j = v - v; j < v + v; j += 0.1) {
                const Sample s{i, j, 0.0, 0.0};
                if (!simulate(a, intent, p0, a0, s, none)) break;  // faster samples of this heading skipped
                f(s);
            }
        return;
    }
    double e_min, e_max, w_min, w_max;
    if (intent == LEFT) {
        e_min = fa + a0;
        e_max = (M_PI - fa) + a0;
        w_min = (M_PI / 2) / a.tp.max_turning_time;
        w_max = (M_PI / 2) / a.tp.min_turning_time;
    } else {
        e_min = -(M_PI - fa) + a0;
        e_max = -fa + a0;
        w_min = (-M_PI / 2) / a.tp.min_turning_time;
        w_max = (-M_PI / 2) / a.tp.max_turning_time;
    }
    for (double i = v - v; i < v + v; i += 0.2)
        for (double j = w_min; j < w_max; j += 0.2)
            for (double e = e_min; e < e_max; e += 0.2) {
                const Sample s{0.0, i, j, e};
                if (simulate(a, intent, p0, a0, s, none)) f(s);
            }
}

__global__ __launch_bounds__(64) void k_predict_traj(TrajArgs a) {
#pragma clang fp contract(off)
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.count * 4) return;
    const int64_t o = t / 4;
    const int intent = (int)(t % 4);
    const int P = a.tp.num_pred, NP = P + 1;
    const double *p0 = a.pos + 3 * o, *v0 = a.vel + 3 * o, *s0 = a.size + 3 * o;
    double *pp = a.ppos + t * NP * 3, *ps = a.psize + t * NP * 3;
    const double v = sqrt(v0[0] * v0[0] + v0[1] * v0[1]);
    const double a0 = atan2(v0[1], v0[0]);
    auto stationary = [&]() {  // modelStop / no valid sample: the current position, growing size
        double sx = s0[0], sy = s0[1];
        for (int k = 0; k < NP; k++) {
            pp[3 * k] = p0[0];
            pp[3 * k + 1] = p0[1];
            pp[3 * k + 2] = p0[2];
            ps[3 * k] = sx;
            ps[3 * k + 1] = sy;
            ps[3 * k + 2] = s0[2];
            const double g = 2 * (v < a.tp.stop_velocity ? v : a.tp.stop_velocity) * a.tp.dt;
            sx += g;
            sy += g;
        }
    };
    if (v <= a.tp.stop_velocity || intent == STOP) {
        // one sample (the current position): mean = it, variance 0 (size += 0), and
        // positionCorrection replaces it by itself
        stationary();
        return;
    }
    // pass 1: sums of the valid samples' points -> mean
    for (int k = 0; k < NP; k++) pp[3 * k] = pp[3 * k + 1] = ps[3 * k] = ps[3 * k + 1] = 0.0;
    int64_t n = 0;
    for_each_sample(a, intent, p0, v, a0, [&](const Sample &s) {
        n++;
        pp[0] += p0[0];
        pp[1] += p0[1];
        simulate(a, intent, p0, a0, s, [&](int k, double x, double y) {
            pp[3 * k] += x;
            pp[3 * k + 1] += y;
        });
    });
    if (n == 0) {
        stationary();
        return;
    }
    for (int k = 0; k < NP; k++) {
        pp[3 * k] = pp[3 * k] / (double)n;
        pp[3 * k + 1] = pp[3 * k + 1] / (double)n;
        pp[3 * k + 2] = p0[2];
    }
    // pass 2: variance sums -> sizes
    for_each_sample(a, intent, p0, v, a0, [&](const Sample &s) {
        double dx = p0[0] - pp[0], dy = p0[1] - pp[1];
        ps[0] += dx * dx;
        ps[1] += dy * dy;
        simulate(a, intent, p0, a0, s, [&](int k, double x, double y) {
            const double ex = x - pp[3 * k], ey = y - pp[3 * k + 1];
            ps[3 * k] += ex * ex;
            ps[3 * k + 1] += ey * ey;
        });
    });
    for (int k = 0; k < NP; k++) {
        ps[3 * k] = s0[0] + 2 * sqrt(ps[3 * k] / (double)n) * a.tp.z_score;
        ps[3 * k + 1] = s0[1] + 2 * sqrt(ps[3 * k + 1] / (double)n) * a.tp.z_score;
        ps[3 * k + 2] = s0[2];
    }
    // positionCorrection: a mean point inside the occupied space -> the closest sample
    bool hit = false;
    for (int k = 0; k < NP && !hit; k++) hit = occupied(a, pp[3 * k], pp[3 * k + 1], pp[3 * k + 2]);
    if (!hit) return;
    double best = INFINITY;
    int64_t best_idx = -1, idx = 0;
    for_each_sample(a, intent, p0, v, a0, [&](const Sample &s) {
        double dx = p0[0] - pp[0], dy = p0[1] - pp[1];
        double sm = sqrt(dx * dx + dy * dy);
        simulate(a, intent, p0, a0, s, [&](int k, double x, double y) {
            const double ex = x - pp[3 * k], ey = y - pp[3 * k + 1];
            sm += sqrt(ex * ex + ey * ey);
        });
        if (sm < best) {  // the reference's early break only skips sums already above the minimum
            best = sm;
            best_idx = idx;
        }
        idx++;
    });
    idx = 0;
    for_each_sample(a, intent, p0, v, a0, [&](const Sample &s) {
        if (idx++ != best_idx) return;
        pp[0] = p0[0];
        pp[1] = p0[1];
        simulate(a, intent, p0, a0, s, [&](int k, double x, double y) {
            pp[3 * k] = x;
            pp[3 * k + 1] = y;
        });
    });
}

}  // namespace impc_predict

extern "C" int impc_predict_traj_device(impc_ctx ctx, const impc_traj_params *tp, const impc_occ_map *map,
                                        const uint8_t *occ_inflated, int64_t count, const double *pos,
                                        const double *vel, const double *size, double *pred_pos, double *pred_size,
                                        void *stream) {
    if (!ctx || !tp || !map) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    if (count < 0 || tp->num_pred < 0 || !(map->resolution > 0) || map->dims[0] < 0 || map->dims[1] < 0 ||
        map->dims[2] < 0)
        return fail(IMPC_INVALID_ARGUMENT, "predict_traj: bad sizes");
    if (count == 0) return IMPC_OK;
    if (!occ_inflated || !pos || !vel || !size || !pred_pos || !pred_size)
        return fail(IMPC_INVALID_ARGUMENT, "predict_traj: null array");
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    impc_predict::TrajArgs a{*tp, *map, occ_inflated, count, pos, vel, size, pred_pos, pred_size};
    hipLaunchKernelGGL(impc_predict::k_predict_traj, dim3((unsigned)((4 * count + 63) / 64)), dim3(64), 0, st, a);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

extern "C" int impc_predict_traj(impc_ctx ctx, const impc_traj_params *tp, const impc_occ_map *map,
                                 const uint8_t *occ_inflated, int64_t count, const double *pos, const double *vel,
                                 const double *size, double *pred_pos, double *pred_size) {
    if (!ctx || !tp || !map) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    if (count < 0 || tp->num_pred < 0 || map->dims[0] < 0 || map->dims[1] < 0 || map->dims[2] < 0)
        return fail(IMPC_INVALID_ARGUMENT, "predict_traj: bad sizes");
    if (count == 0) return IMPC_OK;
    HIP_OK(hipSetDevice(ctx->device));
    const size_t nocc = (size_t)map->dims[0] * map->dims[1] * map->dims[2], n3 = sizeof(double) * count * 3,
                 nout = sizeof(double) * count * 4 * (size_t)(tp->num_pred + 1) * 3;
    auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
    char *buf = nullptr;
    HIP_OK(hipMalloc((void **)&buf, up(nocc) + 3 * up(n3) + 2 * up(nout) + 256));
    uint8_t *docc = (uint8_t *)buf;
    double *dpos = (double *)(buf + up(nocc)), *dvel = (double *)((char *)dpos + up(n3)),
           *dsz = (double *)((char *)dvel + up(n3)), *dpp = (double *)((char *)dsz + up(n3)),
           *dps = (double *)((char *)dpp + up(nout));
    hipStream_t st = ctx->stream;
    int rc = h2d_sync(st, docc, occ_inflated, nocc);
    if (!rc) rc = h2d_sync(st, dpos, pos, n3);
    if (!rc) rc = h2d_sync(st, dvel, vel, n3);
    if (!rc) rc = h2d_sync(st, dsz, size, n3);
    if (!rc) rc = impc_predict_traj_device(ctx, tp, map, docc, count, dpos, dvel, dsz, dpp, dps, nullptr);
    if (!rc) {
        hipError_t e = hipMemcpyAsync(pred_pos, dpp, nout, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(pred_size, dps, nout, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = fail(IMPC_DEVICE_ERROR, std::string("predict_traj download: ") + hipGetErrorString(e));
    }
    (void)hipFree(buf);
    return rc;
}

extern "C" int impc_intent_params_from_config(double max_front_prob, double front_angle_deg, double stop_velocity,
                                              double prob_scale, impc_intent_params *out) {
    if (!out) return fail(IMPC_INVALID_ARGUMENT, "null output");
    if (!(3 * max_front_prob - 1 != 0) || !(stop_velocity > 0))
        return fail(IMPC_INVALID_ARGUMENT, "max_front_prob must differ from 1/3 and stop velocity be > 0");
    out->paraml = out->paramr = (1 - max_front_prob) / (3 * max_front_prob - 1);   // :70-76
    const double fa = front_angle_deg * M_PI / 180;                                // :87
    out->paramf = sqrt(fa * fa / (-2 * log(out->paraml * (1 + sin(fa)) - out->paraml)));  // :88
    out->params = atanh(0.5) / stop_velocity;                                       // :99
    out->pscale = prob_scale;                                                       // :109-114
    return IMPC_OK;
}

extern "C" int impc_intent_prob_device(impc_ctx ctx, const impc_intent_params *p, int64_t count, int32_t H,
                                       const int32_t *hist_len, const double *pos_hist, const double *vel_hist,
                                       double *prob, void *stream) {
    if (!ctx || !p) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    if (count < 0 || H < 0) return fail(IMPC_INVALID_ARGUMENT, "negative size");
    if (count == 0) return IMPC_OK;
    if (!hist_len || !prob || (H > 0 && (!pos_hist || !vel_hist))) return fail(IMPC_INVALID_ARGUMENT, "null array");
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    hipLaunchKernelGGL(impc_predict::k_intent_prob, dim3((unsigned)((count + 63) / 64)), dim3(64), 0, st, *p, count,
                       (int)H, hist_len, pos_hist, vel_hist, prob);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

extern "C" int impc_intent_prob(impc_ctx ctx, const impc_intent_params *p, int64_t count, int32_t H,
                                const int32_t *hist_len, const double *pos_hist, const double *vel_hist,
                                double *prob) {
    if (!ctx || !p) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    if (count < 0 || H < 0) return fail(IMPC_INVALID_ARGUMENT, "negative size");
    if (count == 0) return IMPC_OK;
    for (int64_t o = 0; o < count; o++)
        if (hist_len[o] < 0 || hist_len[o] > H) return fail(IMPC_INVALID_ARGUMENT, "hist_len outside [0, H]");
    HIP_OK(hipSetDevice(ctx->device));
    const size_t nh = sizeof(int32_t) * count, nv = sizeof(double) * count * (size_t)H * 3, np = sizeof(double) * count * 4;
    char *buf = nullptr;
    HIP_OK(hipMalloc((void **)&buf, nh + 2 * nv + np + 1024));
    int32_t *dh = (int32_t *)buf;
    double *dp = (double *)(buf + ((nh + 255) & ~(size_t)255)), *dv = dp + count * (size_t)H * 3,
           *dpr = dv + count * (size_t)H * 3;
    hipStream_t st = ctx->stream;
    int rc = h2d_sync(st, dh, hist_len, nh);
    if (!rc) rc = h2d_sync(st, dp, pos_hist, nv);
    if (!rc) rc = h2d_sync(st, dv, vel_hist, nv);
    if (!rc) rc = impc_intent_prob_device(ctx, p, count, H, dh, dp, dv, dpr, nullptr);
    if (!rc) {
        hipError_t e = hipMemcpyAsync(prob, dpr, np, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = fail(IMPC_DEVICE_ERROR, std::string("intent prob download: ") + hipGetErrorString(e));
    }
    (void)hipFree(buf);
    return rc;
}
