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

}  // namespace impc_predict

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
