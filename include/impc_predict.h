/*
 * impc_predict.h -- intent probabilities of tracked dynamic obstacles (libimpc_qp.so), batched
 * over obstacles (and planning instances) on the device: the first half of dynamic_predictor's
 * predict() that feeds mpcPlanner's fan-out (obIntentProb_).
 *
 * Replaces (reference dynamic_predictor/include/dynamic_predictor/dynamicPredictor.cpp):
 *   initParam (intent part)  :66-115  paraml = paramr = (1 - maxFrontProb) / (3 maxFrontProb - 1),
 *                                      frontAngle in degrees -> rad, paramf = sqrt(frontAngle^2 /
 *                                      (-2 log(paraml (1 + sin frontAngle) - paraml))),
 *                                      params = atanh(0.5) / stopVel, pscale
 *   intentProb               :197-223  P = uniform; for j = 2 .. numHist-2 (oldest to newest,
 *                                      history index 0 = newest): P = T(prevAngle, currAngle,
 *                                      currVel) P.  Deviation: the reference runs j up to
 *                                      numHist-1, where it reads posHist_[-1] / velHist_[-1]
 *                                      (out of bounds, undefined behaviour); that step is not taken
 *   genTransitionMatrix      :227-255  theta = currAngle - prevAngle wrapped to (-pi, pi]; column i
 *                                      = genTransitionVector(theta, |v_xy|, scale with scale(i) =
 *                                      pscale)
 *   genTransitionVector      :257-281  FORWARD / LEFT / RIGHT / STOP probabilities
 * Intent indices follow dynamicPredictor's enum: FORWARD, LEFT, RIGHT, STOP = 0..3.
 * (The trajectory half, predTraj, samples motion models against the occupancy map and is not
 * part of this library.)
 */
#ifndef IMPC_PREDICT_H
#define IMPC_PREDICT_H
#include <stdint.h>
#include "impc_qp.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    double paramf, paraml, paramr, params, pscale;
} impc_intent_params;

/* The derived parameters from the predictor's ROS parameters (max_front_prob, front_angle in
 * degrees, stop_velocity_thereshold, prob_scale_param), as initParam computes them. */
int impc_intent_params_from_config(double max_front_prob, double front_angle_deg, double stop_velocity,
                                   double prob_scale, impc_intent_params *out);

/*
 * DEVICE pointers; asynchronous on `stream` (NULL = the context's stream).  For each of the
 * `count` tracked obstacles: hist_len [count] valid history entries (<= H), pos_hist / vel_hist
 * [count][H][3] with entry 0 the newest (the detector's posHist_ / velHist_).  Output prob
 * [count][4] (obIntentProb_).
 */
int impc_intent_prob_device(impc_ctx ctx, const impc_intent_params *p, int64_t count, int32_t H,
                            const int32_t *hist_len, const double *pos_hist, const double *vel_hist, double *prob,
                            void *stream);

/* Same with host arrays (copied to / from the device; synchronous). */
int impc_intent_prob(impc_ctx ctx, const impc_intent_params *p, int64_t count, int32_t H, const int32_t *hist_len,
                     const double *pos_hist, const double *vel_hist, double *prob);

#ifdef __cplusplus
}
#endif
#endif
