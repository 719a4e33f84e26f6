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

/* ---- Trajectory half: predTraj (dynamicPredictor.cpp:283-566) -- per obstacle and intent the
 * motion-model samples (FORWARD :351-396: heading x speed grid, speeds ascend until the first
 * sample that hits the map; LEFT / RIGHT :398-472: speed x turn rate x end heading grid, hitting
 * samples dropped; STOP / slow obstacles :474-488: stationary with growing size), their mean and
 * variance (genTraj :501-538: size += 2 sqrt(var) z_score) and positionCorrection (:540-566: a
 * mean that hits the map is replaced by the closest sample).  The map is map_manager's inflated
 * occupancy grid (occupancyMap.h:218-269): voxel (floor((p - origin) / res)), outside the grid
 * counts as occupied, address x * dims[1] * dims[2] + y * dims[2] + z. */
typedef struct {
    double origin[3];    /* mapSizeMin_ */
    double resolution;   /* mapRes_ */
    int32_t dims[3];     /* mapVoxelMax_ (mapVoxelMin_ = 0) */
    int32_t reserved;
} impc_occ_map;

typedef struct {
    int32_t num_pred;          /* prediction_size: num_pred + 1 points per trajectory */
    int32_t reserved;
    double dt;                 /* prediction_time_step */
    double stop_velocity;      /* stop_velocity_thereshold */
    double front_angle_deg;    /* front_angle (degrees, as the ROS parameter) */
    double min_turning_time, max_turning_time;
    double z_score;            /* prediction_z_score */
} impc_traj_params;

/* DEVICE pointers; asynchronous.  occ_inflated [dims[0] * dims[1] * dims[2]] (nonzero =
 * occupied); per obstacle the newest history entry pos, vel, size [count][3]; outputs
 * pred_pos / pred_size [count][4][num_pred + 1][3] (obPredPos_ / obPredSize_, the fan-out's
 * pred_pos / pred_size). */
int impc_predict_traj_device(impc_ctx ctx, const impc_traj_params *tp, const impc_occ_map *map,
                             const uint8_t *occ_inflated, int64_t count, const double *pos, const double *vel,
                             const double *size, double *pred_pos, double *pred_size, void *stream);

/* Same with host arrays (synchronous). */
int impc_predict_traj(impc_ctx ctx, const impc_traj_params *tp, const impc_occ_map *map, const uint8_t *occ_inflated,
                      int64_t count, const double *pos, const double *vel, const double *size, double *pred_pos,
                      double *pred_size);

#ifdef __cplusplus
}
#endif
#endif
