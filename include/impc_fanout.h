/*
 * impc_fanout.h -- the intent-hypothesis fan-out of a replan (libimpc_qp.so), batched over
 * planning instances on the device.
 *
 * Replaces, per instance, the host code of mpcPlanner::makePlanWithPred that builds the candidate
 * obstacle sets before the serial solveTraj loop (reference
 * trajectory_planner/include/trajectory_planner/mpcPlanner.cpp):
 *   findClosestObstacle   :663-708   closest dynamic obstacle (distance on the first call or with
 *                                    fewer than 2 previous states; otherwise the direction-weighted
 *                                    score over currentStatesSol_.size()/3 terms, as written:
 *                                    states[0] / states[1] in every term)
 *   getIntentComb         :710-769   the 6 candidates, ordered by descending intent weight
 *                                    (std::sort of (weight, index) pairs, taken from the back):
 *                                    STOP, LEFT, RIGHT, FORWARD, {LEFT, FORWARD}, {RIGHT, FORWARD}
 *                                    for the closest obstacle, every other obstacle at its most
 *                                    probable intent (Eigen maxCoeff: first maximum)
 * Intent indices follow dynamicPredictor's enum: FORWARD, LEFT, RIGHT, STOP = 0..3.
 *
 * The candidates come out in the layouts impc_mpc_build_values_device takes (dyn_pos / dyn_size
 * [nb][K'][L][3]): the four single-intent candidates (K obstacles) in one array, the two
 * two-intent candidates (K + 1 obstacles) in another, so each array is one QP shape.
 */
#ifndef IMPC_FANOUT_H
#define IMPC_FANOUT_H
#include <stdint.h>
#include "impc_qp.h"
#ifdef __cplusplus
extern "C" {
#endif

/*
 * DEVICE pointers; asynchronous on `stream` (NULL = the context's stream).  K >= 1 obstacles
 * per instance (the reference calls getIntentComb only when obPredPos_ is not empty), L
 * prediction steps, P previous-plan slots.
 *   curr_pos    [I][3]            currPos_
 *   first_time  [I] int8          firstTime_
 *   prev_states [I][P][8], prev_count [I]   currentStatesSol_ and its size()
 *   dyn_cur     [I][K][3]         dynamicObstaclesPos_[k][0]
 *   pred_pos, pred_size [I][K][4][L][3]     obPredPos_, obPredSize_
 *   prob        [I][K][4]         obIntentProb_
 * Outputs:
 *   ob_idx      [I] int32         closest obstacle
 *   cand_type   [I][6] int32      intent combination (0..5 as listed above) of candidate c
 *   cand_slot   [I][6] int32      s < 4: candidate c is single[s]; s >= 4: pair[s - 4]
 *   closest_prob [I][4]           obIntentProb_[ob_idx] (the `prob` input of impc_select_best)
 *   single_pos, single_size [I][4][K][L][3]
 *   pair_pos, pair_size     [I][2][K+1][L][3]
 */
int impc_intent_fanout_device(impc_ctx ctx, int64_t instances, int32_t num_obstacles, int32_t pred_len,
                              int32_t prev_len, const double *curr_pos, const int8_t *first_time,
                              const double *prev_states, const int32_t *prev_count, const double *dyn_cur,
                              const double *pred_pos, const double *pred_size, const double *prob, int32_t *ob_idx,
                              int32_t *cand_type, int32_t *cand_slot, double *closest_prob, double *single_pos,
                              double *single_size, double *pair_pos, double *pair_size, void *stream);

/* The selection inputs of the replan's candidates, on the device: for candidate c of instance i
 * (slot s = cand_slot[i][c]) the pointer to its QP solution -- x_single + (4 i + s) n_single or
 * x_pair + (2 i + s - 4) n_pair doubles -- its obstacle count (K or K + 1) and its obstacle sets
 * in impc_select_best_device's padded [I][6][K+1][L][3] layout (zero-filled slot K for the
 * single-intent candidates).  Everything stays on the device; asynchronous on `stream`. */
int impc_fanout_candidates_device(impc_ctx ctx, int64_t instances, int32_t num_obstacles, int32_t pred_len,
                                  const int32_t *cand_slot, const double *single_pos, const double *single_size,
                                  const double *pair_pos, const double *pair_size, const double *x_single,
                                  int64_t n_single, const double *x_pair, int64_t n_pair, const double **x_cand,
                                  int32_t *dyn_count, double *dyn_pos, double *dyn_size, void *stream);

/* Same with host arrays (copied to / from the device; synchronous). */
int impc_intent_fanout(impc_ctx ctx, int64_t instances, int32_t num_obstacles, int32_t pred_len, int32_t prev_len,
                       const double *curr_pos, const int8_t *first_time, const double *prev_states,
                       const int32_t *prev_count, const double *dyn_cur, const double *pred_pos,
                       const double *pred_size, const double *prob, int32_t *ob_idx, int32_t *cand_type,
                       int32_t *cand_slot, double *closest_prob, double *single_pos, double *single_size,
                       double *pair_pos, double *pair_size);

#ifdef __cplusplus
}
#endif
#endif
