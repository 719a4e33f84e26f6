/*
 * impc_select.h -- device-side candidate scoring and selection of a replan (libimpc_qp.so).
 *
 * Replaces, batched over planning instances, the host loop of mpcPlanner::makePlanWithPred that
 * scores every solved intent-combination candidate and picks one (reference
 * trajectory_planner/include/trajectory_planner/mpcPlanner.cpp):
 *
 *   getTrajectoryScore  :771-778   per candidate (consistency, detour, safety)
 *   getConsistencyScore :780-800   mean distance to the previous plan over <= 10 steps, floor 0.1
 *   getDetourScore      :802-814   mean distance to the reference, floor 0.1
 *   getSafetyScore      :816-848   tanh-weighted planar obstacle distance
 *   evaluateTraj        :850-887   mean-normalised scores x intent weight, first maximum
 *   makePlanWithPred    :606-634   only successful candidates are scored; intentType = the
 *                                  candidate's index in getIntentComb order
 *
 * Semantics follow the reference exactly, including its quirks: dynamic obstacles enter
 * maxSize with their full size and static ones with half of it; the weight of candidate i is
 * entry i of (STOP, LEFT, RIGHT, FORWARD, max(LEFT,FORWARD), max(RIGHT,FORWARD)) of the closest
 * obstacle's intent probabilities; a candidate whose obstacles are all far enough that every
 * tanh weight rounds to 0 gets a NaN safety score, as in the reference.
 *
 * Candidate states are read straight from QP solutions (variable order of mpcPlanner: state k at
 * x[8k .. 8k+7]), e.g. the device result arrays of impc_batch_device_results, so a replan's
 * solve -> score -> select stays on the GPU.  Intent probability order: dynamicPredictor's enum
 * (FORWARD, LEFT, RIGHT, STOP).
 */
#ifndef IMPC_SELECT_H
#define IMPC_SELECT_H
#include <stdint.h>

#include "impc_qp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int32_t horizon;            /* N: states scored per candidate */
    int32_t num_candidates;     /* C: candidates per instance (<= 6, getIntentComb order) */
    int32_t max_dynamic;        /* KMAX: dynamic obstacle slots per candidate (padded) */
    int32_t pred_len;           /* L >= N: steps per predicted obstacle trajectory */
    int32_t num_static;         /* S: static obstacles per instance */
    int32_t prev_len;           /* P: states of the previous plan (currentStatesSol_) per instance */
    double dynamic_safety_dist; /* mpc_planner/dynamic_safety_dist */
    double static_safety_dist;  /* mpc_planner/static_safety_dist */
} impc_select_params;

/*
 * All pointers are DEVICE pointers; asynchronous on `stream` (NULL = the context's stream).
 *   x_cand      [I*C]  device pointers to each candidate's QP primal solution
 *   valid       [I][C] int8: solveTraj succeeded (candidates with 0 are skipped, :612-620)
 *   first_time  [I]    int8: planner's firstTime_ (consistency score 0)
 *   prev_states [I][P][8], prev_count [I] (valid states of the previous plan, <= P)
 *   xref        [I][N][8]
 *   st_centroid, st_size [I][S][3]
 *   dyn_count   [I][C] obstacles of each candidate (<= KMAX)
 *   dyn_pos, dyn_size [I][C][KMAX][L][3]
 *   prob        [I][4] intent probabilities of the closest obstacle (FORWARD, LEFT, RIGHT, STOP)
 * Outputs:
 *   best_cand   [I] int32: selected candidate index (-1: no successful candidate)
 *   best_pos    [I] int32: its position among the successful candidates (evaluateTraj's return)
 *   scores      [I][C][3] raw (consistency, detour, safety); weighted [I][C] (NaN for skipped)
 */
int impc_select_best_device(impc_ctx ctx, const impc_select_params *p, int64_t instances,
                            const double *const *x_cand, const int8_t *valid, const int8_t *first_time,
                            const double *prev_states, const int32_t *prev_count, const double *xref,
                            const double *st_centroid, const double *st_size, const int32_t *dyn_count,
                            const double *dyn_pos, const double *dyn_size, const double *prob, int32_t *best_cand,
                            int32_t *best_pos, double *scores, double *weighted, void *stream);

/* Same with host arrays (copied to / from the device, synchronous), except x_cand: a HOST array
 * of I*C DEVICE pointers to the candidates' solutions. */
int impc_select_best(impc_ctx ctx, const impc_select_params *p, int64_t instances, const double *const *x_cand,
                     const int8_t *valid, const int8_t *first_time, const double *prev_states,
                     const int32_t *prev_count, const double *xref, const double *st_centroid, const double *st_size,
                     const int32_t *dyn_count, const double *dyn_pos, const double *dyn_size, const double *prob,
                     int32_t *best_cand, int32_t *best_pos, double *scores, double *weighted);

#ifdef __cplusplus
}
#endif
#endif
