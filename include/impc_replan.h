/*
 * impc_replan.h -- C-ABI of the planner state a batched makePlanWithPred carries between replans
 * on the device (reference: trajectory_planner/include/trajectory_planner/mpcPlanner.cpp).
 *
 * After a replan, each planning instance that took part either has a plan -- the selected
 * candidate of the fan-out branch (:629-639) or the single solve of the first-plan / no-prediction
 * branch (:645-659) -- or none (validTraj = false).  A plan becomes the instance's
 * currentStatesSol_ / currentControlsSol_: the next replan's warm start (solveTraj :485-509, all
 * states then all controls, i.e. the QP solution x itself), its obstacle linearisation point
 * (castMPCToQPConstraintMatrix :1042-1051) and the fan-out's closest-obstacle reference
 * (findClosestObstacle :675-707); firstTime_ clears (:637 / :656).  An instance without a plan
 * keeps its previous state and flag.
 */
#ifndef IMPC_REPLAN_H
#define IMPC_REPLAN_H
#include <stdint.h>
#include "impc_qp.h"
#ifdef __cplusplus
extern "C" {
#endif

/* Commit one replan's plans into the per-instance device state.  Entry r (< count) belongs to
 * planning instance inst[r]; its plan is, either
 *   fan-out branch  (x_cand != NULL): the candidate best_cand[r] of x_cand[r * ncand ..] (device
 *                   addresses of the candidates' QP solutions, impc_fanout_candidates_device; a
 *                   negative best_cand = no valid candidate, impc_select_best_device), or
 *   single solve    (x_rows != NULL): row r of the QP-major solutions x_rows [count][n], valid
 *                   when solveTraj succeeded, i.e. info_rows[r].status_val != OSQP_NON_CVX
 *                   (:513-518).
 * State (DEVICE, indexed by instance): plan_x [*][n] (the warm start), plan_states [*][horizon][8]
 * (the linearisation point, = plan_x's first 8 * horizon values), prev_count [*] (horizon once a
 * plan exists), first_time [*] (cleared), valid [*] (1 / 0 for the listed instances).  n must be
 * 13 * horizon - 5 (8 horizon states + 5 (horizon - 1) controls).  Asynchronous on `stream`. */
int impc_replan_commit_device(impc_ctx ctx, int32_t horizon, int64_t n, int64_t count, const int64_t *inst,
                              const uint64_t *x_cand, int32_t ncand, const int32_t *best_cand, const double *x_rows,
                              const impc_info *info_rows, double *plan_x, double *plan_states, int32_t *prev_count,
                              int8_t *first_time, int8_t *valid, void *stream);

#ifdef __cplusplus
}
#endif
#endif
