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
#include "impc_mpc.h"
#ifdef __cplusplus
extern "C" {
#endif

/* Commit one replan's plans into the per-instance device state.  Entry r (< count) belongs to
 * planning instance inst[r]; its plan is, either
 *   fan-out branch  (x_cand != NULL): the candidate best_cand[r] of x_cand[r * ncand ..] (device
 *                   addresses of the candidates' QP solutions, impc_fanout_candidates_device; a
 *                   negative best_cand = no valid candidate, impc_select_best_device), or
 *   single solve    (x_rows != NULL): row r of the QP-major solutions x_rows [count][n], valid
 *                   when solveTraj succeeded: initSolver did (setup_exitflag 0) and solveProblem
 *                   returned NoError -- osqp_solve's exitflag, 0 for every final status including
 *                   infeasible and NON_CVX (x = OSQP_NAN), 1 only after a failed adaptive-rho
 *                   refactorisation (status UNSOLVED) (:475-478, :513-518).
 * State (DEVICE, indexed by instance): plan_x [*][n] (the warm start), plan_states [*][horizon][8]
 * (the linearisation point, = plan_x's first 8 * horizon values), prev_count [*] (horizon once a
 * plan exists), first_time [*] (cleared), valid [*] (1 / 0 for the listed instances).  n must be
 * 13 * horizon - 5 (8 horizon states + 5 (horizon - 1) controls).  Asynchronous on `stream`. */
int impc_replan_commit_device(impc_ctx ctx, int32_t horizon, int64_t n, int64_t count, const int64_t *inst,
                              const uint64_t *x_cand, int32_t ncand, const int32_t *best_cand, const double *x_rows,
                              const impc_info *info_rows, double *plan_x, double *plan_states, int32_t *prev_count,
                              int8_t *first_time, int8_t *valid, void *stream);

/* ======================================================================================
 * The whole batched makePlanWithPred behind one call (mpcPlanner.cpp:571-661; its C++ caller is
 * mpcNavigation.cpp:316-322).  A replan object holds, for I planning instances with up to K
 * tracked dynamic obstacles each (K_i = predPos.size() per instance and per replan,
 * updatePredObstacles :343-373 -- the detector keeps the obstacles within range and field of view,
 * onboard_detector fakeDetector.cpp:493, so the count varies), the planner state (plan_x /
 * plan_states / prev_count / first_time / valid, as above) and every device buffer and solver
 * batch of a replan, allocated once.
 *
 * impc_replan_run, per instance, as the reference decides (:593-606):
 *   FANOUT          not firstTime_ and predictions present (K_i >= 1): findClosestObstacle +
 *                   getIntentComb (:663-769), the six candidates' castMPCToQP* (four with K_i and
 *                   two with K_i + 1 obstacles), their solveTraj with timeLimit, candidate validity
 *                   (solveTraj's success as for the commit above: OSQP_NAN plans of infeasible or
 *                   diverged QPs included, :475-478, :513-518),
 *                   getTrajectoryScore + evaluateTraj (:771-887);
 *   SINGLE_FIRST    firstTime_ (static and dynamic obstacles cleared, :593-602), or no predictions
 *                   and no current obstacles: ONE obstacle-free solveTraj, no time limit, no warm
 *                   start on a first plan;
 *   SINGLE_CURRENT  not firstTime_, no predictions, c_i >= 1 current dynamic obstacles kept: ONE
 *                   solveTraj with each obstacle's current position / size held over the horizon
 *                   (updateDynamicObstacles :316-341);
 * all of it in ONE grouped solve, then every plan committed into the state (:636-639 / :653-657).
 * The QPs are grouped by obstacle count: shape k (0 .. K + 1) is one solver batch holding every
 * QP of the replan with k dynamic-obstacle rows per stage -- first plans (k = 0), current-obstacle
 * solves (k = c_i), single-intent candidates (k = K_i) and two-intent candidates (k = K_i + 1) -- and
 * the grouped launch spans all of them.  With num_static = S_st > 0 every QP not on a first plan
 * also has S_st static-obstacle rows per stage (after the dynamic ones, with the reference's
 * isDyamic index quirk, :1194), shape 0 holds the not-first plans without dynamic obstacles, and
 * one more shape, K + 2, holds the first plans (no obstacle rows at all).  Which rows exist is decided on the device (a scan over the
 * instances), and the solver reads each shape's QP count from device memory: the call never
 * synchronises with the device and nothing returns to the host -- it queues the whole replan and
 * returns.  Device memory: shape k's batch is sized for its worst case (I rows for k = 0, 4 I for
 * 1 <= k <= K, 2 I for K + 1), about (4 K + 3) I QPs of storage.
 *
 * The budget (:609-628): candidates are issued only while the replan's elapsed time is below
 * issue_cutoff_s (0.15 s); every candidate carries timeLimit = max(limit - t, limit) (= limit for
 * t >= 0).  All six candidates of every instance are issued at one instant -- the end of the
 * device-side assembly -- so the cut-off is one check, made on the device: elapsed = elapsed_s +
 * the device clock from the call's first kernel to the end of the assembly.  Past it no candidate
 * is issued and every fan-out instance selects nothing (validTraj = false).  The single-solve
 * branch has no cut-off.
 * ====================================================================================== */
typedef struct impc_replan_s *impc_replan;

#define IMPC_REPLAN_FANOUT 0
#define IMPC_REPLAN_SINGLE_FIRST 1
#define IMPC_REPLAN_SINGLE_CURRENT 2

typedef struct {
    int64_t instances;         /* I planning instances */
    int32_t num_obstacles;     /* K, 1 <= K <= 30: the most dynamic obstacles an instance tracks
                                  (the obstacle slots of every per-instance input array) */
    int32_t pred_len;          /* L prediction steps per obstacle trajectory */
    impc_mpc_params mpc;       /* initParam values; mpc.horizon = N (the selection's safety
                                  distances are mpc.dynamic_safety_dist / static_safety_dist) */
    impc_settings settings;    /* every solveTraj's OSQP settings (the reference: defaults,
                                  verbose off, warm start on) */
    double issue_cutoff_s;     /* makePlanWithPred's 0.15 s; <= 0: no cut-off */
    int32_t queue_order;       /* IMPC_QUEUE_* of the grouped solve (results are identical) */
    int32_t num_static;        /* S_st, 0 <= S_st <= 30: the static obstacles every instance carries
                                  (obclustering_->getStaticObstacles(), :594) into each solveTraj
                                  and getTrajectoryScore not on a first plan (:593-602, :615-620,
                                  :652); 0 = none (the live planner: clustering disabled, :191-193) */
} impc_replan_config;

/* Per-replan inputs, all DEVICE pointers (K = num_obstacles, L = pred_len, N = horizon).  An
 * instance's obstacles are its first K_i (predictions) / c_i (current) slots. */
typedef struct {
    const double *pos, *vel;       /* [I][3] updateCurrStates */
    const double *xref;            /* [I][N][8] getXRef (e.g. impc_reference_traj_device) */
    const double *dyn_cur;         /* [I][K][3] dynamicObstaclesPos_ (current positions) */
    const double *pred_pos;        /* [I][K][4][L][3] obPredPos_ */
    const double *pred_size;       /* [I][K][4][L][3] obPredSize_ */
    const double *prob;            /* [I][K][4] obIntentProb_ */
    const int8_t *has_pred;        /* [I] obPredPos_.size() != 0; NULL = every instance */
    const double *cur_size;        /* [I][K][3] dynamicObstaclesSize_ kept without predictions;
                                      NULL = none (updatePredObstacles clears them, :364-371) */
    const int32_t *cur_count;      /* [I] c_i current obstacles (0 .. K); NULL with cur_size = K */
    double solver_time_limit;      /* solverTimeLimit_ (0.05 s); <= 0: settings.time_limit */
    double elapsed_s;              /* seconds of the replan already spent before this call
                                      (counted against the issue cut-off) */
    const int32_t *num_pred;       /* [I] K_i = predPos.size() (0 .. K; 0 = no predictions, as
                                      has_pred = 0); NULL = K for every instance */
    const double *st_centroid;     /* [I][S_st][3] staticObstacle::centroid; with num_static > 0 */
    const double *st_size;         /* [I][S_st][3] staticObstacle::size */
    const double *st_yaw;          /* [I][S_st]    staticObstacle::yaw */
} impc_replan_inputs;

/* What the last impc_replan_run did (host values; reading them synchronises the context). */
typedef struct {
    int64_t fanout, single_first, single_current; /* instances per branch */
    int32_t issued;                                /* candidates issued (cut-off not reached) */
    int32_t reserved;
    double time_limit;                             /* the candidates' time limit (s, 0 = none) */
    double stage_s;                                /* branch table + assembly on the device clock
                                                      (s): the elapsed time the cut-off adds */
    double total_s;                                /* host wall of the call (s); the whole replan
                                                      is queued, not waited for */
} impc_replan_stats;

int impc_replan_create(impc_ctx ctx, const impc_replan_config *cfg, impc_replan *out);
int impc_replan_destroy(impc_replan rp);
/* The planner state from the host: plan_x [I][n] (currentStatesSol_ then currentControlsSol_ in
 * QP variable order, n = 13 N - 5; NULL = zeros) and first_time [I] (NULL = every instance on its
 * first plan).  currentStatesSol_.size() follows: 0 on a first plan, N once a plan exists (the
 * reference sets firstTime_ = false only together with a full plan, :636-639 / :653-657). */
int impc_replan_set_state(impc_replan rp, const double *plan_x, const int8_t *first_time);
/* One batched makePlanWithPred (see above).  Stream-ordered on the context stream; returns once
 * every stage is queued (no host synchronisation inside the call). */
int impc_replan_run(impc_replan rp, const impc_replan_inputs *in);
int impc_replan_get_stats(impc_replan rp, impc_replan_stats *out);

/* DEVICE views, valid until the next run / destroy.  State: plan_x [I+1][n] (row I stays zero),
 * plan_states [I+1][N][8], prev_count [I], first_time [I], valid [I] (the last replan's validTraj).
 * Per instance of the last run: branch [I] (IMPC_REPLAN_*), best_cand [I] (fan-out instances:
 * the selected candidate or -1; -1 otherwise), ob_idx [I] (closest obstacle; -1 for single-solve
 * instances), cand_type / cand_slot [I][6] (getIntentComb order; -1 for single-solve instances),
 * num_obs [I] (fan-out: K_i; single solve: the dynamic-obstacle count of its QP = its shape, except
 * a first plan with num_static > 0: shape K + 2), slot_row [I][6] (fan-out: the row of slot s in
 * shape K_i (s < 4) or K_i + 1 (s >= 4); single solve: its row in its shape at [0]; -1
 * elsewhere), shape [I] (the shape of the instance's single solve; fan-out: K_i). */
typedef struct {
    double *plan_x, *plan_states;
    int32_t *prev_count;
    int8_t *first_time, *valid, *branch;
    int32_t *best_cand, *ob_idx, *cand_type, *cand_slot;
    int32_t *num_obs, *slot_row;
    int32_t *shape;
} impc_replan_view;
int impc_replan_view_device(impc_replan rp, impc_replan_view *out);

/* Inspection of the last run (tests, tools; synchronises the context): shape k = the QPs with k
 * dynamic-obstacle rows per stage (0 <= k <= K + 1; k = K + 2: the first plans of a replan object
 * with num_static > 0) -- its solver batch, the number of its rows solved in
 * the last replan, each row's instance and kind (DEVICE int32 row_inst / int8 row_code [count]:
 * 0..3 single-intent slot, 4..5 two-intent slot, 6 first plan / no obstacles, 7 current obstacles;
 * single solves first, then the candidates, each in ascending instance order) and the assembled
 * values (DEVICE, QP-major, `count` rows). */
#define IMPC_REPLAN_ROW_FIRST 6
#define IMPC_REPLAN_ROW_CURRENT 7
int impc_replan_shape(impc_replan rp, int32_t obstacles, impc_batch *batch, int64_t *count, const int32_t **row_inst,
                      const int8_t **row_code, const double **Px, const double **q, const double **Ax,
                      const double **l, const double **u);

/* The vehicle following its plan (mpc_node.cpp:216-224: after a successful makePlan, currPos =
 * getPos(dt), currVel = getVel(dt)): for every instance whose last replan produced a plan
 * (valid[i] = 1), pos[i] / vel[i] = mpcPlanner::getPos(t) / getVel(t) (mpcPlanner.cpp:1257-1290:
 * idx = floor(t / ts) clamped to the plan, linear interpolation towards state idx + 1); other
 * instances keep pos / vel.  DEVICE pos, vel [I][3], updated in place; stream-ordered after the
 * replan.  The next replan's x0 without a host round trip. */
int impc_replan_advance_device(impc_replan rp, double t, double *pos, double *vel);

/* The same for a receding window of single QPs (a persistent batch of mpcPlanner QPs, n = 13
 * horizon - 5): QP b's next x0, pos[b] / vel[b] [B][3], = getPos(t) / getVel(t) of its own last
 * solution when the solve returned one (status SOLVED, SOLVED_INACCURATE, MAX_ITER_REACHED,
 * TIME_LIMIT_REACHED), and (lin_states != NULL) its next linearisation point lin_states[b]
 * [horizon][8] = the solution's states (currentStatesSol_); a QP without a solution (infeasible: x
 * is OSQP_NAN) keeps both.  DEVICE arrays, updated in place after the batch's last solve, on the
 * context stream. */
int impc_batch_follow_plan_device(impc_batch b, int32_t horizon, double ts, double t, double *pos, double *vel,
                                  double *lin_states);

#ifdef __cplusplus
}
#endif
#endif
