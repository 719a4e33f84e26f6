/*
 * impc_minsnap.h -- the minimum-snap polynomial-trajectory QP of trajPlanner::polyTrajSolver
 * (the second OSQP caller of the reference, a persistent OsqpEigen::Solver per axis), assembled
 * for a batch of paths; the QPs are then solved by impc_batch_* (generic kernel) and kept
 * between solves with impc_batch_update_bounds, as polyTrajSolver::updateProblem does.
 *
 * Replaces (reference trajectory_planner/include/trajectory_planner/polyTrajSolver.cpp):
 *   updatePath / getConstraintNum   :53-61, :156-160   n = (deg+1) S, m as below (S segments)
 *   avgTimeAllocation               :129-142           T_0 = 0, T_i = T_{i-1} + |p_i - p_{i-1}| / v
 *   constructP                      :240-272           per segment, i, j in [diff, deg]:
 *                                                      prod_{d<diff} (i-d)(j-d) / (i+j-2 diff+1)
 *                                                      (normalised time: no duration factor)
 *   constructQ                      :308-311           q = 0
 *   constructA                      :313-602           position (2 ends, S-1 waypoints, S-1 C0),
 *                                                      velocity / acceleration (2 ends, S-1
 *                                                      continuity rows scaled by the neighbouring
 *                                                      durations), jerk / snap continuity when
 *                                                      continuity_degree >= 3 / 4
 *   constructBound                  :604-818           per axis: waypoints (+- sc_deviation with
 *                                                      soft constraints), end velocities and
 *                                                      accelerations, zeros for continuity rows
 *   solveX/Y/Z                      :831-868           coefficient d of segment s divided by
 *                                                      (T_{s+1} - T_s)^d
 *   setCorridorConstraint /        :960-1012          corridor rows (impc_minsnap_corridor_*): segment
 *   updateCorridorParam,                               i with size r_i != 0 gets one row per sample t
 *   constructA corridor rows       :557-579           of for (t = 0; t <= 1; t += 1/numCorridor_i),
 *   constructBound corridor rows   :815-835           entries pow(t, d), bounds interp(p_i, p_{i+1}, t)
 *                                                      -+ r_i, in std::unordered_map<double, pose>
 *                                                      order (libstdc++, as the reference iterates)
 * m = 2S + (S+1) + (S+1) + (S-1)(continuity_degree - 2) [+ the corridor samples].
 * P is returned as its upper triangle (OsqpEigen keeps triangularView<Upper>, Data.tpp:38).
 */
#ifndef IMPC_MINSNAP_H
#define IMPC_MINSNAP_H
#include <stdint.h>
#include "impc_mpc.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int32_t poly_degree;       /* poly_traj/polynomial_degree (7) */
    int32_t diff_degree;       /* poly_traj/differential_degree (4: snap) */
    int32_t continuity_degree; /* poly_traj/continuity_degree (3); values < 2 act as 2 (:56); <= 4 */
    double desired_vel;        /* time allocation velocity */
    int32_t soft_constraint;   /* poly_traj/soft_constraint */
    double sc_deviation[3];    /* waypoint half-widths per axis with soft constraints */
} impc_minsnap_params;

/* Problem dimensions for a path of num_waypoints >= 2 points.  Returns 0 on success. */
int impc_minsnap_dims(const impc_minsnap_params *p, int32_t num_waypoints, impc_qp_dims *out);

/* The shared CSC patterns (path independent). */
int impc_minsnap_build_pattern(const impc_minsnap_params *p, int32_t num_waypoints, int64_t *Pp, int64_t *Pi,
                               int64_t *Ap, int64_t *Ai);

/* Values for nb paths, three QPs per path (axes x, y, z; QP 3 b + a):
 *   path                 [nb][W][3]   waypoints
 *   init_vel, end_vel, init_acc, end_acc  [nb][3]  (NULL = zero, setDefaultInit :148-154)
 * Outputs (QP-major): Px [3 nb][nnzP], q [3 nb][n], Ax [3 nb][nnzA], l, u [3 nb][m];
 * seg_time [nb][W] (desiredTime_).  Any output may be NULL. */
int impc_minsnap_build_values(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints, const double *path,
                              const double *init_vel, const double *end_vel, const double *init_acc,
                              const double *end_acc, double *Px, double *q, double *Ax, double *l, double *u,
                              double *seg_time);

/* Bounds only (polyTrajSolver::updateProblem -> updateBounds), same layout as above. */
int impc_minsnap_build_bounds(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints, const double *path,
                              const double *init_vel, const double *end_vel, const double *init_acc,
                              const double *end_acc, double *l, double *u);

/* Corridor constraints.  numCorridor_i = ceil((T_{i+1} - T_i) * corridor_res) of every segment
 * (0 where corridor_size is 0) for nb paths: corridor_size, corridor_num [nb][W-1].  The sample
 * times, hence the pattern and the A values, depend only on the numCorridor vector, so a batch
 * holds paths with equal vectors; the *_corridor_values / _bounds calls take that vector and fail
 * (return 1) for a path whose own vector differs.  corridor_num = NULL is the plain problem. */
int impc_minsnap_corridor_num(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints, const double *path,
                              const double *corridor_size, double corridor_res, int32_t *corridor_num);
int impc_minsnap_corridor_dims(const impc_minsnap_params *p, int32_t num_waypoints, const int32_t *corridor_num,
                               impc_qp_dims *out);
int impc_minsnap_corridor_pattern(const impc_minsnap_params *p, int32_t num_waypoints, const int32_t *corridor_num,
                                  int64_t *Pp, int64_t *Pi, int64_t *Ap, int64_t *Ai);
int impc_minsnap_corridor_values(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints, const double *path,
                                 const double *init_vel, const double *end_vel, const double *init_acc,
                                 const double *end_acc, const int32_t *corridor_num, const double *corridor_size,
                                 double corridor_res, double *Px, double *q, double *Ax, double *l, double *u,
                                 double *seg_time);
int impc_minsnap_corridor_bounds(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints, const double *path,
                                 const double *init_vel, const double *end_vel, const double *init_acc,
                                 const double *end_acc, const int32_t *corridor_num, const double *corridor_size,
                                 double corridor_res, double *l, double *u);

/* solveX/Y/Z's rescaling of the solutions to real time, in place: x [3 nb][n]. */
int impc_minsnap_unscale(const impc_minsnap_params *p, int64_t nb, int32_t num_waypoints, const double *seg_time,
                         double *x);

#ifdef __cplusplus
}
#endif
#endif
