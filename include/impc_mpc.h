/*
 * impc_mpc.h -- C-ABI for the MPC -> QP assembly that trajPlanner::mpcPlanner performs before
 * every OSQP call (reference: trajectory_planner/include/trajectory_planner/mpcPlanner.cpp).
 *
 * It replaces, for a whole batch of planning instances at once:
 *   updateObstacleParam          mpcPlanner.cpp:1148-1197
 *   setDynamicsMatrices          mpcPlanner.cpp:891-901
 *   setInequalityConstraints     mpcPlanner.cpp:904-921
 *   setWeightMatrices            mpcPlanner.cpp:925-931
 *   castMPCToQPHessian           mpcPlanner.cpp:932-951
 *   castMPCToQPGradient          mpcPlanner.cpp:952-966
 *   castMPCToQPConstraintMatrix  mpcPlanner.cpp:984-1072
 *   castMPCToQPConstraintVectors mpcPlanner.cpp:1074-1146
 * including the reference's float-rounding of the Hessian / dynamics entries
 * (mpcPlanner.cpp:940,946,1003,1014), the global-index R quirk (:945) and the isDyamic
 * static-index quirk (:1194).  Variable order: all states x_0..x_{N-1} (8 each), then all
 * controls u_0..u_{N-2} (5 each) (:491,501).
 *
 * All QPs of one call share one sparsity pattern (same N, obstacle counts, half-spaces and
 * parameters); values are returned QP-major (QP b's block at b * len).
 * Sparse matrices are CSC with int64 indices (OSQP c_int under DLONG, osqp_configure.h:31).
 */
#ifndef IMPC_MPC_H
#define IMPC_MPC_H
#include <stdint.h>
#include "impc_qp.h"
#ifdef __cplusplus
extern "C" {
#endif

/* The ROS parameters mpcPlanner::initParam reads (mpcPlanner.cpp:19-173) plus the values set
 * through updateMaxVel/updateMaxAcc/updatePath(ts)/updateFovParam. */
typedef struct {
    int32_t horizon;        /* mpc_planner/horizon: N state nodes, N-1 control stages */
    int32_t num_half_space; /* 0 on the live path (2-arg updateCurrStates, :257-263), 2 with FOV */
    double ts;              /* updatePath(path, ts) */
    double max_vel, max_acc;
    double y_range_min, y_range_max, z_range_min, z_range_max;
    double static_safety_dist, dynamic_safety_dist;
    double static_slack, dynamic_slack; /* *_constraint_slack_ratio */
    double position_weight, velocity_weight, acceleration_weight;
    double half_max[3], half_min[3]; /* updateFovParam (:274-295), used when num_half_space = 2 */
} impc_mpc_params;

typedef struct {
    int64_t n, m, nnzP, nnzA;
} impc_qp_dims;

/* Problem dimensions of one QP shape.  Returns 0 on success. */
int impc_mpc_dims(const impc_mpc_params *p, int32_t num_static, int32_t num_dynamic, impc_qp_dims *out);

/* Shared CSC patterns (P upper triangle as OsqpEigen passes it, Data.tpp:38; A full). */
int impc_mpc_build_pattern(const impc_mpc_params *p, int32_t num_static, int32_t num_dynamic, int64_t *Pp,
                           int64_t *Pi, int64_t *Ap, int64_t *Ai);

/* Per-QP values for nb instances.
 *   curr_pos, curr_vel : [nb][3]           (updateCurrStates)
 *   xref               : [nb][N][8]        (getXRef)
 *   lin_states         : [nb][N][8] or NULL (currentStatesSol_: linearisation point; NULL =
 *                        first call, linearise at curr_pos, :1042-1051)
 *   st_centroid/size   : [nb][S][3], st_yaw : [nb][S]      (staticObstacle)
 *   dyn_pos/dyn_size   : [nb][K][L][3]     (predicted positions / sizes, L = pred_len;
 *                        stage j >= L uses entry L-1 as the reference's .back() does)
 * Outputs (QP-major): Px [nb][nnzP], q [nb][n], Ax [nb][nnzA], l [nb][m], u [nb][m].
 * l/u carry IEEE +-INFINITY where the reference does (OSQP clamps them to +-1e30). */
int impc_mpc_build_values(const impc_mpc_params *p, int64_t nb, const double *curr_pos, const double *curr_vel,
                          const double *xref, const double *lin_states, int32_t num_static, const double *st_centroid,
                          const double *st_size, const double *st_yaw, int32_t num_dynamic, int32_t pred_len,
                          const double *dyn_pos, const double *dyn_size, double *Px, double *q, double *Ax, double *l,
                          double *u);

/* Warm-start primal vector of solveTraj (mpcPlanner.cpp:487-509): previous states/controls,
 * zero when absent.  prev_states [nb][N][8] / prev_controls [nb][N-1][5] may be NULL. */
/* ---- On-device assembly: the same values, built on the GPU.
 * A builder holds, on the device, the instance-independent part of one (horizon, #static,
 * #dynamic) shape -- P, the dynamics/box/half-space entries of A, the bound templates -- and the
 * CSC slots of the obstacle-row entries; impc_mpc_build_values_device then fills q, the x0 rows
 * and the obstacle rows of nb instances (one workgroup per QP, same expressions as
 * castMPCToQPConstraintMatrix/Vectors).  Dynamic-obstacle entries are bit-identical to
 * impc_mpc_build_values; static obstacles with yaw go through the device cos/sin (a few ulp). */
typedef struct impc_mpc_builder_s *impc_mpc_builder;
int impc_mpc_builder_create(impc_ctx ctx, const impc_mpc_params *p, int32_t num_static, int32_t num_dynamic,
                            int32_t pred_len, impc_mpc_builder *out);
int impc_mpc_builder_destroy(impc_mpc_builder b);
/* DEVICE pointers, layouts as impc_mpc_build_values; lin_states may be NULL (first call).
 * Outputs QP-major (ready for impc_batch_set_values_device).  Asynchronous on `stream`
 * (NULL = the context's stream). */
int impc_mpc_build_values_device(impc_mpc_builder b, int64_t nb, const double *curr_pos, const double *curr_vel,
                                 const double *xref, const double *lin_states, const double *st_centroid,
                                 const double *st_size, const double *st_yaw, const double *dyn_pos,
                                 const double *dyn_size, double *Px, double *q, double *Ax, double *l, double *u,
                                 void *stream);

int impc_mpc_warm_start(const impc_mpc_params *p, int64_t nb, const double *prev_states, const double *prev_controls,
                        double *x_ws);

/* mpcPlanner::getXRef / getReferenceTraj (mpcPlanner.cpp:968-981, 1199-1231) for `ni` planning
 * instances on the device, one thread each.  Instance i follows its input path (updatePath,
 * :307-314): points path[path_ptr[i] .. path_ptr[i + 1]) of path (x, y, z), and its state
 * last_idx[i] (lastRefStartIdx_; 0 after updatePath), read and updated in place.  The nearest
 * path point to curr_pos[i] is searched in [last_idx, min(last_idx + (int)(3.0 / ts), len)) (first
 * minimum of the Euclidean distance), then `horizon` consecutive points from there, padded with
 * the last point, become xref[i][k] = (x, y, z, 0, 0, 0, 0, 0) -- an empty path gives curr_pos at
 * every step (state unchanged).  DEVICE pointers: path_ptr [ni + 1] int64, path [*][3],
 * curr_pos [ni][3], last_idx [ni] int32, xref [ni][repeat][horizon][8] (each instance's reference
 * written `repeat` times, the layout of a replan's per-candidate copies).  Asynchronous on
 * `stream` (NULL = the context's stream). */
int impc_reference_traj_device(impc_ctx ctx, int32_t horizon, double ts, int64_t ni, const int64_t *path_ptr,
                               const double *path, const double *curr_pos, int32_t *last_idx, int32_t repeat,
                               double *xref, void *stream);

/* Per-candidate copies of per-instance device rows (makePlanWithPred hands every candidate of a
 * replan the same x0, xRef and linearisation point, mpcPlanner.cpp:609-628): dst row r * repeat + c
 * = src row r, rows of row_bytes bytes (a multiple of 8).  Asynchronous on `stream`. */
int impc_repeat_rows_device(impc_ctx ctx, const void *src, int64_t rows, int64_t row_bytes, int32_t repeat,
                            void *dst, void *stream);

/* Row gather on the device: dst row r = src row idx[r], r < count (idx a DEVICE int64 array; rows
 * of row_bytes bytes, a multiple of 4).  The batched replan compacts the planning instances that
 * take one makePlanWithPred branch with it.  Asynchronous on `stream`. */
int impc_gather_rows_device(impc_ctx ctx, const void *src, int64_t row_bytes, const int64_t *idx, int64_t count,
                            void *dst, void *stream);

/* Strided device-to-device copy (hipMemcpy2DAsync): `rows` rows of `width` bytes from src (row
 * pitch spitch bytes) to dst (pitch dpitch) -- a receding window's next slice of each QP's longer
 * reference / prediction arrays, or x0 columns out of the QP-major solutions.  Asynchronous on
 * `stream` (NULL = the context's stream). */
int impc_copy_rows_device(impc_ctx ctx, void *dst, int64_t dpitch, const void *src, int64_t spitch, int64_t width,
                          int64_t rows, void *stream);

#ifdef __cplusplus
}
#endif
#endif
