/*
 * impc_qp.h -- C-ABI of the MI355X batched OSQP-0.6.2-equivalent QP solver (libimpc_qp.so).
 *
 * Drop-in boundary: the OsqpEigen::Solver call sequence mpcPlanner::solveTraj makes for every
 * QP (reference trajectory_planner/include/trajectory_planner/mpcPlanner.cpp:436-527):
 *
 *   reference call (file:line)                               replaced by
 *   ------------------------------------------------------   -------------------------------
 *   OsqpEigen::Solver solver;            mpcPlanner.cpp:436  impc_ctx_create + impc_batch_create
 *   settings()->setVerbosity/WarmStart/TimeLimit   :440-444  impc_default_settings +
 *     (OsqpEigen Settings.hpp:172-196 -> OSQPSettings          impc_batch_set_settings
 *      types.h:139-176)
 *   data()->setNumberOfVariables/Constraints       :450-452  impc_batch_create(n, m, ...)
 *   data()->setHessianMatrix   (Data.tpp:13-50, upper)  :453  impc_batch_create (pattern) +
 *   data()->setLinearConstraintsMatrix (Data.tpp:52-87) :461    impc_batch_set_values (values)
 *   data()->setGradient/setLowerBound/setUpperBound :457-469  impc_batch_set_values
 *   initSolver()  -> osqp_setup (osqp.h:58)              :475  impc_batch_setup (device)
 *   setWarmStart(x, y) -> osqp_warm_start (osqp.h:157)   :509  impc_batch_warm_start
 *   solveProblem() -> osqp_solve (osqp.h:78)             :513  impc_batch_solve
 *   getSolution()                (Solver.hpp:131)        :526  impc_batch_get
 *   clearSolver() -> osqp_cleanup (osqp.h:90)            :527  impc_batch_destroy
 *   updateGradient/updateBounds (Solver.hpp:151-182;          impc_batch_update_lin_cost /
 *     osqp_update_lin_cost/bounds osqp.h:114-134)               impc_batch_update_bounds
 *
 * One batch = B independent QPs that share one sparsity pattern (the reference's QPs of one
 * (N, #obstacles) shape share it by construction).  Per-QP host arrays are QP-major: QP b's
 * block starts at b * len.  Indices are int64 (OSQP c_int with DLONG, osqp_configure.h:31),
 * values double (c_float).  Status and error codes are OSQP 0.6.2's (constants.h:18-51).
 *
 * Threading: a context and its batches belong to one host thread; solves are asynchronous on
 * the HIP stream passed in (NULL = the context's own stream); impc_batch_get synchronises.
 */
#ifndef IMPC_QP_H
#define IMPC_QP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* OSQP status values (constants.h:18-30) */
#define IMPC_DUAL_INFEASIBLE_INACCURATE 4
#define IMPC_PRIMAL_INFEASIBLE_INACCURATE 3
#define IMPC_SOLVED_INACCURATE 2
#define IMPC_SOLVED 1
#define IMPC_MAX_ITER_REACHED (-2)
#define IMPC_PRIMAL_INFEASIBLE (-3)
#define IMPC_DUAL_INFEASIBLE (-4)
#define IMPC_TIME_LIMIT_REACHED (-6)
#define IMPC_NON_CVX (-7)
#define IMPC_UNSOLVED (-10)

/* OSQP error values (constants.h:43-51) plus library-level errors */
#define IMPC_OK 0
#define IMPC_DATA_VALIDATION_ERROR 1
#define IMPC_SETTINGS_VALIDATION_ERROR 2
#define IMPC_LINSYS_SOLVER_INIT_ERROR 4
#define IMPC_NONCVX_ERROR 5
#define IMPC_MEM_ALLOC_ERROR 6
#define IMPC_WORKSPACE_NOT_INIT_ERROR 7
#define IMPC_DEVICE_ERROR 100
#define IMPC_INVALID_ARGUMENT 101
#define IMPC_UNSUPPORTED 102

/* Field-for-field mirror of OSQPSettings (types.h:139-176, PROFILING build). */
typedef struct {
    double rho;
    double sigma;
    int64_t scaling;
    int64_t adaptive_rho;
    int64_t adaptive_rho_interval; /* 0 = automatic: resolved to check_termination */
    double adaptive_rho_tolerance;
    double adaptive_rho_fraction;
    int64_t max_iter;
    double eps_abs;
    double eps_rel;
    double eps_prim_inf;
    double eps_dual_inf;
    double alpha;
    int64_t linsys_solver; /* accepted for API parity; the device factorisation is always used */
    double delta;
    int64_t polish; /* must be 0 (the reference never polishes); 1 -> IMPC_UNSUPPORTED */
    int64_t polish_refine_iter;
    int64_t verbose; /* ignored (no printing on device) */
    int64_t scaled_termination;
    int64_t check_termination;
    int64_t warm_start;
    double time_limit; /* seconds per QP, on the device clock from the start of the QP's setup; 0 = off */
} impc_settings;

/* Subset of OSQPInfo (types.h:66-89), one per QP. */
typedef struct {
    int64_t iter;
    int64_t status_val;
    int64_t rho_updates;
    int64_t setup_exitflag; /* per-QP osqp_setup outcome: 0, or IMPC_NONCVX_ERROR */
    double obj_val;
    double pri_res;
    double dua_res;
    double rho_estimate;
} impc_info;

typedef struct impc_ctx_s *impc_ctx;
typedef struct impc_batch_s *impc_batch;

/* osqp_set_default_settings (osqp.h:32) */
void impc_default_settings(impc_settings *s);

/* Message of the last error on this host thread. */
const char *impc_last_error(void);

/* Library/ABI version string (with the git revision the library was built at). */
const char *impc_version(void);
/* Build identity of this library: "src-<16 hex>" = a hash of every source file compiled into it
   and the compiler flags (kernel switches included).  Profiles record it (under profiles/); bench.py
   quotes measured HBM traffic only from a PMC summary whose build id equals the loaded library's. */
const char *impc_build_id(void);

int impc_ctx_create(int device, impc_ctx *out);
int impc_ctx_destroy(impc_ctx ctx);
/* The context's HIP stream (hipStream_t), for callers that want to enqueue around solves. */
void *impc_ctx_stream(impc_ctx ctx);
/* Block until all work of this context's device has finished (hipDeviceSynchronize). */
int impc_ctx_synchronize(impc_ctx ctx);

/* Shared pattern: P (n x n, upper triangle, CSC Pp[n+1]/Pi[nnzP]) and A (m x n, CSC Ap[n+1]/
 * Ai[nnzA]).  Runs the symbolic analysis (fill-reducing ordering of P + sigma I + A' R A, its
 * envelope, assembly schedule) once and allocates device storage for `batch` QPs. */
int impc_batch_create(impc_ctx ctx, int64_t n, int64_t m, const int64_t *Pp, const int64_t *Pi, const int64_t *Ap,
                      const int64_t *Ai, int64_t batch, impc_batch *out);
int impc_batch_destroy(impc_batch b);
/* A batch from the context's workspace pool: a released batch with the same pattern (n, m, P and
 * A compared entry by entry) and capacity is reused -- no symbolic or structure analysis, no
 * device allocation, no synchronisation -- else a new one is created.  It comes back in the state
 * impc_batch_create leaves (default settings, no values, no warm start, no time limits, FIFO
 * queue, every QP active, persistent workspace off, profiling off).  impc_batch_release returns it
 * to the pool: the next acquire's uploads are stream-ordered after anything still reading it.
 * impc_ctx_destroy frees the pool (impc_batch_destroy of a released batch takes it out of the
 * pool first).  The OsqpEigen front end's Solver (one per solveTraj call,
 * mpcPlanner.cpp:436 / :527) lives on it. */
int impc_batch_acquire(impc_ctx ctx, int64_t n, int64_t m, const int64_t *Pp, const int64_t *Pi, const int64_t *Ap,
                       const int64_t *Ai, int64_t batch, impc_batch *out);
/* Releasing a batch that is already in the pool fails (IMPC_INVALID_ARGUMENT); past 64 pooled
 * batches the oldest is destroyed. */
int impc_batch_release(impc_batch b);
/* The pool's size: pooled batches and the device bytes they hold (either pointer may be NULL). */
int impc_ctx_pool_stats(impc_ctx ctx, int64_t *batches, int64_t *device_bytes);

int impc_batch_set_settings(impc_batch b, const impc_settings *s);

/* Per-QP values, host, QP-major: Px [B][nnzP], q [B][n], Ax [B][nnzA], l [B][m], u [B][m].
 * Validated like osqp_setup's validate_data (l <= u).  Copied to the device (stream-ordered). */
int impc_batch_set_values(impc_batch b, const double *Px, const double *q, const double *Ax, const double *l,
                          const double *u);
/* Same, from device-resident QP-major arrays (no host round trip; validation skipped). */
int impc_batch_set_values_device(impc_batch b, const double *Px, const double *q, const double *Ax, const double *l,
                                 const double *u);

/* Shared-structure values (host arrays): the batch's QPs share P and every A entry except the
 * nvar positions var_pos (ascending indices into the CSC values of A) -- e.g. the replan QPs of
 * one shape, whose dynamics / box entries are the same and whose obstacle-row entries differ.
 * Px [nnzP] and Ax [nnzA] once, Ax_var [B][nvar], q [B][n], l [B][m], u [B][m] per QP.  The
 * solve then reads the shared values from L2 instead of B copies from HBM; results are those of
 * impc_batch_set_values on the expanded arrays. */
int impc_batch_set_values_shared(impc_batch b, const double *Px, const double *Ax, int64_t nvar,
                                 const int64_t *var_pos, const double *Ax_var, const double *q, const double *l,
                                 const double *u);

/* osqp_warm_start(x, y) for every QP (host, QP-major; y may be NULL = zero duals, the solveTraj
 * warm start: then no duals are uploaded or read by the solve).  As in OSQP
 * it turns the warm_start setting on.  On a set-up workspace (generic kernel after a solve,
 * structured kernel with a persistent workspace) it replaces the iterates and keeps scaling, rho
 * and factor.  Pass x = NULL to clear a pending warm start (the next setup cold-starts). */
int impc_batch_warm_start(impc_batch b, const double *x, const double *y);
/* The same from DEVICE arrays (QP-major x [B][n], y [B][m] or NULL = zero duals): the copies are
 * queued on the context stream after every launch already issued, no host synchronisation (the
 * closed replan loop hands each candidate the previous winner this way). */
int impc_batch_warm_start_device(impc_batch b, const double *x, const double *y);
/* Solve only the first `count` QPs of the batch (1 <= count <= B; B after create): a batch
 * created once at a capacity serves smaller per-call sets (a replan's single-solve instances, the
 * OsqpEigen front end's workspace pool).  Rows >= count are not read or written by the solves;
 * their results keep whatever they held.  Changing the count discards a persistent workspace. */
int impc_batch_set_active(impc_batch b, int64_t count);

/* osqp_setup's numeric part on the device: Ruiz scaling, rho vector, KKT assembly and
 * factorisation, then the pending warm start.  Asynchronous on `stream` (NULL = ctx stream). */
int impc_batch_setup(impc_batch b, void *stream);

/* osqp_solve on the device for every QP (ADMM, termination, adaptive rho with in-kernel
 * refactorisation, unscaling).  Runs impc_batch_setup first if values changed since the last
 * setup.  Asynchronous on `stream`. */
int impc_batch_solve(impc_batch b, void *stream);

/* One persistent launch for several structured batches (e.g. the pattern buckets of a replan:
 * candidates with K and K+1 obstacles): a single work queue over all their QPs, so the slow QPs
 * at the end of one batch overlap the others' work.  The batches must share the context and the
 * structured kernel's team shape (impc_batch_stats.kernel == IMPC_KERNEL_STRUCTURED; n <= 256, i.e.
 * N <= 20, or 256 < n <= 768).  Results land in each batch as after impc_batch_solve.  With profiling
 * on for bs[0], its impc_batch_get_timings reports the grouped kernel. */
int impc_batch_solve_group(impc_batch *bs, int count, void *stream);

/* Synchronise and copy results to host (any pointer may be NULL): x [B][n], y [B][m], info [B]. */
int impc_batch_get(impc_batch b, double *x, double *y, impc_info *info);

/* Device pointers of the QP-major result arrays, valid until the next solve / destroy. */
int impc_batch_device_results(impc_batch b, double **x, double **y, impc_info **info);

/* Persistent-workspace updates (osqp_update_lin_cost / osqp_update_bounds, osqp.h:114-134):
 * rescale with the existing scaling, keep the factorisation unless a constraint changes type
 * (equality / inequality / loose), and keep the iterates as the next warm start. */
int impc_batch_update_lin_cost(impc_batch b, const double *q);
int impc_batch_update_bounds(impc_batch b, const double *l, const double *u);
/* The same from DEVICE arrays (q [B][n]; l, u [B][m]), stream-ordered on the context stream after
 * every launch already issued, no host synchronisation and no l <= u check (the caller's; a
 * receding-horizon loop builds the next step's values on the device). */
int impc_batch_update_lin_cost_device(impc_batch b, const double *q);
int impc_batch_update_bounds_device(impc_batch b, const double *l, const double *u);
/* osqp_update_P / osqp_update_A / osqp_update_P_A (osqp.h:137-156, OsqpEigen Solver.tpp:15-212) on
 * a persistent structured workspace: new values of P and / or A (host, QP-major [B][nnzP] /
 * [B][nnzA], same patterns; NULL = unchanged).  As OSQP 0.6.2 does (unscale_data, the new values,
 * scale_data, update_matrices), the next solve runs the Ruiz scaling afresh on the new data,
 * refactors with the kept rho and continues from the kept SCALED iterates (x, z, y are not
 * rescaled).  The generic kernel has no in-place form (IMPC_UNSUPPORTED: set the values again and
 * warm start). */
int impc_batch_update_matrices(impc_batch b, const double *Px, const double *Ax);
/* The same from DEVICE arrays, stream-ordered on the context stream (a receding loop that
 * re-linearises its obstacle rows on the device every step). */
int impc_batch_update_matrices_device(impc_batch b, const double *Px, const double *Ax);

/* Kernel selection.  AUTO picks the one-QP-per-wavefront structured kernel when the pattern is
 * the stage-structured mpcPlanner QP and fits its register layout, else the
 * generic one-QP-per-lane kernel.  The persistent update calls work on both (structured: after
 * impc_batch_set_persistent). */
#define IMPC_KERNEL_AUTO 0
#define IMPC_KERNEL_GENERIC 1
#define IMPC_KERNEL_STRUCTURED 2
int impc_batch_set_kernel(impc_batch b, int kernel);

/* Device memory utilities for callers without their own HIP plumbing (FFI bindings, tests):
 * allocation on the context's device and synchronous copies. */
int impc_device_alloc(impc_ctx ctx, int64_t bytes, void **out);
int impc_device_free(impc_ctx ctx, void *ptr);
int impc_copy_to_device(impc_ctx ctx, void *dst, const void *src, int64_t bytes);
int impc_copy_to_host(impc_ctx ctx, void *dst, const void *src, int64_t bytes);

/* Pipelined transfers: host <-> device copies of one batch overlapped with the solve of another.
 * Pinned host memory (hipHostMalloc) for the asynchronous copies, extra streams and the ordering
 * between them (waiter waits for the work queued on signaler so far), stream synchronisation. */
int impc_host_alloc(impc_ctx ctx, int64_t bytes, void **out);
int impc_host_free(impc_ctx ctx, void *ptr);
int impc_stream_create(impc_ctx ctx, void **stream);
int impc_stream_destroy(impc_ctx ctx, void *stream);
int impc_stream_wait(impc_ctx ctx, void *waiter, void *signaler);
int impc_stream_synchronize(impc_ctx ctx, void *stream);
/* The per-QP values of a shared-structure batch (after impc_batch_set_values_shared, which fixes
 * P, A and var_pos): Ax_var [B][nvar], q [B][n], l [B][m], u [B][m] and, when x_ws is not NULL,
 * the warm start x [B][n] with zero duals -- queued on `stream` (NULL = the context's) with no
 * host synchronisation and no validation (l <= u is the caller's).  The host arrays must stay
 * valid until the stream has passed the copies (pinned memory overlaps them with solves); the
 * caller orders the stream against solves of this batch (impc_stream_wait). */
int impc_batch_set_values_async(impc_batch b, const double *Ax_var, const double *q, const double *l, const double *u,
                                const double *x_ws, void *stream);
/* Results (as impc_batch_get; any pointer may be NULL) copied on `stream`, not waited for. */
int impc_batch_get_async(impc_batch b, double *x, double *y, impc_info *info, void *stream);

/* Problem / analysis facts (for tests and roofline accounting). */
typedef struct {
    int64_t n, m, nnzP, nnzA, batch, batch_stride;
    int64_t nnzL;        /* envelope entries of the factor of P + sigma I + A' R A */
    int64_t nnzLcol;     /* column-envelope entries */
    int64_t n_terms;     /* A' R A assembly terms */
    int64_t bandwidth;   /* max row length of the envelope */
    int64_t device_bytes;
    int64_t kernel;          /* IMPC_KERNEL_GENERIC or IMPC_KERNEL_STRUCTURED for the next solve */
    int64_t structured_ok;   /* 1 if the pattern qualifies for the structured kernel */
    /* structured team shape (0 when structured_ok is 0): lanes per QP (64: one QP per wavefront,
     * 256: one QP per 4-wavefront workgroup), variable and general-row slots per lane */
    int64_t team_lanes, var_slots, row_slots;
} impc_batch_stats;
int impc_batch_get_stats(impc_batch b, impc_batch_stats *out);

/* Kernel timing with HIP events recorded on the solve stream around k_setup, k_solve and the
 * output transposes (profiling on: events are recorded by every subsequent setup/solve). */
int impc_batch_set_profiling(impc_batch b, int on);
/* Durations (ms) of the last profiled setup / solve-kernel / output-transpose launches.  For the
 * structured kernel solve_ms spans the whole solve call on its stream: with the longest-first queue
 * (impc_batch_set_queue_order) that includes the queue-key kernel and the radix sort (~0.7 ms at
 * 65,536 QPs) before the solver kernel; the per-QP latencies (impc_batch_get_qp_latency) do not. */
int impc_batch_get_timings(impc_batch b, double *setup_ms, double *solve_ms, double *output_ms);

/* Persistent workspace (structured kernel; OSQP's workspace kept between osqp_solve calls, as a
 * persistent OsqpEigen::Solver does -- polyTrajSolver.cpp:183-237).  With it on, each solve keeps
 * the QPs' scaling, rho and scaled iterates on the device; impc_batch_update_lin_cost /
 * impc_batch_update_bounds (osqp_update_lin_cost / osqp_update_bounds semantics) then apply to
 * the next solve, which continues from the stored iterates (an explicit impc_batch_warm_start is
 * applied once instead).  New values (impc_batch_set_values*) start over with a full setup.
 * Costs 8 (24 + 3 n + 2 m_general) bytes per QP of device memory and that much HBM traffic per
 * solve.  Off by default. */
int impc_batch_set_persistent(impc_batch b, int on);
/* Debug read-back of the persistent workspaces after a solve (no reference counterpart: OSQP's
 * OSQPWorkspace fields work->x, work->z, work->y and settings->rho, types.h:182-289): per QP the
 * rho and the SCALED iterates in OSQP's variable / row order, host arrays rho [B], x [B][n],
 * z [B][m], y [B][m] (any may be NULL).  After a solve that ended without a solution the iterates
 * are zero (store_solution's cold_start).  Synchronises the context.  The parity tests load them
 * into the oracle's workspace before each step of a chained loop. */
int impc_batch_get_persistent(impc_batch b, double *rho, double *x, double *z, double *y);

/* Per-QP solve latency (ms) of the last profiled structured-kernel solve: from the moment a
 * workgroup takes the QP off the work queue (the tick its time limit counts from) to its results
 * being written, on the device's constant-rate clock (rate: impc_ctx_clock_rate), for each of the
 * B QPs.  Profiling must be on before the solve. */
int impc_batch_get_qp_latency(impc_batch b, double *ms);

/* Per-QP OSQP time limits (seconds, host array [B]; 0 = none), overriding the settings'
 * time_limit for the following solves; NULL returns to the settings' value.  The reference sets
 * each solveTraj call's own limit (mpcPlanner.cpp:442-444: setTimeLimit(timeLimit) only when
 * not firstTime_, timeLimit = max(solverTimeLimit_ - t, solverTimeLimit_) at :613-615), so one
 * batch of candidates from several planners carries one limit per QP. */
int impc_batch_set_time_limits(impc_batch b, const double *time_limit);

/* Work-queue order of the structured kernel's persistent launches (no reference counterpart: the
 * reference solves each candidate in its own loop iteration, mpcPlanner.cpp:609-628).
 *   IMPC_QUEUE_FIFO (default): QPs are dequeued in batch order (a grouped launch: batch by batch).
 *   IMPC_QUEUE_LONGEST_FIRST: before each launch the device estimates every QP's difficulty from its
 *     own inputs, key = ||A x_ws - proj_[l,u](A x_ws)||_inf + q_weight * ||q||_inf (the warm start's
 *     constraint violation plus a scale of the linear cost), and the launch dequeues its QPs in
 *     descending key order across all its batches, so the QPs that run longest start first and the
 *     launch tail shrinks (a launch is ordered when any of its batches asks for it; each batch's
 *     keys use its own q_weight).
 * The order changes no result: each QP is solved alone from its own inputs.  The generic kernel
 * (one QP per lane, no queue) ignores it. */
#define IMPC_QUEUE_FIFO 0
#define IMPC_QUEUE_LONGEST_FIRST 1
int impc_batch_set_queue_order(impc_batch b, int mode, double q_weight);

/* The device clock the time limits and latencies are measured on: its rate in Hz, from
 * hipDeviceAttributeWallClockRate (queried once per context). */
int impc_ctx_clock_rate(impc_ctx ctx, double *hz);
/* Clock self-check (diagnostics, tests): one kernel spins on the device clock until `seconds`
 * have passed at the reported rate; *event_seconds = the same launch timed by HIP events on the
 * context stream.  The two agree when the rate is right. */
int impc_ctx_clock_check(impc_ctx ctx, double seconds, double *event_seconds);

/* Factor-order permutation chosen by the symbolic analysis (perm[k] = variable at position k). */
int impc_batch_get_perm(impc_batch b, int64_t *perm);

#ifdef __cplusplus
}
#endif
#endif
