// lib_internal.hpp -- library-internal hooks of impc_qp.hip for the other HIP translation units
// of libimpc_qp.so (replan_run.hip).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/impc_mpc.h"
#include "../../include/impc_qp.h"

namespace impc_lib {
// solveTraj's success for one solved QP (mpcPlanner.cpp:475-478, :513-518): initSolver (osqp_setup)
// succeeded and solveProblem returned NoError.  osqp_solve's exitflag -- what solveProblem returns
// -- is 0 for every final status, infeasible, max-iter, time limit and a NON_CVX from the residual
// test included (x = OSQP_NAN then), and 1 only when an adaptive-rho refactorisation fails, which
// leaves the status UNSOLVED; a failed setup is reported as NON_CVX with setup_exitflag set.
__host__ __device__ inline bool solve_traj_ok(const impc_info &inf) {
    return inf.setup_exitflag == 0 && inf.status_val != IMPC_UNSOLVED;
}
// record the message of the last error (impc_last_error) and return `code`
int set_error(int code, const std::string &msg);
int num_cu(impc_ctx ctx);
int device(impc_ctx ctx);
hipStream_t stream(impc_ctx ctx);
// the context stream waits for every launch the context noted on caller streams
int order_after_all(impc_ctx ctx);

// A batch's device input arrays (QP-major, capacity B rows), for producers that write them in
// place (the replan's assembly and warm-start gathers): begin orders the context stream after
// every launch that may still read them; end marks the batch's values (and a primal warm start
// with zero duals when warm_x) as set, as impc_batch_set_values_device + _warm_start_device do.
struct BatchInputs {
    double *Px, *q, *Ax, *l, *u, *xws;
    int64_t n, m, nnzP, nnzA, B;
};
int batch_inputs_begin(impc_batch b, BatchInputs *out);
int batch_inputs_end(impc_batch b, bool warm_x);
// the same arrays without ordering (read-only inspection after the caller synchronised)
int batch_inputs_view(impc_batch b, BatchInputs *out);
// The batch's active QP count from device memory (structured kernel): every later solve takes the
// first *d_count of its B QPs, the count read by the kernels themselves -- no host round trip
// between the producer that decides it and the solve.  NULL returns to B (impc_batch_set_active).
int batch_set_active_device(impc_batch b, const int64_t *d_count);
// The batch's per-QP time-limit array [B] on the device (allocated zero = no limit on first use),
// switched on for the following solves; producers write it in place.
int batch_tlim_device(impc_batch b, double **out);
// seconds per tick of the device clock the time limits run on (hipDeviceAttributeWallClockRate)
double tick_s(impc_ctx ctx);
// The device builder over replan rows (mpc_build.hpp Args: dcount / row_inst / osrc / held arrays;
// static obstacles per instance, [*][builder's S][3] / [*][S], unread when the builder has none),
// writing the QP values into a batch's input arrays; asynchronous on `st`.
int build_rows(impc_mpc_builder bd, int64_t cap, const int64_t *dcount, const int32_t *row_inst, const int64_t *osrc,
               const double *pos, const double *vel, const double *xref, const double *lin, const double *pred_pos,
               const double *pred_size, const double *held_pos, const double *held_size, const double *st_centroid,
               const double *st_size, const double *st_yaw, const BatchInputs &out, hipStream_t st);
}  // namespace impc_lib
