// lib_internal.hpp -- library-internal hooks of impc_qp.hip for the other HIP translation units
// of libimpc_qp.so (replan_run.hip).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/impc_qp.h"

namespace impc_lib {
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
}  // namespace impc_lib
