// queue.hpp -- work-queue order of the structured kernels' persistent launches
// (impc_batch_set_queue_order, include/impc_qp.h).
//
// A persistent launch keeps 2 QPs per CU in flight and pulls the next QP index with one atomic.
// Dequeued in batch order, the few QPs that run to thousands of ADMM iterations (OSQP's
// max_iter = 4000 cap) start wherever they happen to sit and, when they sit near the end, finish
// long after the rest: the launch tail.  With a shard of 8,192 QPs per GPU (config 3 split eight
// ways, mpcPlanner.cpp:609-628 is the per-instance loop it replaces) that tail is a large part of
// the launch.  IMPC_QUEUE_LONGEST_FIRST estimates every QP's difficulty on the device from its
// own inputs and dequeues the launch's QPs in descending order of that estimate (the classic
// longest-processing-time-first list schedule):
//
//   key = || A x_ws - proj_[l,u](A x_ws) ||_inf  +  q_weight * || q ||_inf
//
// The first term is how far the warm start (solveTraj's previous plan) is from feasible for this
// QP's constraints -- a hypothesis whose obstacle crosses the previous plan needs a long re-plan;
// the second is a scale of the linear cost (for the MPC QP, q = -Q xRef: how far the reference
// runs ahead of the state).  The order changes no QP's arithmetic: every QP is solved by one
// workgroup from its own inputs, so results are bitwise those of the FIFO order.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace impc {

struct QueueKeyArgs {
    int64_t B, n, m, first;
    const int32_t *row_ptr;   // CSR of A's pattern [m + 1]
    const int32_t *row_col;   // [nnzA] column of each CSR entry
    const int32_t *row_ent;   // [nnzA] CSC entry index of each CSR entry
    const double *Ax;         // QP-major [B][nnzA], or the shared copy [nnzA]
    int32_t shared;           // shared-structure values: entry p is Ax_var[b][vmap[p]] when vmap[p] >= 0
    int64_t nvar;
    const int32_t *vmap;
    const double *Ax_var;
    const double *q, *l, *u, *xws;  // QP-major
    int32_t has_ws;
    double q_weight;
    const int64_t *dcount;  // active rows in device memory (rows >= *dcount: key -inf, last), or null
    int32_t fifo;           // key = -(queue index): the FIFO order as a permutation (device counts)
};

// One 256-thread workgroup per QP (grid-stride): rows of A x_ws against [l, u], |q|, a block max.
// Writes key[first + b] and the QP's launch-wide queue index first + b.
__global__ __launch_bounds__(256) void k_queue_key(QueueKeyArgs a, double *key, uint32_t *idx) {
    __shared__ double red[8];
    const int64_t nact = a.dcount ? *a.dcount : a.B;
    for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
        if (b >= nact || a.fifo) {  // (uniform per workgroup)
            if (threadIdx.x == 0) {
                key[a.first + b] = b >= nact ? -INFINITY : -(double)(a.first + b);
                idx[a.first + b] = (uint32_t)(a.first + b);
            }
            continue;
        }
        double v = 0.0;
        for (int64_t r = threadIdx.x; r < a.m; r += blockDim.x) {
            double ax = 0.0;
            if (a.has_ws) {
                for (int32_t k = a.row_ptr[r]; k < a.row_ptr[r + 1]; k++) {
                    const int32_t p = a.row_ent[k];
                    double av;
                    if (a.shared) {
                        const int32_t vm = a.vmap[p];
                        av = vm >= 0 ? a.Ax_var[b * a.nvar + vm] : a.Ax[p];
                    } else {
                        av = a.Ax[b * (int64_t)a.row_ptr[a.m] + p];
                    }
                    ax += av * a.xws[b * a.n + a.row_col[k]];
                }
            }
            // infinite bounds give -inf here, never a violation
            v = fmax(v, fmax(a.l[b * a.m + r] - ax, ax - a.u[b * a.m + r]));
        }
        double qm = 0.0;
        for (int64_t j = threadIdx.x; j < a.n; j += blockDim.x) qm = fmax(qm, fabs(a.q[b * a.n + j]));
        for (int o = 32; o >= 1; o >>= 1) {
            v = fmax(v, __shfl_xor(v, o));
            qm = fmax(qm, __shfl_xor(qm, o));
        }
        if ((threadIdx.x & 63) == 0) {
            red[threadIdx.x >> 6] = v;
            red[4 + (threadIdx.x >> 6)] = qm;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double vv = red[0], qq = red[4];
            for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
                vv = fmax(vv, red[w]);
                qq = fmax(qq, red[4 + w]);
            }
            const double k = vv + a.q_weight * qq;
            key[a.first + b] = k == k ? k : 0.0;  // NaN inputs: no priority
            idx[a.first + b] = (uint32_t)(a.first + b);
        }
        __syncthreads();
    }
}

}  // namespace impc
