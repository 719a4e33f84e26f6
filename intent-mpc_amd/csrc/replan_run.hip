// replan_run.hip -- the whole batched makePlanWithPred behind one C-ABI call (include/impc_replan.h,
// impc_replan_*), part of libimpc_qp.so.
//
// Reference: trajectory_planner/include/trajectory_planner/mpcPlanner.cpp:571-661 (makePlanWithPred),
// called per planning instance by mpcNavigation.cpp:316-322.  Per instance it takes one of three
// branches (:593-606) -- the intent fan-out with six candidate solves and a selection, or ONE
// solveTraj (first plan, or no predictions) -- and commits the plan it gets into the planner state.
// Here every instance of a batch goes through one call:
//
//   k_branch_table       the branch of every instance and the compacted instance lists of each
//                        branch (ascending), one workgroup; the three counts are the only bytes
//                        the host reads back (they size the shapes' QP sets)
//   gathers / repeats    the fan-out instances' inputs compacted (impc_gather_rows_device), each
//                        candidate's x0 / xRef / linearisation point repeated per candidate
//                        (impc_repeat_rows_device), the warm starts gathered from the plan state
//                        straight into the batches' input arrays
//   fan-out              impc_intent_fanout_device (findClosestObstacle + getIntentComb)
//   assembly             impc_mpc_build_values_device per shape, written in place into the batches
//   solve                ONE impc_batch_solve_group over every shape that has QPs
//   validity             k_cand_valid: solveTraj's success from the candidates' impc_info
//   selection            impc_fanout_candidates_device + impc_select_best_device
//   commit               impc_replan_commit_device (fan-out winners, single solves), k_scatter
//                        (per-instance outputs)
//
// No x, y or QP value leaves the device.  The host work per call is the launches, one read of
// the branch counts and the issue cut-off check (:613), which needs the assembly to have finished.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/impc_fanout.h"
#include "../../include/impc_mpc.h"
#include "../../include/impc_qp.h"
#include "../../include/impc_replan.h"
#include "../../include/impc_select.h"
#include "lib_internal.hpp"

#define RP_HIP(expr)                                                                                        \
    do {                                                                                                    \
        hipError_t e_ = (expr);                                                                             \
        if (e_ != hipSuccess)                                                                               \
            return impc_lib::set_error(IMPC_DEVICE_ERROR, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define RP_TRY(expr)         \
    do {                     \
        int rc_ = (expr);    \
        if (rc_) return rc_; \
    } while (0)

namespace impc_rp {

constexpr int kTableLanes = 1024;

// The branch of every instance (:593-606) and the instance lists of each branch in ascending
// order, by one workgroup: lane t owns a contiguous range of instances, an exclusive scan of the
// per-lane counts gives each lane its output offsets.  Also resets the per-instance outputs of
// the run (best_cand, ob_idx, cand_type, cand_slot = -1).
//   ws_first[r]: the warm-start row of the r-th SINGLE_FIRST instance: row I (zeros) on a first
//   plan (solveTraj :487-508, firstTime_), else the instance's plan.
__global__ __launch_bounds__(kTableLanes) void k_branch_table(int64_t I, const int8_t *__restrict__ first_time,
                                                              const int8_t *__restrict__ has_pred,
                                                              const int32_t *__restrict__ cur_count, int cur_all,
                                                              int8_t *__restrict__ branch, int64_t *__restrict__ inst_f,
                                                              int64_t *__restrict__ inst_0, int64_t *__restrict__ ws_0,
                                                              int64_t *__restrict__ inst_1, int64_t *__restrict__ counts,
                                                              int32_t *__restrict__ best, int32_t *__restrict__ ob,
                                                              int32_t *__restrict__ ctype, int32_t *__restrict__ cslot) {
    __shared__ int64_t scan[3][kTableLanes];
    const int t = threadIdx.x;
    const int64_t per = (I + kTableLanes - 1) / kTableLanes;
    const int64_t i0 = std::min<int64_t>(I, t * per), i1 = std::min<int64_t>(I, i0 + per);
    auto decide = [&](int64_t i) -> int {
        const bool ft = first_time[i] != 0;
        const bool hp = has_pred ? has_pred[i] != 0 : true;
        const bool cur = cur_count ? cur_count[i] > 0 : cur_all != 0;
        return (!ft && hp) ? IMPC_REPLAN_FANOUT : (!ft && cur) ? IMPC_REPLAN_SINGLE_CURRENT : IMPC_REPLAN_SINGLE_FIRST;
    };
    int64_t c[3] = {0, 0, 0};
    for (int64_t i = i0; i < i1; i++) c[decide(i)]++;
    for (int k = 0; k < 3; k++) scan[k][t] = c[k];
    __syncthreads();
    for (int off = 1; off < kTableLanes; off <<= 1) {  // inclusive Hillis-Steele scan
        int64_t v[3];
        for (int k = 0; k < 3; k++) v[k] = t >= off ? scan[k][t - off] : 0;
        __syncthreads();
        for (int k = 0; k < 3; k++) scan[k][t] += v[k];
        __syncthreads();
    }
    int64_t o[3];
    for (int k = 0; k < 3; k++) o[k] = scan[k][t] - c[k];
    for (int64_t i = i0; i < i1; i++) {
        const int br = decide(i);
        branch[i] = (int8_t)br;
        if (br == IMPC_REPLAN_FANOUT) {
            inst_f[o[0]++] = i;
        } else if (br == IMPC_REPLAN_SINGLE_FIRST) {
            ws_0[o[1]] = first_time[i] != 0 ? I : i;
            inst_0[o[1]++] = i;
        } else {
            inst_1[o[2]++] = i;
        }
        best[i] = -1;
        ob[i] = -1;
        for (int k = 0; k < 6; k++) ctype[6 * i + k] = cslot[6 * i + k] = -1;
    }
    if (t == kTableLanes - 1)
        for (int k = 0; k < 3; k++) counts[k] = scan[k][t];
}

// updateDynamicObstacles (:316-341): each current obstacle's position / size held over the T
// prediction steps of the single-solve QP: out[r][k][s][:] = src[inst[r]][k][:]
__global__ void k_hold(const double *__restrict__ src, const int64_t *__restrict__ inst, int64_t count, int32_t K,
                       int32_t T, double *__restrict__ out) {
    const int64_t total = count * K * T * 3;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = e % 3, s = e / 3, k = (s / T) % K, r = s / ((int64_t)T * K);
        out[e] = src[(inst[r] * K + k) * 3 + c];
    }
}

// candidate c of fan-out instance j is valid when it was issued and solveTraj succeeded
// (solveProblem NoError = every OSQP status but NON_CVX, :513-518); slot s < 4 is row 4 j + s of
// the single-intent batch, else row 2 j + s - 4 of the two-intent batch (fanout.hpp)
__global__ void k_cand_valid(int64_t nf, const int32_t *__restrict__ cand_slot, const impc_info *__restrict__ info_s,
                             const impc_info *__restrict__ info_p, int issued, int8_t *__restrict__ valid) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nf * 6; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = e / 6;
        const int32_t s = cand_slot[e];
        const impc_info &inf = s < 4 ? info_s[4 * j + s] : info_p[2 * j + (s - 4)];
        valid[e] = (issued && inf.status_val != IMPC_NON_CVX) ? 1 : 0;
    }
}

// the fan-out instances' per-instance outputs, from their compacted rows to instance order
__global__ void k_scatter(int64_t nf, const int64_t *__restrict__ inst_f, const int32_t *__restrict__ best_f,
                          const int32_t *__restrict__ ob_f, const int32_t *__restrict__ ctype_f,
                          const int32_t *__restrict__ cslot_f, int32_t *__restrict__ best, int32_t *__restrict__ ob,
                          int32_t *__restrict__ ctype, int32_t *__restrict__ cslot) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nf; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = inst_f[j];
        best[i] = best_f[j];
        ob[i] = ob_f[j];
        for (int k = 0; k < 6; k++) {
            ctype[6 * i + k] = ctype_f[6 * j + k];
            cslot[6 * i + k] = cslot_f[6 * j + k];
        }
    }
}

// mpcPlanner::getPos / getVel (mpcPlanner.cpp:1257-1290) of every instance with a plan
__global__ void k_advance(int64_t I, int32_t N, int64_t n, double ts, double t, const int8_t *__restrict__ valid,
                          const double *__restrict__ plan_x, double *__restrict__ pos, double *__restrict__ vel) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < I; i += (int64_t)gridDim.x * blockDim.x) {
        if (!valid[i]) continue;
        int idx = (int)floor(t / ts);
        const double dt = t - idx * ts;
        idx = max(0, min(idx, N - 1));
        const int nxt = min(idx + 1, N - 1);
        const double *s = plan_x + i * n + 8 * idx, *e = plan_x + i * n + 8 * nxt;
        for (int c = 0; c < 3; c++) {
            pos[3 * i + c] = s[c] + (e[c] - s[c]) / ts * dt;
            vel[3 * i + c] = s[3 + c] + (e[3 + c] - s[3 + c]) / ts * dt;
        }
    }
}

// device allocations of one replan object, released together
struct Arena {
    std::vector<void *> ptrs;
    int alloc(size_t bytes, void **out) {
        RP_HIP(hipMalloc(out, std::max<size_t>(bytes, 8)));
        ptrs.push_back(*out);
        return IMPC_OK;
    }
    template <class T>
    int get(size_t count, T **out) {
        return alloc(count * sizeof(T), (void **)out);
    }
    void release() {
        for (void *p : ptrs) (void)hipFree(p);
        ptrs.clear();
    }
};

// one QP shape of the replan: its solver batch, its on-device builder, and the per-QP inputs of
// the assembly (cap rows)
struct Shape {
    int32_t K = 0, L = 0, rep = 1;
    int64_t cap = 0, count = 0, ninst = 0;
    impc_qp_dims dm{};
    impc_batch batch = nullptr;
    impc_mpc_builder bld = nullptr;
    double *pos = nullptr, *vel = nullptr, *xref = nullptr, *lin = nullptr;
    double *dpos = nullptr, *dsize = nullptr;  // the current-obstacle shape's held obstacles
    const int64_t *inst = nullptr;            // instances of the last run (device)
    bool tlim_known = false;
    double tlim = 0.0;                        // per-QP time limit uploaded last (< 0: none)
};

}  // namespace impc_rp

using namespace impc_rp;

struct impc_replan_s {
    impc_ctx ctx = nullptr;
    impc_replan_config cfg{};
    int64_t I = 0, n = 0;
    int32_t N = 0, K = 0, L = 0;
    Arena mem;
    // planner state
    double *plan_x = nullptr, *plan_states = nullptr;
    int32_t *prev_count = nullptr;
    int8_t *first_time = nullptr, *valid = nullptr, *zeros8 = nullptr;
    // branch table
    int8_t *branch = nullptr;
    int64_t *inst_f = nullptr, *inst_0 = nullptr, *ws_0 = nullptr, *inst_1 = nullptr, *d_counts = nullptr;
    int64_t *h_counts = nullptr;  // pinned
    // per-instance outputs
    int32_t *best = nullptr, *ob = nullptr, *ctype = nullptr, *cslot = nullptr;
    // fan-out: compacted inputs and outputs
    double *f_pos = nullptr, *f_vel = nullptr, *f_xref = nullptr, *f_lin = nullptr, *f_dcur = nullptr;
    double *f_ppos = nullptr, *f_psize = nullptr, *f_prob = nullptr, *f_ws = nullptr;
    int32_t *f_pc = nullptr;
    int32_t *f_ob = nullptr, *f_ctype = nullptr, *f_cslot = nullptr;
    double *f_cprob = nullptr, *s_pos = nullptr, *s_size = nullptr, *p_pos = nullptr, *p_size = nullptr;
    // selection
    const double **x_cand = nullptr;
    int32_t *dyn_count = nullptr, *best_f = nullptr, *best_pos = nullptr;
    double *dyn_pos = nullptr, *dyn_size = nullptr, *scores = nullptr, *weighted = nullptr;
    int8_t *cvalid = nullptr;
    Shape sh[4];  // 0 single-intent, 1 two-intent, 2 single solve (no obstacles), 3 current obstacles
    impc_replan_stats stats{};
};

namespace {

int fail(int code, const char *msg) { return impc_lib::set_error(code, msg); }

int make_shape(impc_replan rp, Shape &s, int32_t K, int32_t L, int32_t rep, int64_t cap, bool held) {
    s.K = K, s.L = L, s.rep = rep, s.cap = cap;
    RP_TRY(impc_mpc_dims(&rp->cfg.mpc, 0, K, &s.dm));
    std::vector<int64_t> Pp(s.dm.n + 1), Pi(std::max<int64_t>(s.dm.nnzP, 1)), Ap(s.dm.n + 1), Ai(s.dm.nnzA);
    RP_TRY(impc_mpc_build_pattern(&rp->cfg.mpc, 0, K, Pp.data(), Pi.data(), Ap.data(), Ai.data()));
    RP_TRY(impc_batch_create(rp->ctx, s.dm.n, s.dm.m, Pp.data(), Pi.data(), Ap.data(), Ai.data(), cap, &s.batch));
    RP_TRY(impc_batch_set_settings(s.batch, &rp->cfg.settings));
    if (rp->cfg.queue_order == IMPC_QUEUE_LONGEST_FIRST) {
        // impc.scenarios.queue_weight: ||q||_inf / (position weight (N - 1)) weighed 1:10
        const double qw = 1.0 / (10.0 * (rp->N - 1) * rp->cfg.mpc.position_weight);
        RP_TRY(impc_batch_set_queue_order(s.batch, IMPC_QUEUE_LONGEST_FIRST, qw));
    }
    RP_TRY(impc_mpc_builder_create(rp->ctx, &rp->cfg.mpc, 0, K, L, &s.bld));
    const int64_t N = rp->N;
    // x0, reference and linearisation point of every QP: per-candidate copies (rep > 1) or the
    // single solves' gathered rows
    RP_TRY(rp->mem.get((size_t)(cap * 3), &s.pos));
    RP_TRY(rp->mem.get((size_t)(cap * 3), &s.vel));
    RP_TRY(rp->mem.get((size_t)(cap * N * 8), &s.xref));
    RP_TRY(rp->mem.get((size_t)(cap * N * 8), &s.lin));
    if (held) {
        RP_TRY(rp->mem.get((size_t)(cap * K * L * 3), &s.dpos));
        RP_TRY(rp->mem.get((size_t)(cap * K * L * 3), &s.dsize));
    }
    return IMPC_OK;
}

void free_shape(Shape &s) {
    if (s.batch) (void)impc_batch_destroy(s.batch);
    if (s.bld) (void)impc_mpc_builder_destroy(s.bld);
    s.batch = nullptr;
    s.bld = nullptr;
}

// per-QP time limits of a shape's batch, uploaded only when they change (the upload waits for the
// launches in flight): `v` for every QP, or none (v == 0 with no limit in the settings)
int set_limit(impc_replan rp, Shape &s, double v) {
    if (s.tlim_known && s.tlim == v) return IMPC_OK;
    if (v == 0.0 && rp->cfg.settings.time_limit == 0.0) {
        RP_TRY(impc_batch_set_time_limits(s.batch, nullptr));
    } else {
        std::vector<double> lim((size_t)s.cap, v);
        RP_TRY(impc_batch_set_time_limits(s.batch, lim.data()));
    }
    s.tlim_known = true;
    s.tlim = v;
    return IMPC_OK;
}

// The assembly of one shape's `ninst` instances into its batch: x0, reference and linearisation
// point per QP (already in s.pos / vel / xref / lin), the obstacle sets (dyn_pos / dyn_size), the
// warm start gathered from the plan state by ws_idx and repeated per candidate (ws_tmp: [ninst][n]
// scratch when rep > 1).
int assemble(impc_replan rp, Shape &s, int64_t ninst, const double *lin, const double *dyn_pos, const double *dyn_size,
             const int64_t *ws_idx, double *ws_tmp) {
    s.ninst = ninst;
    s.count = ninst * s.rep;
    if (!s.count) return IMPC_OK;
    impc_ctx ctx = rp->ctx;
    impc_lib::BatchInputs in{};
    RP_TRY(impc_lib::batch_inputs_begin(s.batch, &in));
    if (in.n != rp->n) return fail(IMPC_INVALID_ARGUMENT, "replan shape: n != 13 N - 5");
    const int64_t wbytes = 8 * rp->n;
    if (s.rep == 1) {
        RP_TRY(impc_gather_rows_device(ctx, rp->plan_x, wbytes, ws_idx, ninst, in.xws, nullptr));
    } else {
        RP_TRY(impc_gather_rows_device(ctx, rp->plan_x, wbytes, ws_idx, ninst, ws_tmp, nullptr));
        RP_TRY(impc_repeat_rows_device(ctx, ws_tmp, ninst, wbytes, s.rep, in.xws, nullptr));
    }
    RP_TRY(impc_mpc_build_values_device(s.bld, s.count, s.pos, s.vel, s.xref, lin, nullptr, nullptr, nullptr, dyn_pos,
                                        dyn_size, in.Px, in.q, in.Ax, in.l, in.u, nullptr));
    RP_TRY(impc_lib::batch_inputs_end(s.batch, true));
    return impc_batch_set_active(s.batch, s.count);
}

unsigned grid_for(impc_replan rp, int64_t work) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, (int64_t)impc_lib::num_cu(rp->ctx) * 8));
}

}  // namespace

extern "C" {

int impc_replan_create(impc_ctx ctx, const impc_replan_config *cfg, impc_replan *out) {
    if (!ctx || !cfg || !out) return fail(IMPC_INVALID_ARGUMENT, "replan: null context, config or output");
    *out = nullptr;
    const int64_t I = cfg->instances;
    const int32_t N = cfg->mpc.horizon, K = cfg->num_obstacles, L = cfg->pred_len;
    if (I < 1 || I > ((int64_t)1 << 26) || N < 2 || K < 1 || L < 1)
        return fail(IMPC_INVALID_ARGUMENT, "replan: instances >= 1, horizon >= 2, num_obstacles >= 1, pred_len >= 1");
    if (cfg->mpc.num_half_space != 0)
        return fail(IMPC_UNSUPPORTED, "replan: the live planner path has no FOV half-spaces (num_half_space = 0)");
    if (cfg->queue_order != IMPC_QUEUE_FIFO && cfg->queue_order != IMPC_QUEUE_LONGEST_FIRST)
        return fail(IMPC_INVALID_ARGUMENT, "replan: unknown queue order");
    RP_HIP(hipSetDevice(impc_lib::device(ctx)));
    std::unique_ptr<impc_replan_s> rp(new impc_replan_s());
    rp->ctx = ctx;
    rp->cfg = *cfg;
    rp->I = I, rp->N = N, rp->K = K, rp->L = L;
    rp->n = 13 * (int64_t)N - 5;
    const int64_t n = rp->n;
    Arena &a = rp->mem;
    int rc = IMPC_OK;
    auto cleanup = [&]() {
        for (Shape &s : rp->sh) free_shape(s);
        if (rp->h_counts) (void)hipHostFree(rp->h_counts);
        rp->mem.release();
    };
#define RP_CK(expr)       \
    if ((rc = (expr))) {  \
        cleanup();        \
        return rc;        \
    }
    RP_CK(a.get((size_t)((I + 1) * n), &rp->plan_x));
    RP_CK(a.get((size_t)((I + 1) * N * 8), &rp->plan_states));
    RP_CK(a.get((size_t)I, &rp->prev_count));
    RP_CK(a.get((size_t)I, &rp->first_time));
    RP_CK(a.get((size_t)I, &rp->valid));
    RP_CK(a.get((size_t)I, &rp->zeros8));
    RP_CK(a.get((size_t)I, &rp->branch));
    RP_CK(a.get((size_t)I, &rp->inst_f));
    RP_CK(a.get((size_t)I, &rp->inst_0));
    RP_CK(a.get((size_t)I, &rp->ws_0));
    RP_CK(a.get((size_t)I, &rp->inst_1));
    RP_CK(a.get((size_t)4, &rp->d_counts));
    RP_CK(a.get((size_t)I, &rp->best));
    RP_CK(a.get((size_t)I, &rp->ob));
    RP_CK(a.get((size_t)(6 * I), &rp->ctype));
    RP_CK(a.get((size_t)(6 * I), &rp->cslot));
    RP_CK(a.get((size_t)(3 * I), &rp->f_pos));
    RP_CK(a.get((size_t)(3 * I), &rp->f_vel));
    RP_CK(a.get((size_t)(I * N * 8), &rp->f_xref));
    RP_CK(a.get((size_t)(I * N * 8), &rp->f_lin));
    RP_CK(a.get((size_t)(I * K * 3), &rp->f_dcur));
    RP_CK(a.get((size_t)(I * K * 4 * L * 3), &rp->f_ppos));
    RP_CK(a.get((size_t)(I * K * 4 * L * 3), &rp->f_psize));
    RP_CK(a.get((size_t)(I * K * 4), &rp->f_prob));
    RP_CK(a.get((size_t)(I * n), &rp->f_ws));
    RP_CK(a.get((size_t)I, &rp->f_pc));
    RP_CK(a.get((size_t)I, &rp->f_ob));
    RP_CK(a.get((size_t)(6 * I), &rp->f_ctype));
    RP_CK(a.get((size_t)(6 * I), &rp->f_cslot));
    RP_CK(a.get((size_t)(4 * I), &rp->f_cprob));
    RP_CK(a.get((size_t)(I * 4 * K * L * 3), &rp->s_pos));
    RP_CK(a.get((size_t)(I * 4 * K * L * 3), &rp->s_size));
    RP_CK(a.get((size_t)(I * 2 * (K + 1) * L * 3), &rp->p_pos));
    RP_CK(a.get((size_t)(I * 2 * (K + 1) * L * 3), &rp->p_size));
    RP_CK(a.get((size_t)(6 * I), &rp->x_cand));
    RP_CK(a.get((size_t)(6 * I), &rp->dyn_count));
    RP_CK(a.get((size_t)I, &rp->best_f));
    RP_CK(a.get((size_t)I, &rp->best_pos));
    RP_CK(a.get((size_t)(I * 6 * (K + 1) * L * 3), &rp->dyn_pos));
    RP_CK(a.get((size_t)(I * 6 * (K + 1) * L * 3), &rp->dyn_size));
    RP_CK(a.get((size_t)(I * 6 * 3), &rp->scores));
    RP_CK(a.get((size_t)(I * 6), &rp->weighted));
    RP_CK(a.get((size_t)(I * 6), &rp->cvalid));
    if (hipHostMalloc((void **)&rp->h_counts, 4 * sizeof(int64_t), hipHostMallocDefault) != hipSuccess) {
        rp->h_counts = nullptr;
        cleanup();
        return fail(IMPC_MEM_ALLOC_ERROR, "replan: pinned counts");
    }
    hipStream_t st = impc_lib::stream(ctx);
    if (hipMemsetAsync(rp->zeros8, 0, (size_t)I, st) != hipSuccess ||
        hipMemsetAsync(rp->valid, 0, (size_t)I, st) != hipSuccess) {
        cleanup();
        return fail(IMPC_DEVICE_ERROR, "replan: memset");
    }
    // fan-out shapes (single-intent K obstacles, 4 per instance; two-intent K + 1, 2 per instance)
    // and the obstacle-free single solve; the current-obstacle shape is created on first use
    RP_CK(make_shape(rp.get(), rp->sh[0], K, L, 4, 4 * I, false));
    RP_CK(make_shape(rp.get(), rp->sh[1], K + 1, L, 2, 2 * I, false));
    RP_CK(make_shape(rp.get(), rp->sh[2], 0, 1, 1, I, false));
#undef RP_CK
    rc = impc_replan_set_state(rp.get(), nullptr, nullptr);
    if (rc) {
        cleanup();
        return rc;
    }
    *out = rp.release();
    return IMPC_OK;
}

int impc_replan_destroy(impc_replan rp) {
    if (!rp) return IMPC_OK;
    (void)hipSetDevice(impc_lib::device(rp->ctx));
    (void)impc_ctx_synchronize(rp->ctx);
    for (Shape &s : rp->sh) free_shape(s);
    if (rp->h_counts) (void)hipHostFree(rp->h_counts);
    rp->mem.release();
    delete rp;
    return IMPC_OK;
}

int impc_replan_set_state(impc_replan rp, const double *plan_x, const int8_t *first_time) {
    if (!rp) return fail(IMPC_INVALID_ARGUMENT, "null replan");
    const int64_t I = rp->I, n = rp->n, N = rp->N;
    std::vector<double> px((size_t)((I + 1) * n), 0.0), ps((size_t)((I + 1) * N * 8), 0.0);
    if (plan_x) std::memcpy(px.data(), plan_x, sizeof(double) * (size_t)(I * n));
    for (int64_t i = 0; i < I; i++) std::memcpy(&ps[(size_t)(i * N * 8)], &px[(size_t)(i * n)], sizeof(double) * 8 * N);
    std::vector<int8_t> ft((size_t)I, 1);
    if (first_time)
        for (int64_t i = 0; i < I; i++) ft[(size_t)i] = first_time[i] ? 1 : 0;
    std::vector<int32_t> pc((size_t)I);
    for (int64_t i = 0; i < I; i++) pc[(size_t)i] = ft[(size_t)i] ? 0 : (int32_t)N;  // currentStatesSol_.size()
    std::vector<int8_t> v((size_t)I, 0);
    RP_TRY(impc_copy_to_device(rp->ctx, rp->plan_x, px.data(), (int64_t)(px.size() * 8)));
    RP_TRY(impc_copy_to_device(rp->ctx, rp->plan_states, ps.data(), (int64_t)(ps.size() * 8)));
    RP_TRY(impc_copy_to_device(rp->ctx, rp->first_time, ft.data(), I));
    RP_TRY(impc_copy_to_device(rp->ctx, rp->prev_count, pc.data(), 4 * I));
    RP_TRY(impc_copy_to_device(rp->ctx, rp->valid, v.data(), I));
    return IMPC_OK;
}

int impc_replan_run(impc_replan rp, const impc_replan_inputs *in) {
    using clk = std::chrono::steady_clock;
    const auto t_entry = clk::now();
    if (!rp || !in) return fail(IMPC_INVALID_ARGUMENT, "replan: null object or inputs");
    if (!in->pos || !in->vel || !in->xref || !in->dyn_cur || !in->pred_pos || !in->pred_size || !in->prob)
        return fail(IMPC_INVALID_ARGUMENT, "replan: pos, vel, xref, dyn_cur, pred_pos, pred_size, prob are required");
    if (in->cur_count && !in->cur_size) return fail(IMPC_INVALID_ARGUMENT, "replan: cur_count needs cur_size");
    impc_ctx ctx = rp->ctx;
    RP_HIP(hipSetDevice(impc_lib::device(ctx)));
    hipStream_t st = impc_lib::stream(ctx);
    RP_TRY(impc_lib::order_after_all(ctx));
    const int64_t I = rp->I, n = rp->n, N = rp->N, K = rp->K, L = rp->L;

    // ---- branch table (:593-606); the three counts come back to the host
    hipLaunchKernelGGL(k_branch_table, dim3(1), dim3(kTableLanes), 0, st, I, rp->first_time, in->has_pred,
                       in->cur_count, in->cur_size ? 1 : 0, rp->branch, rp->inst_f, rp->inst_0, rp->ws_0, rp->inst_1,
                       rp->d_counts, rp->best, rp->ob, rp->ctype, rp->cslot);
    RP_HIP(hipGetLastError());
    RP_HIP(hipMemcpyAsync(rp->h_counts, rp->d_counts, 3 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    RP_HIP(hipStreamSynchronize(st));
    const int64_t nf = rp->h_counts[0], n0 = rp->h_counts[1], n1 = rp->h_counts[2];
    Shape &S = rp->sh[0], &P = rp->sh[1], &F0 = rp->sh[2];
    if (n1 && !rp->sh[3].batch) RP_TRY(make_shape(rp, rp->sh[3], (int32_t)K, (int32_t)N, 1, I, true));
    Shape &C1 = rp->sh[3];

    // ---- fan-out branch: its instances' inputs compacted, the six candidates, the assembly
    if (nf) {
        const int64_t *idx = rp->inst_f;
        RP_TRY(impc_gather_rows_device(ctx, in->pos, 24, idx, nf, rp->f_pos, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, in->vel, 24, idx, nf, rp->f_vel, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, in->xref, 64 * N, idx, nf, rp->f_xref, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, rp->plan_states, 64 * N, idx, nf, rp->f_lin, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, rp->prev_count, 4, idx, nf, rp->f_pc, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, in->dyn_cur, 24 * K, idx, nf, rp->f_dcur, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, in->pred_pos, 8 * K * 4 * L * 3, idx, nf, rp->f_ppos, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, in->pred_size, 8 * K * 4 * L * 3, idx, nf, rp->f_psize, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, in->prob, 32 * K, idx, nf, rp->f_prob, nullptr));
        // fan-out instances are never on their first plan (the branch's condition)
        RP_TRY(impc_intent_fanout_device(ctx, nf, (int32_t)K, (int32_t)L, (int32_t)N, rp->f_pos, rp->zeros8, rp->f_lin,
                                         rp->f_pc, rp->f_dcur, rp->f_ppos, rp->f_psize, rp->f_prob, rp->f_ob,
                                         rp->f_ctype, rp->f_cslot, rp->f_cprob, rp->s_pos, rp->s_size, rp->p_pos,
                                         rp->p_size, nullptr));
        for (Shape *s : {&S, &P}) {
            RP_TRY(impc_repeat_rows_device(ctx, rp->f_pos, nf, 24, s->rep, s->pos, nullptr));
            RP_TRY(impc_repeat_rows_device(ctx, rp->f_vel, nf, 24, s->rep, s->vel, nullptr));
            RP_TRY(impc_repeat_rows_device(ctx, rp->f_xref, nf, 64 * N, s->rep, s->xref, nullptr));
            RP_TRY(impc_repeat_rows_device(ctx, rp->f_lin, nf, 64 * N, s->rep, s->lin, nullptr));
            s->inst = rp->inst_f;
        }
        RP_TRY(assemble(rp, S, nf, S.lin, rp->s_pos, rp->s_size, idx, rp->f_ws));
        RP_TRY(assemble(rp, P, nf, P.lin, rp->p_pos, rp->p_size, idx, rp->f_ws));
    } else {
        S.count = P.count = S.ninst = P.ninst = 0;
    }
    // ---- single solve, first plan / no obstacles: no linearisation point (no obstacle rows)
    F0.inst = rp->inst_0;
    if (n0) {
        RP_TRY(impc_gather_rows_device(ctx, in->pos, 24, rp->inst_0, n0, F0.pos, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, in->vel, 24, rp->inst_0, n0, F0.vel, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, in->xref, 64 * N, rp->inst_0, n0, F0.xref, nullptr));
    }
    RP_TRY(assemble(rp, F0, n0, nullptr, nullptr, nullptr, rp->ws_0, nullptr));
    // ---- single solve with the current obstacles held over the horizon
    if (n1) {
        C1.inst = rp->inst_1;
        RP_TRY(impc_gather_rows_device(ctx, in->pos, 24, rp->inst_1, n1, C1.pos, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, in->vel, 24, rp->inst_1, n1, C1.vel, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, in->xref, 64 * N, rp->inst_1, n1, C1.xref, nullptr));
        RP_TRY(impc_gather_rows_device(ctx, rp->plan_states, 64 * N, rp->inst_1, n1, C1.lin, nullptr));
        const int64_t hw = n1 * K * N * 3;
        hipLaunchKernelGGL(k_hold, dim3(grid_for(rp, hw)), dim3(256), 0, st, in->dyn_cur, rp->inst_1, n1, (int32_t)K,
                           (int32_t)N, C1.dpos);
        hipLaunchKernelGGL(k_hold, dim3(grid_for(rp, hw)), dim3(256), 0, st, in->cur_size, rp->inst_1, n1, (int32_t)K,
                           (int32_t)N, C1.dsize);
        RP_HIP(hipGetLastError());
        RP_TRY(assemble(rp, C1, n1, C1.lin, C1.dpos, C1.dsize, rp->inst_1, nullptr));
    } else if (C1.batch) {
        C1.count = C1.ninst = 0;
    }

    // ---- the issue cut-off (:613) after the assembly; the candidates' time limit (:614)
    RP_HIP(hipStreamSynchronize(st));
    const auto t_staged = clk::now();
    const double elapsed = in->elapsed_s + std::chrono::duration<double>(t_staged - t_entry).count();
    const bool issued = !(rp->cfg.issue_cutoff_s > 0.0) || elapsed < rp->cfg.issue_cutoff_s;
    double tl = rp->cfg.settings.time_limit;
    if (in->solver_time_limit > 0.0) tl = std::max(in->solver_time_limit - elapsed, in->solver_time_limit);
    std::vector<impc_batch> launch;
    for (Shape *s : {&S, &P})
        if (s->count && issued) {
            RP_TRY(set_limit(rp, *s, tl));
            launch.push_back(s->batch);
        }
    for (Shape *s : {&F0, &C1})  // solveTraj's default (none on a first plan, :442-444)
        if (s->batch && s->count) {
            RP_TRY(set_limit(rp, *s, 0.0));
            launch.push_back(s->batch);
        }
    if (!issued) S.count = P.count = 0;  // nothing of the fan-out ran (impc_replan_shape)
    if (!launch.empty()) RP_TRY(impc_batch_solve_group(launch.data(), (int)launch.size(), nullptr));

    // ---- candidate validity, selection, commit
    if (nf) {
        impc_info *info_s = nullptr, *info_p = nullptr;
        double *x_s = nullptr, *x_p = nullptr;
        RP_TRY(impc_batch_device_results(S.batch, &x_s, nullptr, &info_s));
        RP_TRY(impc_batch_device_results(P.batch, &x_p, nullptr, &info_p));
        hipLaunchKernelGGL(k_cand_valid, dim3(grid_for(rp, 6 * nf)), dim3(256), 0, st, nf, rp->f_cslot, info_s, info_p,
                           issued ? 1 : 0, rp->cvalid);
        RP_HIP(hipGetLastError());
        RP_TRY(impc_fanout_candidates_device(ctx, nf, (int32_t)K, (int32_t)L, rp->f_cslot, rp->s_pos, rp->s_size,
                                             rp->p_pos, rp->p_size, x_s, S.dm.n, x_p, P.dm.n, rp->x_cand,
                                             rp->dyn_count, rp->dyn_pos, rp->dyn_size, nullptr));
        impc_select_params sp{};
        sp.horizon = (int32_t)N, sp.num_candidates = 6, sp.max_dynamic = (int32_t)K + 1, sp.pred_len = (int32_t)L;
        sp.num_static = 0, sp.prev_len = (int32_t)N;
        sp.dynamic_safety_dist = rp->cfg.mpc.dynamic_safety_dist;
        sp.static_safety_dist = rp->cfg.mpc.static_safety_dist;
        RP_TRY(impc_select_best_device(ctx, &sp, nf, rp->x_cand, rp->cvalid, rp->zeros8, rp->f_lin, rp->f_pc,
                                       rp->f_xref, nullptr, nullptr, rp->dyn_count, rp->dyn_pos, rp->dyn_size,
                                       rp->f_cprob, rp->best_f, rp->best_pos, rp->scores, rp->weighted, nullptr));
        RP_TRY(impc_replan_commit_device(ctx, (int32_t)N, n, nf, rp->inst_f, (const uint64_t *)rp->x_cand, 6,
                                         rp->best_f, nullptr, nullptr, rp->plan_x, rp->plan_states, rp->prev_count,
                                         rp->first_time, rp->valid, nullptr));
        hipLaunchKernelGGL(k_scatter, dim3(grid_for(rp, nf)), dim3(256), 0, st, nf, rp->inst_f, rp->best_f, rp->f_ob,
                           rp->f_ctype, rp->f_cslot, rp->best, rp->ob, rp->ctype, rp->cslot);
        RP_HIP(hipGetLastError());
    }
    for (Shape *s : {&F0, &C1}) {
        if (!s->batch || !s->count) continue;
        double *x = nullptr;
        impc_info *info = nullptr;
        RP_TRY(impc_batch_device_results(s->batch, &x, nullptr, &info));
        RP_TRY(impc_replan_commit_device(ctx, (int32_t)N, n, s->count, s->inst, nullptr, 0, nullptr, x, info,
                                         rp->plan_x, rp->plan_states, rp->prev_count, rp->first_time, rp->valid,
                                         nullptr));
    }
    const auto t_end = clk::now();
    impc_replan_stats &o = rp->stats;
    o.fanout = nf, o.single_first = n0, o.single_current = n1;
    o.issued = issued ? 1 : 0;
    o.time_limit = tl;
    o.stage_s = std::chrono::duration<double>(t_staged - t_entry).count();
    o.total_s = std::chrono::duration<double>(t_end - t_entry).count();
    return IMPC_OK;
}

int impc_replan_get_stats(impc_replan rp, impc_replan_stats *out) {
    if (!rp || !out) return fail(IMPC_INVALID_ARGUMENT, "replan: null object or output");
    *out = rp->stats;
    return IMPC_OK;
}

int impc_replan_view_device(impc_replan rp, impc_replan_view *out) {
    if (!rp || !out) return fail(IMPC_INVALID_ARGUMENT, "replan: null object or output");
    out->plan_x = rp->plan_x, out->plan_states = rp->plan_states, out->prev_count = rp->prev_count;
    out->first_time = rp->first_time, out->valid = rp->valid, out->branch = rp->branch;
    out->best_cand = rp->best, out->ob_idx = rp->ob, out->cand_type = rp->ctype, out->cand_slot = rp->cslot;
    return IMPC_OK;
}

int impc_replan_shape(impc_replan rp, int32_t shape, impc_batch *batch, int64_t *count, const int64_t **inst,
                      const double **Px, const double **q, const double **Ax, const double **l, const double **u) {
    if (!rp || shape < 0 || shape > 3) return fail(IMPC_INVALID_ARGUMENT, "replan: shape must be 0..3");
    const Shape &s = rp->sh[shape];
    if (batch) *batch = s.batch;
    if (count) *count = s.batch ? s.count : 0;
    if (inst) *inst = s.inst;
    impc_lib::BatchInputs bi{};
    if (s.batch) {
        RP_TRY(impc_lib::batch_inputs_view(s.batch, &bi));  // the inputs of the last assembly
    }
    if (Px) *Px = bi.Px;
    if (q) *q = bi.q;
    if (Ax) *Ax = bi.Ax;
    if (l) *l = bi.l;
    if (u) *u = bi.u;
    return IMPC_OK;
}

int impc_replan_advance_device(impc_replan rp, double t, double *pos, double *vel) {
    if (!rp || !pos || !vel || !(t >= 0.0)) return fail(IMPC_INVALID_ARGUMENT, "replan advance: t >= 0, pos, vel");
    RP_HIP(hipSetDevice(impc_lib::device(rp->ctx)));
    hipLaunchKernelGGL(k_advance, dim3(grid_for(rp, rp->I)), dim3(256), 0, impc_lib::stream(rp->ctx), rp->I, rp->N,
                       rp->n, rp->cfg.mpc.ts, t, rp->valid, rp->plan_x, pos, vel);
    RP_HIP(hipGetLastError());
    return IMPC_OK;
}

}  // extern "C"
