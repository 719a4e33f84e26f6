// replan_run.hip -- the whole batched makePlanWithPred behind one C-ABI call (include/impc_replan.h,
// impc_replan_*), part of libimpc_qp.so.
//
// Reference: trajectory_planner/include/trajectory_planner/mpcPlanner.cpp:571-661 (makePlanWithPred),
// called per planning instance by mpcNavigation.cpp:316-322.  Per instance it takes one of three
// branches (:593-606) -- the intent fan-out with six candidate solves and a selection, or ONE
// solveTraj (first plan, or no predictions) -- and commits the plan it gets into the planner state.
// Every instance may track a different number of obstacles (predPos.size(), :343-373).  Here every
// instance of a batch goes through one call, and the call never waits for the device:
//
//   k_plan_rows   one workgroup: the branch of every instance and the rows of every QP shape
//                 (shape k = the QPs with k obstacle rows per stage), by a scan over the instances;
//                 the device clock at the start of the replan
//   k_pick        one thread per instance: findClosestObstacle + getIntentComb's candidate order
//   k_prep        one wavefront per row: the warm start, the time limit and the obstacle sources
//                 (which prediction / current obstacle each obstacle row linearises)
//   build         impc_lib::build_rows per shape: the device builder straight from the per-instance
//                 inputs, written in place into the shape's solver batch
//   k_issue       the issue cut-off (:613) on the device clock; each shape's solve count
//   solve         ONE impc_batch_solve_group over every shape, each batch's QP count read from
//                 device memory by the solver itself
//   k_cand        the candidates' validity (solveProblem NoError), solution pointers, obstacle sets
//   selection     impc_select_best_device over every instance (non-fan-out instances: no candidate)
//   k_commit      every plan into the planner state
//
// No x, y, QP value or count leaves the device, and nothing on the host waits for it.
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

constexpr int kPlanLanes = 512;
constexpr int kMaxObstacles = 30;
constexpr int FORWARD = 0, LEFT = 1, RIGHT = 2, STOP = 3;  // dynamicPredictor's intent enum

// Shape k's rows in the flat row arrays: shape 0 holds the single solves without dynamic
// obstacles (<= I rows); shapes 1..K at most four rows per instance (the four single-intent
// candidates of an instance with K_i = k, or the two two-intent candidates of one with K_i + 1 =
// k, or one current-obstacle single solve with c_i = k); shape K + 1 the two-intent candidates of
// the instances with K_i = K (<= 2 I rows); shape K + 2, present with static obstacles only, the
// first plans (<= I rows; without static obstacles they are shape 0's).
__host__ __device__ inline int64_t shape_base(int64_t I, int K, int k) {
    return k == 0 ? 0 : k <= K + 1 ? I + 4 * I * (int64_t)(k - 1) : I * (4 * (int64_t)K + 3);
}
__host__ __device__ inline int64_t shape_cap(int64_t I, int K, int k) {
    return k == 0 ? I : k <= K ? 4 * I : k == K + 1 ? 2 * I : I;
}
__host__ __device__ inline int shape_of(int64_t I, int K, int64_t f) {
    if (f < I) return 0;
    if (f >= I * (4 * (int64_t)K + 3)) return K + 2;
    const int64_t k = 1 + (f - I) / (4 * I);
    return (int)(k < K + 1 ? k : K + 1);
}
// the dynamic-obstacle rows per stage of shape k's QPs
__host__ __device__ inline int shape_dyn(int K, int k) { return k <= K + 1 ? k : 0; }

// per-shape device pointers, fixed when the replan object is created
struct ShapeDev {
    double *xws, *tlim;       // the batch's warm-start input [cap][n] and time limits [cap]
    const double *x;          // the batch's primal solutions [cap][n]
    const impc_info *info;    // [cap]
    int64_t *osrc;            // obstacle sources [cap][k] (build_rows)
};

// The branch of one instance (:593-606), its predicted-obstacle count K_i and current count c_i.
struct Decide {
    const int8_t *first_time, *has_pred;
    const int32_t *num_pred, *cur_count;
    int32_t K, cur_all;
    __device__ void operator()(int64_t i, int &br, int &ki, int &ci) const {
        const bool ft = first_time[i] != 0;
        ki = num_pred ? min(max(num_pred[i], 0), K) : K;
        const bool hp = (has_pred ? has_pred[i] != 0 : true) && ki > 0;  // obPredPos_.size() != 0
        ci = cur_count ? min(max(cur_count[i], 0), K) : (cur_all ? K : 0);
        br = (!ft && hp) ? IMPC_REPLAN_FANOUT : (!ft && ci > 0) ? IMPC_REPLAN_SINGLE_CURRENT : IMPC_REPLAN_SINGLE_FIRST;
    }
};

struct PlanArgs {
    int64_t I;
    int32_t K, S, first_shape;  // first_shape: the first plans' shape (K + 2 with static obstacles, else 0)
    Decide decide;
    int8_t *branch;
    int32_t *num_obs, *shp, *slot_row, *best;
    int32_t *row_inst;
    int8_t *row_code;
    int64_t *cnt;               // [S] single solves per shape, [S .. 2S) rows per shape, [2S .. 2S+3) branches
    unsigned long long *clk;    // [0] the device clock at the start of the replan
};

// The shape of a single solve: a first plan's QP has no obstacle rows (static and dynamic obstacles
// cleared, :593-602), any other has the current obstacles' c_i (0 with SINGLE_FIRST) and the statics.
__device__ inline int single_shape(const PlanArgs &a, int64_t i, int br, int ci) {
    return br == IMPC_REPLAN_SINGLE_CURRENT ? ci : a.decide.first_time[i] != 0 ? a.first_shape : 0;
}

// One workgroup of kPlanLanes lanes, lane t owning a contiguous range of instances.  Counters
// [R = 2S + 3][kPlanLanes] in LDS (rows 0..S-1: single solves of shape k, S..2S-1: candidate rows
// of shape k, 2S..2S+2: instances per branch), an exclusive scan over the lanes (a wavefront scan
// of 64 lanes, then the wavefront totals), and a second pass that writes each instance's rows in
// ascending order: every shape holds its single solves first, then its candidates.
__global__ __launch_bounds__(kPlanLanes) void k_plan_rows(PlanArgs a) {
    extern __shared__ int32_t cl[];  // [R][kPlanLanes], then wave totals [R][kPlanLanes / 64]
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, NW = kPlanLanes / 64;
    const int S = a.S, R = 2 * S + 3;
    int32_t *wt = cl + R * kPlanLanes;
    if (t == 0) a.clk[0] = wall_clock64();
    const int64_t per = (a.I + kPlanLanes - 1) / kPlanLanes;
    const int64_t i0 = min(a.I, (int64_t)t * per), i1 = min(a.I, i0 + per);
    for (int r = 0; r < R; r++) cl[r * kPlanLanes + t] = 0;
    for (int64_t i = i0; i < i1; i++) {
        int br, ki, ci;
        a.decide(i, br, ki, ci);
        cl[(2 * S + br) * kPlanLanes + t]++;
        if (br == IMPC_REPLAN_FANOUT) {
            cl[(S + ki) * kPlanLanes + t] += 4;
            cl[(S + ki + 1) * kPlanLanes + t] += 2;
        } else {
            cl[single_shape(a, i, br, ci) * kPlanLanes + t]++;
        }
    }
    for (int r = 0; r < R; r++) {  // exclusive scan inside each wavefront
        const int v = cl[r * kPlanLanes + t];
        int x = v;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        cl[r * kPlanLanes + t] = x - v;
        if (lane == 63) wt[r * NW + w] = x;
    }
    __syncthreads();
    for (int r = 0; r < R; r++) {
        int add = 0;
        for (int ww = 0; ww < w; ww++) add += wt[r * NW + ww];
        cl[r * kPlanLanes + t] += add;
    }
    auto total = [&](int r) {
        int64_t s = 0;
        for (int ww = 0; ww < NW; ww++) s += wt[r * NW + ww];
        return s;
    };
    for (int64_t i = i0; i < i1; i++) {
        int br, ki, ci;
        a.decide(i, br, ki, ci);
        a.branch[i] = (int8_t)br;
        a.best[i] = -1;
        int32_t *sr = a.slot_row + 6 * i;
        for (int s = 0; s < 6; s++) sr[s] = -1;
        if (br == IMPC_REPLAN_FANOUT) {
            a.num_obs[i] = ki;
            a.shp[i] = ki;
            for (int s = 0; s < 6; s++) {
                const int k = s < 4 ? ki : ki + 1;
                const int64_t r = total(k) + cl[(S + k) * kPlanLanes + t]++;
                const int64_t f = shape_base(a.I, a.K, k) + r;
                a.row_inst[f] = (int32_t)i;
                a.row_code[f] = (int8_t)s;
                sr[s] = (int32_t)r;
            }
        } else {
            const int k = single_shape(a, i, br, ci);
            const int64_t r = cl[k * kPlanLanes + t]++;
            const int64_t f = shape_base(a.I, a.K, k) + r;
            a.row_inst[f] = (int32_t)i;
            a.row_code[f] = (int8_t)(br == IMPC_REPLAN_SINGLE_FIRST ? IMPC_REPLAN_ROW_FIRST : IMPC_REPLAN_ROW_CURRENT);
            a.num_obs[i] = br == IMPC_REPLAN_SINGLE_FIRST ? 0 : ci;
            a.shp[i] = k;
            sr[0] = (int32_t)r;
        }
    }
    if (t == 0) {
        for (int k = 0; k < S; k++) {
            a.cnt[k] = total(k);
            a.cnt[S + k] = total(k) + total(S + k);
        }
        for (int b = 0; b < 3; b++) a.cnt[2 * S + b] = total(2 * S + b);
    }
}

__device__ inline double norm3(double a, double b, double c) {
#pragma clang fp contract(off)
    return sqrt((a * a + b * b) + c * c);
}

// maxCoeff (:762): the first most probable intent of one obstacle's [4] probabilities
__device__ inline int max_intent(const double *p) {
    int m = 0;
    for (int q = 1; q < 4; q++)
        if (p[q] > p[m]) m = q;
    return m;
}

struct PickArgs {
    int64_t I;
    int32_t K, N;
    const int8_t *branch;
    const int32_t *num_obs;
    const double *pos, *plan_states, *dyn_cur, *prob;
    const int32_t *prev_count;
    int32_t *ob, *ctype, *cslot, *slot_type;
    double *cprob;
};

// findClosestObstacle (:663-708, over the instance's K_i obstacles; a fan-out instance is never on
// its first plan) and getIntentComb's order (:719-756: std::sort of (weight, index) pairs, taken
// from the back); single-solve instances get -1.  As impc_intent_fanout_device (fanout.hpp), with
// the obstacle count per instance.
__global__ __launch_bounds__(64) void k_pick(PickArgs a) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.I) return;
    int32_t *ct = a.ctype + 6 * i, *cs = a.cslot + 6 * i, *sty = a.slot_type + 6 * i;
    if (a.branch[i] != IMPC_REPLAN_FANOUT) {
        a.ob[i] = -1;
        for (int c = 0; c < 6; c++) ct[c] = cs[c] = sty[c] = -1;
        return;
    }
    const int K = a.K, Ki = a.num_obs[i];
    const double *cp = a.pos + 3 * i, *dc = a.dyn_cur + i * K * 3;
    int ob = -1;
    double minD = INFINITY;
    const int pc = a.prev_count[i];
    if (pc < 2) {  // distance to the current position (:676-686)
        for (int k = 0; k < Ki; k++) {
            const double d = norm3(cp[0] - dc[3 * k], cp[1] - dc[3 * k + 1], cp[2] - dc[3 * k + 2]);
            if (d < minD) {
                minD = d;
                ob = k;
            }
        }
    } else {  // direction-weighted, every term at states[0] / states[1] as written (:687-706)
        const double *s = a.plan_states + i * (int64_t)a.N * 8, *ns = s + 8;
        const double traj = atan2(ns[1] - s[1], ns[0] - s[0]);
        for (int k = 0; k < Ki; k++) {
            const double obs = atan2(dc[3 * k + 1] - s[1], dc[3 * k] - s[0]);
            const double d = norm3(s[0] - dc[3 * k], s[1] - dc[3 * k + 1], s[2] - dc[3 * k + 2]);
            double dist = 0.0;
            for (int j = 0; j < pc / 3; j++) {
                const double w = exp((double)-j);
                dist += w * d * (3.0 - cos(traj - obs));
                if (dist > minD) break;
            }
            if (dist < minD) {
                minD = dist;
                ob = k;
            }
        }
    }
    if (ob < 0) ob = 0;  // only with NaN inputs (the reference would index -1)
    a.ob[i] = ob;
    const double *pr = a.prob + (i * K + ob) * 4;
    const double w[6] = {pr[STOP], pr[LEFT], pr[RIGHT], pr[FORWARD], pr[LEFT] < pr[FORWARD] ? pr[FORWARD] : pr[LEFT],
                         pr[RIGHT] < pr[FORWARD] ? pr[FORWARD] : pr[RIGHT]};
    int type_at[6];
    for (int t = 0; t < 6; t++) {
        int pos = 0;
        for (int u = 0; u < 6; u++)
            if (w[t] < w[u] || (!(w[u] < w[t]) && t < u)) pos++;
        type_at[pos] = t;
    }
    int ns_ = 0, np_ = 0;
    for (int c = 0; c < 6; c++) {
        const int t = type_at[c];
        const int s = t < 4 ? ns_++ : 4 + np_++;
        ct[c] = t;
        cs[c] = s;
        sty[s] = t;
    }
    for (int q = 0; q < 4; q++) a.cprob[4 * i + q] = pr[q];
}

// Obstacle o of slot s's candidate (getIntentComb :731-768): the closest obstacle's intents
// first, then every other obstacle in index order at its most probable intent.
__device__ inline void cand_obstacle(int ob, int t, bool pair, int o, const double *prob_i, int &k, int &intent) {
    const int nfirst = pair ? 2 : 1;
    if (o < nfirst) {
        k = ob;
        constexpr int single_intent[4] = {STOP, LEFT, RIGHT, FORWARD};
        intent = t < 4 ? single_intent[t] : (o == 0 ? (t == 4 ? LEFT : RIGHT) : FORWARD);
    } else {
        const int q = o - nfirst;
        k = q < ob ? q : q + 1;
        intent = max_intent(prob_i + 4 * k);
    }
}

struct PrepArgs {
    int64_t I, n, total;
    int32_t K, L, S;
    const int64_t *cnt;
    const ShapeDev *sh;
    const int32_t *row_inst, *ob, *slot_type;
    const int8_t *row_code, *first_time;
    const double *plan_x, *prob;
    double cand_limit;
};

// One wavefront per row (grid-stride over every shape's capacity; rows past a shape's count are
// skipped): the warm start (solveTraj :485-509: the plan, or zeros on a first plan -- row I of
// plan_x), the row's time limit (candidates: timeLimit; single solves: none, :442-444) and the
// sources of its obstacle rows for the builder.
__global__ __launch_bounds__(64) void k_prep(PrepArgs a) {
    for (int64_t f = blockIdx.x; f < a.total; f += gridDim.x) {
        const int k = shape_of(a.I, a.K, f);
        const int64_t r = f - shape_base(a.I, a.K, k);
        if (r >= a.cnt[a.S + k]) continue;
        const ShapeDev sd = a.sh[k];
        const int64_t i = a.row_inst[f];
        const int code = a.row_code[f];
        const double *src = a.plan_x + ((code == IMPC_REPLAN_ROW_FIRST && a.first_time[i]) ? a.I : i) * a.n;
        double *dst = sd.xws + r * a.n;
        for (int64_t e = threadIdx.x; e < a.n; e += blockDim.x) dst[e] = src[e];
        if (threadIdx.x == 0) sd.tlim[r] = code < 6 ? a.cand_limit : 0.0;
        const int kd = shape_dyn(a.K, k);
        for (int o = threadIdx.x; o < kd; o += blockDim.x) {
            int64_t off;
            if (code == IMPC_REPLAN_ROW_CURRENT) {  // held over the horizon
                off = ((i * a.K + o) * 3) << 1 | 1;
            } else {
                int kk, intent;
                cand_obstacle(a.ob[i], a.slot_type[6 * i + code], code >= 4, o, a.prob + i * a.K * 4, kk, intent);
                off = ((((i * a.K + kk) * 4 + intent) * (int64_t)a.L) * 3) << 1;
            }
            sd.osrc[r * kd + o] = off;
        }
    }
}

// The issue cut-off (:612-613) after the assembly, on the device clock; the solve count of each
// shape (its single solves always, its candidates when issued)
__global__ void k_issue(int32_t S, int64_t *cnt, int64_t *solve, unsigned long long *clk, int32_t *issued_out,
                        double elapsed_s, double tick, double cutoff) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const unsigned long long now = wall_clock64();
    clk[1] = now;
    const double elapsed = elapsed_s + (double)(now - clk[0]) * tick;
    const bool issued = !(cutoff > 0.0) || elapsed < cutoff;
    for (int k = 0; k < S; k++) solve[k] = issued ? cnt[S + k] : cnt[k];
    *issued_out = issued ? 1 : 0;
}

struct CandArgs {
    int64_t I, n;
    int32_t K, L;
    const ShapeDev *sh;
    const int8_t *branch;
    const int32_t *num_obs, *slot_row, *cslot, *slot_type, *ob;
    const int32_t *issued;
    const double *pred_pos, *pred_size, *prob;
    const double **x_cand;
    int32_t *dyn_count;
    int8_t *valid;
    double *dpos, *dsize;  // [I][6][K + 1][L][3], the selection's padded obstacle sets
};

// per (instance, candidate): solveTraj's success (impc_lib::solve_traj_ok, :475-478, :513-518) when issued,
// the pointer to the solution, the obstacle count
__global__ void k_cand(CandArgs a) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.I * 6; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / 6;
        if (a.branch[i] != IMPC_REPLAN_FANOUT) {
            a.valid[e] = 0;
            a.x_cand[e] = nullptr;
            a.dyn_count[e] = 0;
            continue;
        }
        const int s = a.cslot[e], k = s < 4 ? a.num_obs[i] : a.num_obs[i] + 1;
        const int64_t r = a.slot_row[6 * i + s];
        a.valid[e] = (*a.issued && impc_lib::solve_traj_ok(a.sh[k].info[r])) ? 1 : 0;
        a.x_cand[e] = a.sh[k].x + r * a.n;
        a.dyn_count[e] = k;
    }
}

// the candidates' obstacle sets in the selection's padded layout (entries past a candidate's
// count are never read by the selection and are not written)
__global__ void k_sel_sets(CandArgs a) {
    const int64_t per_c = (int64_t)(a.K + 1) * a.L, total = a.I * 6 * per_c;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t ic = e / per_c, i = ic / 6;
        if (a.branch[i] != IMPC_REPLAN_FANOUT) continue;
        const int rr = (int)(e - ic * per_c), o = rr / a.L, st = rr % a.L;
        const int s = a.cslot[ic];
        const bool pair = s >= 4;
        if (o >= a.num_obs[i] + (pair ? 1 : 0)) continue;
        int kk, intent;
        cand_obstacle(a.ob[i], a.slot_type[6 * i + s], pair, o, a.prob + i * a.K * 4, kk, intent);
        const int64_t src = (((i * a.K + kk) * 4 + intent) * (int64_t)a.L + st) * 3;
        for (int d = 0; d < 3; d++) {
            a.dpos[e * 3 + d] = a.pred_pos[src + d];
            a.dsize[e * 3 + d] = a.pred_size[src + d];
        }
    }
}

struct CommitArgs {
    int64_t I, n;
    int32_t N;
    const ShapeDev *sh;
    const int8_t *branch;
    const int32_t *shp, *slot_row, *best;
    const double *const *x_cand;
    double *plan_x, *plan_states;
    int32_t *prev_count;
    int8_t *first_time, *valid;
};

// every plan into the planner state (:629-639 / :653-657): the selected candidate of a fan-out
// instance, the single solve when solveTraj succeeded; an instance without a plan keeps its state
__global__ __launch_bounds__(64) void k_commit(CommitArgs a) {
    for (int64_t i = blockIdx.x; i < a.I; i += gridDim.x) {
        const double *src = nullptr;
        if (a.branch[i] == IMPC_REPLAN_FANOUT) {
            const int b = a.best[i];
            if (b >= 0) src = a.x_cand[6 * i + b];
        } else {
            const int k = a.shp[i];
            const int64_t r = a.slot_row[6 * i];
            if (impc_lib::solve_traj_ok(a.sh[k].info[r])) src = a.sh[k].x + r * a.n;
        }
        if (src) {
            for (int64_t e = threadIdx.x; e < a.n; e += blockDim.x) {
                const double v = src[e];
                a.plan_x[i * a.n + e] = v;
                if (e < (int64_t)8 * a.N) a.plan_states[i * (int64_t)a.N * 8 + e] = v;
            }
        }
        if (threadIdx.x == 0) {
            if (src) {
                a.prev_count[i] = a.N;
                a.first_time[i] = 0;
            }
            a.valid[i] = src ? 1 : 0;
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

// one QP shape of the replan (k dynamic- and nst static-obstacle rows per stage): its solver batch
// and on-device builder
struct Shape {
    int32_t k = 0, nst = 0;
    int64_t cap = 0;
    impc_qp_dims dm{};
    impc_batch batch = nullptr;
    impc_mpc_builder bld = nullptr;
    ShapeDev dev{};
};

}  // namespace impc_rp

using namespace impc_rp;

struct impc_replan_s {
    impc_ctx ctx = nullptr;
    impc_replan_config cfg{};
    int64_t I = 0, n = 0, rows = 0;
    int32_t N = 0, K = 0, L = 0, S = 0;
    Arena mem;
    // planner state
    double *plan_x = nullptr, *plan_states = nullptr;
    int32_t *prev_count = nullptr;
    int8_t *first_time = nullptr, *valid = nullptr, *zeros8 = nullptr;
    // rows of the shapes and per-instance outputs
    int8_t *branch = nullptr, *row_code = nullptr;
    int32_t *row_inst = nullptr, *num_obs = nullptr, *shp = nullptr, *slot_row = nullptr, *slot_type = nullptr;
    int32_t *best = nullptr, *ob = nullptr, *ctype = nullptr, *cslot = nullptr, *issued = nullptr;
    int64_t *cnt = nullptr, *solve = nullptr;
    unsigned long long *clk = nullptr;
    double *cprob = nullptr;
    ShapeDev *d_sh = nullptr;
    // selection
    const double **x_cand = nullptr;
    int32_t *dyn_count = nullptr, *best_pos = nullptr;
    double *dyn_pos = nullptr, *dyn_size = nullptr, *scores = nullptr, *weighted = nullptr;
    int8_t *cvalid = nullptr;
    int32_t nst = 0;        // static obstacles per instance (cfg.num_static)
    std::vector<Shape> sh;  // S = K + 2 shapes by dynamic-obstacle count, + the first plans' with statics
    std::vector<impc_batch> group;
    impc_replan_stats stats{};
    bool ran = false;
    double last_limit = 0.0;
    double last_total_s = 0.0;
};

namespace {

int fail(int code, const char *msg) { return impc_lib::set_error(code, msg); }

int make_shape(impc_replan rp, Shape &s, int32_t k, int32_t nst, int64_t cap) {
    s.k = k, s.nst = nst, s.cap = cap;
    RP_TRY(impc_mpc_dims(&rp->cfg.mpc, nst, k, &s.dm));
    std::vector<int64_t> Pp(s.dm.n + 1), Pi(std::max<int64_t>(s.dm.nnzP, 1)), Ap(s.dm.n + 1), Ai(s.dm.nnzA);
    RP_TRY(impc_mpc_build_pattern(&rp->cfg.mpc, nst, k, Pp.data(), Pi.data(), Ap.data(), Ai.data()));
    RP_TRY(impc_batch_create(rp->ctx, s.dm.n, s.dm.m, Pp.data(), Pi.data(), Ap.data(), Ai.data(), cap, &s.batch));
    RP_TRY(impc_batch_set_settings(s.batch, &rp->cfg.settings));
    if (rp->cfg.queue_order == IMPC_QUEUE_LONGEST_FIRST) {
        // impc.scenarios.queue_weight: ||q||_inf / (position weight (N - 1)) weighed 1:10
        const double qw = 1.0 / (10.0 * (rp->N - 1) * rp->cfg.mpc.position_weight);
        RP_TRY(impc_batch_set_queue_order(s.batch, IMPC_QUEUE_LONGEST_FIRST, qw));
    }
    RP_TRY(impc_batch_set_kernel(s.batch, IMPC_KERNEL_STRUCTURED));
    RP_TRY(impc_mpc_builder_create(rp->ctx, &rp->cfg.mpc, nst, k, rp->L, &s.bld));
    impc_lib::BatchInputs bi{};
    RP_TRY(impc_lib::batch_inputs_view(s.batch, &bi));
    double *x = nullptr;
    impc_info *info = nullptr;
    RP_TRY(impc_batch_device_results(s.batch, &x, nullptr, &info));
    s.dev.xws = bi.xws;
    s.dev.x = x;
    s.dev.info = info;
    RP_TRY(impc_lib::batch_tlim_device(s.batch, &s.dev.tlim));
    RP_TRY(rp->mem.get((size_t)std::max<int64_t>(1, cap * k), &s.dev.osrc));
    return IMPC_OK;
}

void free_shape(Shape &s) {
    if (s.batch) (void)impc_batch_destroy(s.batch);
    if (s.bld) (void)impc_mpc_builder_destroy(s.bld);
    s.batch = nullptr;
    s.bld = nullptr;
}

unsigned grid_for(impc_replan rp, int64_t work, int per = 256) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + per - 1) / per, (int64_t)impc_lib::num_cu(rp->ctx) * 8));
}

}  // namespace

extern "C" {

int impc_replan_create(impc_ctx ctx, const impc_replan_config *cfg, impc_replan *out) {
    if (!ctx || !cfg || !out) return fail(IMPC_INVALID_ARGUMENT, "replan: null context, config or output");
    *out = nullptr;
    const int64_t I = cfg->instances;
    const int32_t N = cfg->mpc.horizon, K = cfg->num_obstacles, L = cfg->pred_len;
    if (I < 1 || I > ((int64_t)1 << 24) || N < 2 || K < 1 || K > kMaxObstacles || L < 1 || cfg->num_static < 0 ||
        cfg->num_static > kMaxObstacles)
        return fail(IMPC_INVALID_ARGUMENT, "replan: 1 <= instances <= 2^24, horizon >= 2, 1 <= num_obstacles <= 30, "
                                           "pred_len >= 1, 0 <= num_static <= 30");
    if (cfg->mpc.num_half_space != 0)
        return fail(IMPC_UNSUPPORTED, "replan: the live planner path has no FOV half-spaces (num_half_space = 0)");
    if (cfg->queue_order != IMPC_QUEUE_FIFO && cfg->queue_order != IMPC_QUEUE_LONGEST_FIRST)
        return fail(IMPC_INVALID_ARGUMENT, "replan: unknown queue order");
    RP_HIP(hipSetDevice(impc_lib::device(ctx)));
    std::unique_ptr<impc_replan_s> rp(new impc_replan_s());
    rp->ctx = ctx;
    rp->cfg = *cfg;
    rp->I = I, rp->N = N, rp->K = K, rp->L = L, rp->nst = cfg->num_static;
    rp->S = K + 2 + (rp->nst > 0 ? 1 : 0);
    rp->n = 13 * (int64_t)N - 5;
    rp->rows = shape_base(I, K, rp->S - 1) + shape_cap(I, K, rp->S - 1);
    const int64_t n = rp->n, S = rp->S;
    Arena &a = rp->mem;
    int rc = IMPC_OK;
    auto cleanup = [&]() {
        for (Shape &s : rp->sh) free_shape(s);
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
    RP_CK(a.get((size_t)rp->rows, &rp->row_inst));
    RP_CK(a.get((size_t)rp->rows, &rp->row_code));
    RP_CK(a.get((size_t)I, &rp->num_obs));
    RP_CK(a.get((size_t)I, &rp->shp));
    RP_CK(a.get((size_t)(6 * I), &rp->slot_row));
    RP_CK(a.get((size_t)(6 * I), &rp->slot_type));
    RP_CK(a.get((size_t)I, &rp->best));
    RP_CK(a.get((size_t)I, &rp->ob));
    RP_CK(a.get((size_t)(6 * I), &rp->ctype));
    RP_CK(a.get((size_t)(6 * I), &rp->cslot));
    RP_CK(a.get((size_t)1, &rp->issued));
    RP_CK(a.get((size_t)(2 * S + 3), &rp->cnt));
    RP_CK(a.get((size_t)S, &rp->solve));
    RP_CK(a.get((size_t)2, &rp->clk));
    RP_CK(a.get((size_t)(4 * I), &rp->cprob));
    RP_CK(a.get((size_t)S, &rp->d_sh));
    RP_CK(a.get((size_t)(6 * I), &rp->x_cand));
    RP_CK(a.get((size_t)(6 * I), &rp->dyn_count));
    RP_CK(a.get((size_t)I, &rp->best_pos));
    RP_CK(a.get((size_t)(I * 6 * (K + 1) * L * 3), &rp->dyn_pos));
    RP_CK(a.get((size_t)(I * 6 * (K + 1) * L * 3), &rp->dyn_size));
    RP_CK(a.get((size_t)(I * 6 * 3), &rp->scores));
    RP_CK(a.get((size_t)(I * 6), &rp->weighted));
    RP_CK(a.get((size_t)(I * 6), &rp->cvalid));
    hipStream_t st = impc_lib::stream(ctx);
    if (hipMemsetAsync(rp->zeros8, 0, (size_t)I, st) != hipSuccess ||
        hipMemsetAsync(rp->valid, 0, (size_t)I, st) != hipSuccess ||
        hipMemsetAsync(rp->cnt, 0, sizeof(int64_t) * (size_t)(2 * S + 3), st) != hipSuccess ||
        hipMemsetAsync(rp->solve, 0, sizeof(int64_t) * (size_t)S, st) != hipSuccess) {
        cleanup();
        return fail(IMPC_DEVICE_ERROR, "replan: memset");
    }
    // one solver batch per shape, each reading its QP count from device memory
    rp->sh.resize((size_t)S);
    std::vector<ShapeDev> hdev((size_t)S);
    for (int32_t k = 0; k < S; k++) {
        Shape &s = rp->sh[(size_t)k];
        RP_CK(make_shape(rp.get(), s, shape_dyn(K, k), k <= K + 1 ? rp->nst : 0, shape_cap(I, K, k)));
        RP_CK(impc_lib::batch_set_active_device(s.batch, rp->solve + k));
        hdev[(size_t)k] = s.dev;
        rp->group.push_back(s.batch);
    }
    RP_CK(impc_copy_to_device(ctx, rp->d_sh, hdev.data(), (int64_t)(sizeof(ShapeDev) * hdev.size())));
    {  // the row scan's counters: (2 S + 3) x (lanes + wave totals) int32 of LDS
        const size_t lds = sizeof(int32_t) * (size_t)(2 * S + 3) * (kPlanLanes + kPlanLanes / 64);
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute((const void *)k_plan_rows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
                hipSuccess) {
            cleanup();
            return fail(IMPC_DEVICE_ERROR, "replan: LDS of the row scan");
        }
    }
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
    if (rp->nst > 0 && (!in->st_centroid || !in->st_size || !in->st_yaw))
        return fail(IMPC_INVALID_ARGUMENT, "replan: num_static > 0 needs st_centroid, st_size, st_yaw");
    impc_ctx ctx = rp->ctx;
    RP_HIP(hipSetDevice(impc_lib::device(ctx)));
    hipStream_t st = impc_lib::stream(ctx);
    RP_TRY(impc_lib::order_after_all(ctx));
    const int64_t I = rp->I, n = rp->n;
    const int32_t N = rp->N, K = rp->K, L = rp->L, S = rp->S;

    // ---- the branch and the rows of every instance (:593-606)
    PlanArgs pa{I,
                K,
                S,
                rp->nst > 0 ? K + 2 : 0,
                Decide{rp->first_time, in->has_pred, in->num_pred, in->cur_count, K, in->cur_size ? 1 : 0},
                rp->branch,
                rp->num_obs,
                rp->shp,
                rp->slot_row,
                rp->best,
                rp->row_inst,
                rp->row_code,
                rp->cnt,
                rp->clk};
    const size_t lds = sizeof(int32_t) * (size_t)(2 * S + 3) * (kPlanLanes + kPlanLanes / 64);
    hipLaunchKernelGGL(k_plan_rows, dim3(1), dim3(kPlanLanes), lds, st, pa);
    RP_HIP(hipGetLastError());
    // ---- the fan-out's closest obstacle and candidate order
    PickArgs pk{I, K, N, rp->branch, rp->num_obs, in->pos, rp->plan_states, in->dyn_cur, in->prob, rp->prev_count,
                rp->ob, rp->ctype, rp->cslot, rp->slot_type, rp->cprob};
    hipLaunchKernelGGL(k_pick, dim3((unsigned)((I + 63) / 64)), dim3(64), 0, st, pk);
    RP_HIP(hipGetLastError());
    // ---- warm starts, time limits, obstacle sources; the assembly of every shape in place
    // (timeLimit = max(solverTimeLimit_ - t, solverTimeLimit_) = solverTimeLimit_ for t >= 0, :614)
    const double tl = in->solver_time_limit > 0.0 ? in->solver_time_limit : rp->cfg.settings.time_limit;
    PrepArgs pp{I, n, rp->rows, K, L, S, rp->cnt, rp->d_sh, rp->row_inst, rp->ob, rp->slot_type, rp->row_code,
                rp->first_time, rp->plan_x, in->prob, tl};
    hipLaunchKernelGGL(k_prep, dim3(grid_for(rp, rp->rows, 1)), dim3(64), 0, st, pp);
    RP_HIP(hipGetLastError());
    for (int32_t k = 0; k < S; k++) {
        Shape &s = rp->sh[(size_t)k];
        impc_lib::BatchInputs bi{};
        RP_TRY(impc_lib::batch_inputs_begin(s.batch, &bi));
        const bool stat = s.nst > 0;
        RP_TRY(impc_lib::build_rows(s.bld, s.cap, rp->cnt + S + k, rp->row_inst + shape_base(I, K, k), s.dev.osrc,
                                    in->pos, in->vel, in->xref, rp->plan_states, in->pred_pos, in->pred_size,
                                    in->dyn_cur, in->cur_size, stat ? in->st_centroid : nullptr,
                                    stat ? in->st_size : nullptr, stat ? in->st_yaw : nullptr, bi, st));
        RP_TRY(impc_lib::batch_inputs_end(s.batch, true));
    }
    // ---- the issue cut-off on the device clock; ONE grouped solve over every shape
    hipLaunchKernelGGL(k_issue, dim3(1), dim3(64), 0, st, S, rp->cnt, rp->solve, rp->clk, rp->issued, in->elapsed_s,
                       impc_lib::tick_s(ctx), rp->cfg.issue_cutoff_s);
    RP_HIP(hipGetLastError());
    RP_TRY(impc_batch_solve_group(rp->group.data(), (int)rp->group.size(), nullptr));
    // ---- candidate validity, selection, commit
    CandArgs ca{I, n, K, L, rp->d_sh, rp->branch, rp->num_obs, rp->slot_row, rp->cslot, rp->slot_type, rp->ob,
                rp->issued, in->pred_pos, in->pred_size, in->prob, rp->x_cand, rp->dyn_count, rp->cvalid, rp->dyn_pos,
                rp->dyn_size};
    hipLaunchKernelGGL(k_cand, dim3(grid_for(rp, 6 * I)), dim3(256), 0, st, ca);
    hipLaunchKernelGGL(k_sel_sets, dim3(grid_for(rp, I * 6 * (K + 1) * L)), dim3(256), 0, st, ca);
    RP_HIP(hipGetLastError());
    impc_select_params sp{};
    sp.horizon = N, sp.num_candidates = 6, sp.max_dynamic = K + 1, sp.pred_len = L;
    sp.num_static = rp->nst, sp.prev_len = N;  // getTrajectoryScore's staticObstacles (:620)
    sp.dynamic_safety_dist = rp->cfg.mpc.dynamic_safety_dist;
    sp.static_safety_dist = rp->cfg.mpc.static_safety_dist;
    RP_TRY(impc_select_best_device(ctx, &sp, I, rp->x_cand, rp->cvalid, rp->zeros8, rp->plan_states, rp->prev_count,
                                   in->xref, rp->nst ? in->st_centroid : nullptr, rp->nst ? in->st_size : nullptr,
                                   rp->dyn_count, rp->dyn_pos, rp->dyn_size, rp->cprob,
                                   rp->best, rp->best_pos, rp->scores, rp->weighted, nullptr));
    CommitArgs cm{I, n, N, rp->d_sh, rp->branch, rp->shp, rp->slot_row, rp->best, rp->x_cand, rp->plan_x,
                  rp->plan_states, rp->prev_count, rp->first_time, rp->valid};
    hipLaunchKernelGGL(k_commit, dim3(grid_for(rp, I, 1)), dim3(64), 0, st, cm);
    RP_HIP(hipGetLastError());
    rp->ran = true;
    rp->last_limit = tl;
    rp->last_total_s = std::chrono::duration<double>(clk::now() - t_entry).count();
    return IMPC_OK;
}

int impc_replan_get_stats(impc_replan rp, impc_replan_stats *out) {
    if (!rp || !out) return fail(IMPC_INVALID_ARGUMENT, "replan: null object or output");
    std::memset(out, 0, sizeof(*out));
    if (!rp->ran) return IMPC_OK;
    RP_TRY(impc_ctx_synchronize(rp->ctx));
    const int32_t S = rp->S;
    std::vector<int64_t> c((size_t)(2 * S + 3));
    unsigned long long ck[2];
    int32_t iss = 0;
    RP_TRY(impc_copy_to_host(rp->ctx, c.data(), rp->cnt, (int64_t)(sizeof(int64_t) * c.size())));
    RP_TRY(impc_copy_to_host(rp->ctx, ck, rp->clk, (int64_t)sizeof(ck)));
    RP_TRY(impc_copy_to_host(rp->ctx, &iss, rp->issued, (int64_t)sizeof(iss)));
    out->fanout = c[(size_t)(2 * S + IMPC_REPLAN_FANOUT)];
    out->single_first = c[(size_t)(2 * S + IMPC_REPLAN_SINGLE_FIRST)];
    out->single_current = c[(size_t)(2 * S + IMPC_REPLAN_SINGLE_CURRENT)];
    out->issued = iss;
    out->time_limit = rp->last_limit;
    out->stage_s = (double)(ck[1] - ck[0]) * impc_lib::tick_s(rp->ctx);
    out->total_s = rp->last_total_s;
    return IMPC_OK;
}

int impc_replan_view_device(impc_replan rp, impc_replan_view *out) {
    if (!rp || !out) return fail(IMPC_INVALID_ARGUMENT, "replan: null object or output");
    out->plan_x = rp->plan_x, out->plan_states = rp->plan_states, out->prev_count = rp->prev_count;
    out->first_time = rp->first_time, out->valid = rp->valid, out->branch = rp->branch;
    out->best_cand = rp->best, out->ob_idx = rp->ob, out->cand_type = rp->ctype, out->cand_slot = rp->cslot;
    out->num_obs = rp->num_obs, out->slot_row = rp->slot_row, out->shape = rp->shp;
    return IMPC_OK;
}

int impc_replan_shape(impc_replan rp, int32_t obstacles, impc_batch *batch, int64_t *count, const int32_t **row_inst,
                      const int8_t **row_code, const double **Px, const double **q, const double **Ax,
                      const double **l, const double **u) {
    if (!rp || obstacles < 0 || obstacles >= rp->S)
        return fail(IMPC_INVALID_ARGUMENT, "replan: shape must be in 0 .. num_obstacles + 1 (+ 2 with num_static)");
    const Shape &s = rp->sh[(size_t)obstacles];
    int64_t c = 0;
    if (rp->ran) {
        RP_TRY(impc_ctx_synchronize(rp->ctx));
        RP_TRY(impc_copy_to_host(rp->ctx, &c, rp->solve + obstacles, (int64_t)sizeof(c)));
    }
    if (batch) *batch = s.batch;
    if (count) *count = c;
    const int64_t base = shape_base(rp->I, rp->K, obstacles);
    if (row_inst) *row_inst = rp->row_inst + base;
    if (row_code) *row_code = rp->row_code + base;
    impc_lib::BatchInputs bi{};
    RP_TRY(impc_lib::batch_inputs_view(s.batch, &bi));  // the inputs of the last assembly
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
