// mpc_qp.cpp -- batched restatement of mpcPlanner's MPC -> QP assembly (host C++).
//
// Reference: trajectory_planner/include/trajectory_planner/mpcPlanner.cpp
//   updateObstacleParam :1148-1197, setDynamicsMatrices :891-901, setInequalityConstraints
//   :904-921, setWeightMatrices :925-931, castMPCToQPHessian :932-951, castMPCToQPGradient
//   :952-966, castMPCToQPConstraintMatrix :984-1072, castMPCToQPConstraintVectors :1074-1146.
//
// The reference inserts entries one by one into an Eigen::SparseMatrix and OsqpEigen copies it
// to CSC with rows sorted inside each column and explicitly inserted zeros kept
// (SparseMatrixHelper.tpp:11-58).  Here the insertion sequence is generated once per QP shape,
// sorted to CSC order once (the shared pattern), and every QP's values are scattered straight
// into their CSC slots.  Arithmetic is written in the reference's evaluation order so the
// values are bit-identical to the reference expressions (build with -ffp-contract=off).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/impc_mpc.h"
#include "mpc_qp_internal.hpp"

namespace {

constexpr int kNx = 8;  // mpcPlanner.h:42 numStates
constexpr int kNu = 5;  // mpcPlanner.h:43 numControls

struct Shape {
    int N, W, S, Kd, K, H;
    int64_t n, m;
    int64_t off_box, off_half, off_obs;  // row offsets of the constraint blocks
};

bool make_shape(const impc_mpc_params *p, int32_t ns, int32_t nd, Shape *s) {
    if (!p || p->horizon < 2 || ns < 0 || nd < 0) return false;
    if (p->num_half_space != 0 && p->num_half_space != 2) return false;
    s->N = p->horizon;
    s->W = p->horizon - 1;
    s->S = ns;
    s->Kd = nd;
    s->K = ns + nd;
    s->H = p->num_half_space;
    s->n = (int64_t)kNx * s->N + (int64_t)kNu * s->W;
    s->off_box = (int64_t)kNx * s->N;
    s->off_half = s->off_box + s->n;
    s->off_obs = s->off_half + (int64_t)s->H * s->W;
    s->m = s->off_obs + (int64_t)s->K * s->W;
    return true;
}

// setDynamicsMatrices (:891-901), evaluated in double exactly as the Eigen expressions.
void dynamics(double ts, double A[kNx][kNx], double B[kNx][kNu]) {
    for (int r = 0; r < kNx; r++) {
        for (int c = 0; c < kNx; c++) A[r][c] = 0.0;
        for (int c = 0; c < kNu; c++) B[r][c] = 0.0;
    }
    for (int d = 0; d < 3; d++) {
        A[d][d] = 1.0;
        A[d][3 + d] = 1.0 * ts;  // Identity() * ts
        A[3 + d][3 + d] = 1.0;
        B[d][d] = ((1.0 * 1) / 2) * std::pow(ts, 2);  // Identity() * 1/2 * pow(ts, 2)
        B[3 + d][d] = 1.0 * ts;
    }
    B[6][3] = 1.0;  // B.block(6, 3, 2, 2) = Identity()
    B[7][4] = 1.0;
}

struct Trip {
    int64_t row, col;
};

// Insertion sequence of castMPCToQPConstraintMatrix (:994-1071); values produced separately.
void a_insertions(const impc_mpc_params *p, const Shape &s, std::vector<Trip> &t) {
    double A[kNx][kNx], B[kNx][kNu];
    dynamics(p->ts, A, B);
    t.clear();
    for (int64_t i = 0; i < (int64_t)kNx * s.N; i++) t.push_back({i, i});
    for (int i = 0; i < s.W; i++)
        for (int j = 0; j < kNx; j++)
            for (int k = 0; k < kNx; k++)
                if ((float)A[j][k] != 0) t.push_back({(int64_t)kNx * (i + 1) + j, (int64_t)kNx * i + k});
    for (int i = 0; i < s.W; i++)
        for (int j = 0; j < kNx; j++)
            for (int k = 0; k < kNu; k++)
                if ((float)B[j][k] != 0)
                    t.push_back({(int64_t)kNx * (i + 1) + j, (int64_t)kNu * i + k + (int64_t)kNx * s.N});
    for (int64_t i = 0; i < s.n; i++) t.push_back({i + s.off_box, i});
    if (s.H) {
        for (int i = 0; i < s.W; i++) {
            int64_t r0 = (int64_t)s.H * i + 0 + s.off_half, r1 = (int64_t)s.H * i + 1 + s.off_half;
            t.push_back({r0, (int64_t)kNx * i + 0});
            t.push_back({r0, (int64_t)kNx * i + 1});
            t.push_back({r1, (int64_t)kNx * i + 0});
            t.push_back({r1, (int64_t)kNx * i + 1});
        }
    }
    // isDyamic (:1151-1195): dynamic obstacles flagged 1, then flags [0, S) overwritten with 0
    // (the static loop indexes isDyamic by the static index i, not i + numDynamicOb).
    std::vector<int> is_dyn(s.K, 0);
    for (int i = 0; i < s.Kd; i++) is_dyn[i] = 1;
    for (int i = 0; i < s.S; i++) is_dyn[i] = 0;
    for (int i = 0; i < s.W; i++)
        for (int j = 0; j < s.K; j++) {
            int64_t row = (int64_t)i * s.K + j + s.off_obs;
            t.push_back({row, (int64_t)kNx * i});
            t.push_back({row, (int64_t)kNx * i + 1});
            t.push_back({row, (int64_t)kNx * i + 2});
            t.push_back({row, (int64_t)kNx * s.N + (int64_t)kNu * i + (is_dyn[j] ? 3 : 4)});
        }
}

// CSC order of the insertion sequence: slot[k] = CSC position of the k-th inserted entry.
void csc_from_insertions(int64_t ncols, const std::vector<Trip> &t, int64_t *colptr, int64_t *rowind,
                         std::vector<int64_t> &slot) {
    std::vector<int64_t> order(t.size());
    for (size_t k = 0; k < t.size(); k++) order[k] = (int64_t)k;
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
        return t[a].col != t[b].col ? t[a].col < t[b].col : t[a].row < t[b].row;
    });
    slot.assign(t.size(), 0);
    std::vector<int64_t> cnt(ncols + 1, 0);
    for (const Trip &e : t) cnt[e.col + 1]++;
    for (int64_t c = 0; c < ncols; c++) cnt[c + 1] += cnt[c];
    if (colptr) std::memcpy(colptr, cnt.data(), sizeof(int64_t) * (ncols + 1));
    for (size_t pos = 0; pos < order.size(); pos++) {
        slot[order[pos]] = (int64_t)pos;
        if (rowind) rowind[pos] = t[order[pos]].row;
    }
}

// castMPCToQPHessian (:932-951): diagonal, float-rounded, zero entries skipped, R indexed by
// the GLOBAL variable index modulo numControls (:945).
void hessian_diag(const impc_mpc_params *p, const Shape &s, std::vector<int64_t> &cols, std::vector<double> &vals) {
    const double Q[kNx] = {p->position_weight, p->position_weight, p->position_weight, p->velocity_weight,
                           p->velocity_weight, p->velocity_weight, 100.0, 1000.0};
    const double R[kNu] = {p->acceleration_weight, p->acceleration_weight, p->acceleration_weight, 1.0, 1.0};
    cols.clear();
    vals.clear();
    for (int64_t i = 0; i < s.n; i++) {
        float value = i < (int64_t)kNx * s.N ? (float)Q[i % kNx] : (float)R[i % kNu];
        if (value != 0) {
            cols.push_back(i);
            vals.push_back((double)value);
        }
    }
}

struct Ellipsoid {
    double ox, oy, oz, sx, sy, sz, yaw;
};

}  // namespace

extern "C" int impc_mpc_dims(const impc_mpc_params *p, int32_t num_static, int32_t num_dynamic, impc_qp_dims *out) {
    Shape s;
    if (!out || !make_shape(p, num_static, num_dynamic, &s)) return 1;
    std::vector<Trip> t;
    a_insertions(p, s, t);
    std::vector<int64_t> pc;
    std::vector<double> pv;
    hessian_diag(p, s, pc, pv);
    out->n = s.n;
    out->m = s.m;
    out->nnzP = (int64_t)pc.size();
    out->nnzA = (int64_t)t.size();
    return 0;
}

extern "C" int impc_mpc_build_pattern(const impc_mpc_params *p, int32_t num_static, int32_t num_dynamic, int64_t *Pp,
                                      int64_t *Pi, int64_t *Ap, int64_t *Ai) {
    Shape s;
    if (!make_shape(p, num_static, num_dynamic, &s)) return 1;
    std::vector<int64_t> pc;
    std::vector<double> pv;
    hessian_diag(p, s, pc, pv);
    if (Pp) {
        size_t k = 0;
        for (int64_t j = 0; j < s.n; j++) {
            Pp[j] = (int64_t)k;
            if (k < pc.size() && pc[k] == j) {
                if (Pi) Pi[k] = j;
                k++;
            }
        }
        Pp[s.n] = (int64_t)k;
    }
    std::vector<Trip> t;
    a_insertions(p, s, t);
    std::vector<int64_t> slot;
    csc_from_insertions(s.n, t, Ap, Ai, slot);
    return 0;
}

extern "C" int impc_mpc_build_values(const impc_mpc_params *p, int64_t nb, const double *curr_pos,
                                     const double *curr_vel, const double *xref, const double *lin_states,
                                     int32_t num_static, const double *st_centroid, const double *st_size,
                                     const double *st_yaw, int32_t num_dynamic, int32_t pred_len,
                                     const double *dyn_pos, const double *dyn_size, double *Px, double *q, double *Ax,
                                     double *l, double *u) {
    Shape s;
    if (!make_shape(p, num_static, num_dynamic, &s) || nb < 0) return 1;
    if (num_dynamic > 0 && (pred_len < 1 || !dyn_pos || !dyn_size)) return 2;
    if (num_static > 0 && (!st_centroid || !st_size || !st_yaw)) return 2;
    if (!curr_pos || !curr_vel || !xref) return 2;
    const int N = s.N, W = s.W, K = s.K;
    const int64_t n = s.n, m = s.m;

    std::vector<Trip> t;
    a_insertions(p, s, t);
    const int64_t nnzA = (int64_t)t.size();
    std::vector<int64_t> slot;
    std::vector<int64_t> colptr(n + 1);
    csc_from_insertions(n, t, colptr.data(), nullptr, slot);
    std::vector<int64_t> pc;
    std::vector<double> pv;
    hessian_diag(p, s, pc, pv);
    const int64_t nnzP = (int64_t)pc.size();

    double Ad[kNx][kNx], Bd[kNx][kNu];
    dynamics(p->ts, Ad, Bd);
    // setInequalityConstraints (:904-921)
    const double xMin[kNx] = {-INFINITY, p->y_range_min, p->z_range_min, -p->max_vel, -p->max_vel, -p->max_vel,
                              -INFINITY, -INFINITY};
    const double xMax[kNx] = {INFINITY, p->y_range_max, p->z_range_max, p->max_vel, p->max_vel, p->max_vel,
                              INFINITY, INFINITY};
    const double skslimit = 1.0 - std::pow((1 - p->static_slack), 2);
    const double skdlimit = 1.0 - std::pow((1 - p->dynamic_slack), 2);
    const double uMin[kNu] = {-p->max_acc, -p->max_acc, -p->max_acc, 0.0, 0.0};
    const double uMax[kNu] = {p->max_acc, p->max_acc, p->max_acc, skdlimit, skslimit};
    const double Qd[kNx] = {p->position_weight, p->position_weight, p->position_weight, p->velocity_weight,
                            p->velocity_weight, p->velocity_weight, 100.0, 1000.0};

    std::vector<double> tv(nnzA);
    std::vector<Ellipsoid> ob((size_t)W * K);
    for (int64_t b = 0; b < nb; b++) {
        const double *cp = curr_pos + 3 * b, *cv = curr_vel + 3 * b;
        const double *xr = xref + (int64_t)N * kNx * b;
        const double *ls = lin_states ? lin_states + (int64_t)N * kNx * b : nullptr;
        // ---- updateObstacleParam (:1148-1197): dynamic obstacles first, then static
        for (int j = 0; j < W; j++) {
            for (int i = 0; i < s.Kd; i++) {
                int jj = j < pred_len ? j : pred_len - 1;  // .back() when the prediction is shorter
                const double *pp = dyn_pos + (((int64_t)b * s.Kd + i) * pred_len + jj) * 3;
                const double *ps = dyn_size + (((int64_t)b * s.Kd + i) * pred_len + jj) * 3;
                Ellipsoid &e = ob[(size_t)j * K + i];
                e.ox = pp[0];
                e.oy = pp[1];
                e.oz = pp[2];
                e.sx = ps[0] / 2 + p->dynamic_safety_dist;
                e.sy = ps[1] / 2 + p->dynamic_safety_dist;
                e.sz = ps[2] / 2 + p->dynamic_safety_dist;
                e.yaw = 0.0;
            }
            for (int i = 0; i < s.S; i++) {
                const double *c = st_centroid + ((int64_t)b * s.S + i) * 3;
                const double *z = st_size + ((int64_t)b * s.S + i) * 3;
                Ellipsoid &e = ob[(size_t)j * K + s.Kd + i];
                e.ox = c[0];
                e.oy = c[1];
                e.oz = c[2];
                e.sx = z[0] / 2 + p->static_safety_dist;
                e.sy = z[1] / 2 + p->static_safety_dist;
                e.sz = z[2] / 2 + p->static_safety_dist;
                e.yaw = st_yaw[(int64_t)b * s.S + i];
            }
        }
        // ---- P values (:932-951)
        if (Px)
            for (int64_t k = 0; k < nnzP; k++) Px[b * nnzP + k] = pv[k];
        // ---- q (:952-966): Q * (-xRef[i])
        if (q) {
            double *qb = q + b * n;
            for (int64_t k = 0; k < n; k++) qb[k] = 0.0;
            for (int i = 0; i < N; i++)
                for (int j = 0; j < kNx; j++) qb[(int64_t)i * kNx + j] = Qd[j] * (-xr[(int64_t)i * kNx + j]);
        }
        // ---- A values in insertion order (:994-1071)
        size_t k = 0;
        for (int64_t i = 0; i < (int64_t)kNx * N; i++) tv[k++] = -1;
        for (int i = 0; i < W; i++)
            for (int j = 0; j < kNx; j++)
                for (int c = 0; c < kNx; c++) {
                    float value = (float)Ad[j][c];
                    if (value != 0) tv[k++] = value;
                }
        for (int i = 0; i < W; i++)
            for (int j = 0; j < kNx; j++)
                for (int c = 0; c < kNu; c++) {
                    float value = (float)Bd[j][c];
                    if (value != 0) tv[k++] = value;
                }
        for (int64_t i = 0; i < n; i++) tv[k++] = 1;
        if (s.H)
            for (int i = 0; i < W; i++) {
                tv[k++] = p->half_max[0];
                tv[k++] = p->half_max[1];
                tv[k++] = p->half_min[0];
                tv[k++] = p->half_min[1];
            }
        double *lb = l ? l + b * m : nullptr;
        double *ub = u ? u + b * m : nullptr;
        for (int i = 0; i < W; i++) {
            double cx, cy, cz;
            if (ls) {
                cx = ls[(int64_t)i * kNx + 0];
                cy = ls[(int64_t)i * kNx + 1];
                cz = ls[(int64_t)i * kNx + 2];
            } else {
                cx = cp[0];
                cy = cp[1];
                cz = cp[2];
            }
            for (int j = 0; j < K; j++) {
                const Ellipsoid &e = ob[(size_t)i * K + j];
                double fxx = 2 * ((cx - e.ox) * std::cos(e.yaw) + (cy - e.oy) * std::sin(e.yaw)) / std::pow(e.sx, 2) *
                                 std::cos(e.yaw) +
                             2 * (-(cx - e.ox) * std::sin(e.yaw) + (cy - e.oy) * std::cos(e.yaw)) / std::pow(e.sy, 2) *
                                 (-std::sin(e.yaw));
                double fyy = 2 * ((cx - e.ox) * std::cos(e.yaw) + (cy - e.oy) * std::sin(e.yaw)) / std::pow(e.sx, 2) *
                                 std::sin(e.yaw) +
                             2 * (-(cx - e.ox) * std::sin(e.yaw) + (cy - e.oy) * std::cos(e.yaw)) / std::pow(e.sy, 2) *
                                 (std::cos(e.yaw));
                double fzz = 2 * ((cz - e.oz)) / std::pow(e.sz, 2);
                tv[k++] = fxx;
                tv[k++] = fyy;
                tv[k++] = fzz;
                tv[k++] = -1;
                if (lb) {
                    double fxyz =
                        std::pow((cx - e.ox) * std::cos(e.yaw) + (cy - e.oy) * std::sin(e.yaw), 2) / std::pow(e.sx, 2) +
                        std::pow(-(cx - e.ox) * std::sin(e.yaw) + (cy - e.oy) * std::cos(e.yaw), 2) / std::pow(e.sy, 2) +
                        std::pow((cz - e.oz), 2) / std::pow(e.sz, 2);
                    lb[s.off_obs + (int64_t)i * K + j] = 1 - fxyz + fxx * cx + fyy * cy + fzz * cz;
                }
                if (ub) ub[s.off_obs + (int64_t)i * K + j] = INFINITY;
            }
        }
        if (Ax) {
            double *ab = Ax + b * nnzA;
            for (int64_t e = 0; e < nnzA; e++) ab[slot[e]] = tv[e];
        }
        // ---- l, u (:1074-1146)
        if (lb && ub) {
            const double x0[kNx] = {cp[0], cp[1], cp[2], cv[0], cv[1], cv[2], 0.0, 0.0};
            for (int64_t r = 0; r < (int64_t)kNx * N; r++) lb[r] = 0.0;
            for (int d = 0; d < kNx; d++) lb[d] = -x0[d];
            for (int64_t r = 0; r < (int64_t)kNx * N; r++) ub[r] = lb[r];
            for (int i = 0; i < N; i++)
                for (int d = 0; d < kNx; d++) {
                    lb[s.off_box + (int64_t)kNx * i + d] = xMin[d];
                    ub[s.off_box + (int64_t)kNx * i + d] = xMax[d];
                }
            for (int i = 0; i < W; i++)
                for (int d = 0; d < kNu; d++) {
                    lb[s.off_box + (int64_t)kNu * i + (int64_t)kNx * N + d] = uMin[d];
                    ub[s.off_box + (int64_t)kNu * i + (int64_t)kNx * N + d] = uMax[d];
                }
            if (s.H)
                for (int i = 0; i < W; i++) {
                    lb[s.off_half + (int64_t)s.H * i + 0] = -INFINITY;
                    ub[s.off_half + (int64_t)s.H * i + 0] = p->half_max[2];
                    lb[s.off_half + (int64_t)s.H * i + 1] = p->half_min[2];
                    ub[s.off_half + (int64_t)s.H * i + 1] = INFINITY;
                }
        }
    }
    return 0;
}

int impc_mpc_obstacle_layout(const impc_mpc_params *p, int32_t num_static, int32_t num_dynamic,
                             std::vector<int64_t> &slots, int64_t &obs_row_off) {
    Shape s;
    if (!make_shape(p, num_static, num_dynamic, &s)) return 1;
    std::vector<Trip> t;
    a_insertions(p, s, t);
    std::vector<int64_t> slot;
    csc_from_insertions(s.n, t, nullptr, nullptr, slot);
    const int64_t nob = (int64_t)4 * s.W * s.K, base = (int64_t)t.size() - nob;
    slots.assign(slot.begin() + base, slot.end());
    obs_row_off = s.off_obs;
    return 0;
}

extern "C" int impc_mpc_warm_start(const impc_mpc_params *p, int64_t nb, const double *prev_states,
                                   const double *prev_controls, double *x_ws) {
    Shape s;
    if (!make_shape(p, 0, 0, &s) || !x_ws) return 1;
    for (int64_t b = 0; b < nb; b++) {
        double *xb = x_ws + b * s.n;
        for (int64_t k = 0; k < s.n; k++) xb[k] = 0.0;
        if (prev_states)
            for (int64_t k = 0; k < (int64_t)kNx * s.N; k++) xb[k] = prev_states[b * (int64_t)kNx * s.N + k];
        if (prev_controls)
            for (int64_t k = 0; k < (int64_t)kNu * s.W; k++)
                xb[(int64_t)kNx * s.N + k] = prev_controls[b * (int64_t)kNu * s.W + k];
    }
    return 0;
}
