// admm_core.hpp -- one OSQP 0.6.2-equivalent QP solve, executed by ONE lane (one QP per thread).
//
// Data layout: every per-QP array is batch-interleaved ("SoA over the batch"): element e of the
// QP handled by lane `lane` lives at base[e * S + lane], S = padded batch size.  Consecutive
// lanes of a wavefront therefore touch consecutive 8-byte words on every access (one 512-B
// coalesced transaction per wave instruction), while all index arrays (the shared sparsity
// pattern and the symbolic programs of symbolic.hpp) are wave-uniform and are read through the
// scalar cache.
//
// Algorithm: OSQP 0.6.2 as restated in oracle/osqp_oracle.c (the functions named in comments
// are OSQP's, declared in reference third_party/osqp/auxil.h / scaling.h / lin_alg.h), with the
// linear system solved through the reduced matrix M = P + sigma I + A' diag(rho) A:
//     x~ = M^{-1} (sigma x - q + A'(rho z - y)),   z~ = A x~
// which equals OSQP's quasi-definite KKT solve (update_xz_tilde) in exact arithmetic.
//
// Functions are __host__ __device__ so that tests/native/core_harness.cpp can exercise the exact
// same code on the CPU (test infrastructure only; the product entry points launch it on the GPU).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/impc_qp.h"

#define IMPC_HD __host__ __device__ inline

namespace impc {

constexpr double kInf = 1e30;               // OSQP_INFTY (constants.h:100)
constexpr double kNan = 2143289344.0;       // OSQP_NAN = (c_float)0x7fc00000UL (constants.h:96)
constexpr double kDivTol = 1.0 / 1e30;      // OSQP_DIVISION_TOL (constants.h:104)
constexpr double kRhoMin = 1e-06, kRhoMax = 1e06, kRhoEqOverIneq = 1e03, kRhoTol = 1e-04;  // :64-67
constexpr double kMinScaling = 1e-04, kMaxScaling = 1e+04;                                  // :87-88

struct DevSettings {
    double rho, sigma, adaptive_rho_tolerance, eps_abs, eps_rel, eps_prim_inf, eps_dual_inf, alpha, time_limit;
    double tick_s;  // seconds per device-clock tick (hipDeviceAttributeWallClockRate of the context's device)
    int32_t scaling, adaptive_rho, rho_interval, max_iter, scaled_termination, check_termination, warm_start;
};

// Shared (wave-uniform) pattern + programs, see symbolic.hpp.
struct DevSym {
    int32_t n, m, nnzP, nnzA, nnzM, nnzL, nPt, nAt;
    const int32_t *Pp, *Pi, *Ap, *Ai, *Arp, *Arpos, *Arcol, *Arcolf, *perm, *iperm;
    const int32_t *Mp, *Mi, *Mdiag, *Pt_dest, *Pt_src, *At_dest, *At_a, *At_b, *At_r;
    const int32_t *Lp, *Li, *Lrp, *Lrc, *Lrpos, *upd_ptr, *upd_c, *upd_js, *upd_je, *upd_w;
};

// Per-QP scalar slots (interleaved like every other array).
// SC_TSETUP: device-clock ticks the QP's osqp_setup took (a first solve's time limit counts the
// setup time, OSQP 0.6.2's setup_time, and nothing that ran between setup and solve)
enum : int32_t { SC_C = 0, SC_CINV, SC_RHO, SC_SETUP_ERR, SC_TSETUP, SC_NSCAL };

// Batch-interleaved per-QP arrays.
struct DevWork {
    int64_t S;
    // inputs (original values)
    const double *Px, *q, *Ax, *l, *u, *xws, *yws;
    // working (scaled) data
    double *Ps, *qs, *As, *ls, *us, *D, *Dinv, *E, *Einv, *rho, *rhoinv, *ctype, *scal;
    // iterates
    double *x, *z, *y, *v, *w, *dx, *dy;
    // factorisation
    double *Mval, *Lx, *Dinvf, *yf;
    // temporaries
    double *tn1, *tm1;
    // outputs (interleaved)
    double *xo, *yo;
    impc_info *info;  // QP-major
    const double *tlim = nullptr;  // per-QP time limits [B] (impc_batch_set_time_limits), or the settings'
};

#define IMPC_AT(arr, e) (arr)[(int64_t)(e) * S + lane]

IMPC_HD double dmax(double a, double b) { return a > b ? a : b; }  // c_max
IMPC_HD double dmin(double a, double b) { return a < b ? a : b; }  // c_min

// ------------------------------------------------------------------ KKT assembly + LDL^T
// M = P + sigma I + A' R A in factor order, then QDLDL_factor's arithmetic replayed from the
// symbolic program.  Returns 0, or 1 when a pivot is not positive (non-convex / not SPD).
IMPC_HD int assemble_and_factor(const DevSym &sy, const DevWork &wk, const DevSettings &st, int lane) {
    const int64_t S = wk.S;
    for (int32_t p = 0; p < sy.nnzM; p++) IMPC_AT(wk.Mval, p) = 0.0;
    for (int32_t t = 0; t < sy.nPt; t++) IMPC_AT(wk.Mval, sy.Pt_dest[t]) += IMPC_AT(wk.Ps, sy.Pt_src[t]);
    for (int32_t k = 0; k < sy.n; k++) IMPC_AT(wk.Mval, sy.Mdiag[k]) += st.sigma;
    for (int32_t t = 0; t < sy.nAt; t++)
        IMPC_AT(wk.Mval, sy.At_dest[t]) +=
            IMPC_AT(wk.As, sy.At_a[t]) * IMPC_AT(wk.rho, sy.At_r[t]) * IMPC_AT(wk.As, sy.At_b[t]);
    // QDLDL_factor, numeric part
    for (int32_t k = 0; k < sy.n; k++) IMPC_AT(wk.yf, k) = 0.0;
    int bad = 0;
    for (int32_t k = 0; k < sy.n; k++) {
        double Dk = 0.0;
        for (int32_t p = sy.Mp[k]; p < sy.Mp[k + 1]; p++) {
            int32_t r = sy.Mi[p];
            double val = IMPC_AT(wk.Mval, p);
            if (r == k)
                Dk = val;
            else
                IMPC_AT(wk.yf, r) = val;
        }
        for (int32_t t = sy.upd_ptr[k]; t < sy.upd_ptr[k + 1]; t++) {
            int32_t c = sy.upd_c[t];
            double yv = IMPC_AT(wk.yf, c);
            int32_t je = sy.upd_je[t];
            for (int32_t j = sy.upd_js[t]; j < je; j++) IMPC_AT(wk.yf, sy.Li[j]) -= IMPC_AT(wk.Lx, j) * yv;
            double lv = yv * IMPC_AT(wk.Dinvf, c);
            IMPC_AT(wk.Lx, sy.upd_w[t]) = lv;
            Dk -= yv * lv;
            IMPC_AT(wk.yf, c) = 0.0;
        }
        if (!(Dk > 0.0)) bad = 1;
        IMPC_AT(wk.Dinvf, k) = 1.0 / Dk;
    }
    return bad;
}

// x~ = M^{-1} rhs; rhs and result in wk.w (factor order).  QDLDL_solve arithmetic:
// L y = b (row gather), y *= Dinv, L' x = y (column gather).
IMPC_HD void ldl_solve(const DevSym &sy, const DevWork &wk, int lane) {
    const int64_t S = wk.S;
    for (int32_t i = 0; i < sy.n; i++) {
        double s = IMPC_AT(wk.w, i);
        for (int32_t t = sy.Lrp[i]; t < sy.Lrp[i + 1]; t++)
            s -= IMPC_AT(wk.Lx, sy.Lrpos[t]) * IMPC_AT(wk.w, sy.Lrc[t]);
        IMPC_AT(wk.w, i) = s;
    }
    for (int32_t i = sy.n - 1; i >= 0; i--) {
        double s = IMPC_AT(wk.w, i) * IMPC_AT(wk.Dinvf, i);
        for (int32_t j = sy.Lp[i]; j < sy.Lp[i + 1]; j++) s -= IMPC_AT(wk.Lx, j) * IMPC_AT(wk.w, sy.Li[j]);
        IMPC_AT(wk.w, i) = s;
    }
}

// rho_vec from constraint types (set_rho_vec, auxil.h:34) and v = rho z - y.
IMPC_HD void set_rho_vec(const DevSym &sy, const DevWork &wk, double rho, int lane) {
    const int64_t S = wk.S;
    for (int32_t i = 0; i < sy.m; i++) {
        double li = IMPC_AT(wk.ls, i), ui = IMPC_AT(wk.us, i), r, t;
        if ((li < -kInf * kMinScaling) && (ui > kInf * kMinScaling)) {
            t = -1.0;
            r = kRhoMin;
        } else if (ui - li < kRhoTol) {
            t = 1.0;
            r = kRhoEqOverIneq * rho;
        } else {
            t = 0.0;
            r = rho;
        }
        IMPC_AT(wk.ctype, i) = t;
        IMPC_AT(wk.rho, i) = r;
        IMPC_AT(wk.rhoinv, i) = 1. / r;
    }
}

IMPC_HD void refresh_v(const DevSym &sy, const DevWork &wk, int lane) {
    const int64_t S = wk.S;
    for (int32_t i = 0; i < sy.m; i++)
        IMPC_AT(wk.v, i) = IMPC_AT(wk.rho, i) * IMPC_AT(wk.z, i) - IMPC_AT(wk.y, i);
}

// osqp_warm_start (osqp.h:157) into a set-up workspace: x <- Dinv x_ws, y <- c Einv y_ws,
// z <- A x (scaled data); the caller refreshes v.
IMPC_HD void apply_warm_start(const DevSym &sy, const DevWork &wk, const DevSettings &st, double c, int lane) {
    const int64_t S = wk.S;
    const int32_t n = sy.n, m = sy.m;
    const bool scaled = st.scaling > 0;
    for (int32_t j = 0; j < n; j++)
        IMPC_AT(wk.x, j) = scaled ? IMPC_AT(wk.Dinv, j) * IMPC_AT(wk.xws, j) : IMPC_AT(wk.xws, j);
    for (int32_t i = 0; i < m; i++) {
        double yi = IMPC_AT(wk.yws, i);
        if (scaled) {
            yi = IMPC_AT(wk.Einv, i) * yi;
            yi *= c;
        }
        IMPC_AT(wk.y, i) = yi;
    }
    for (int32_t i = 0; i < m; i++) {  // z = A x
        double s = 0.0;
        for (int32_t k = sy.Arp[i]; k < sy.Arp[i + 1]; k++) s += IMPC_AT(wk.As, sy.Arpos[k]) * IMPC_AT(wk.x, sy.Arcol[k]);
        IMPC_AT(wk.z, i) = s;
    }
}

// --------------------------------------------------------------------------- osqp_setup
// validate (bounds), copy + clamp, scale_data (Ruiz, scaling.h:21), set_rho_vec, factor, and
// the optional osqp_warm_start (osqp.h:157).  Returns the per-QP setup exitflag.
IMPC_HD int qp_setup(const DevSym &sy, const DevWork &wk, const DevSettings &st, int lane, int has_ws) {
    const int64_t S = wk.S;
    const int32_t n = sy.n, m = sy.m;
    for (int32_t k = 0; k < sy.nnzP; k++) IMPC_AT(wk.Ps, k) = IMPC_AT(wk.Px, k);
    for (int32_t k = 0; k < n; k++) IMPC_AT(wk.qs, k) = IMPC_AT(wk.q, k);
    for (int32_t k = 0; k < sy.nnzA; k++) IMPC_AT(wk.As, k) = IMPC_AT(wk.Ax, k);
    for (int32_t i = 0; i < m; i++) {
        IMPC_AT(wk.ls, i) = dmin(dmax(IMPC_AT(wk.l, i), -kInf), kInf);
        IMPC_AT(wk.us, i) = dmin(dmax(IMPC_AT(wk.u, i), -kInf), kInf);
    }
    double c = 1.0;
    for (int32_t j = 0; j < n; j++) IMPC_AT(wk.D, j) = 1.0;
    for (int32_t i = 0; i < m; i++) IMPC_AT(wk.E, i) = 1.0;
    double *Dt = wk.tn1, *Et = wk.tm1;
    for (int32_t it = 0; it < st.scaling; it++) {
        // compute_inf_norm_cols_KKT: D_t = max(colnorm_sym(P), colnorm(A)); E_t = rownorm(A)
        for (int32_t j = 0; j < n; j++) IMPC_AT(Dt, j) = 0.0;
        for (int32_t j = 0; j < n; j++)
            for (int32_t k = sy.Pp[j]; k < sy.Pp[j + 1]; k++) {
                int32_t i = sy.Pi[k];
                double a = fabs(IMPC_AT(wk.Ps, k));
                IMPC_AT(Dt, j) = dmax(a, IMPC_AT(Dt, j));
                if (i != j) IMPC_AT(Dt, i) = dmax(a, IMPC_AT(Dt, i));
            }
        for (int32_t j = 0; j < n; j++) {
            double a = 0.0;
            for (int32_t k = sy.Ap[j]; k < sy.Ap[j + 1]; k++) a = dmax(fabs(IMPC_AT(wk.As, k)), a);
            IMPC_AT(Dt, j) = dmax(IMPC_AT(Dt, j), a);
        }
        for (int32_t i = 0; i < m; i++) {
            double a = 0.0;
            for (int32_t k = sy.Arp[i]; k < sy.Arp[i + 1]; k++) a = dmax(fabs(IMPC_AT(wk.As, sy.Arpos[k])), a);
            IMPC_AT(Et, i) = a;
        }
        // limit_scaling, sqrt, reciprocal
        for (int32_t j = 0; j < n; j++) {
            double d = IMPC_AT(Dt, j);
            d = d < kMinScaling ? 1.0 : d;
            d = d > kMaxScaling ? kMaxScaling : d;
            IMPC_AT(Dt, j) = 1.0 / sqrt(d);
        }
        for (int32_t i = 0; i < m; i++) {
            double e = IMPC_AT(Et, i);
            e = e < kMinScaling ? 1.0 : e;
            e = e > kMaxScaling ? kMaxScaling : e;
            IMPC_AT(Et, i) = 1.0 / sqrt(e);
        }
        // P <- D P D, A <- E A D, q <- D q, D *= D_t, E *= E_t
        for (int32_t j = 0; j < n; j++) {
            double dj = IMPC_AT(Dt, j);
            for (int32_t k = sy.Pp[j]; k < sy.Pp[j + 1]; k++)
                IMPC_AT(wk.Ps, k) = (IMPC_AT(wk.Ps, k) * IMPC_AT(Dt, sy.Pi[k])) * dj;
            for (int32_t k = sy.Ap[j]; k < sy.Ap[j + 1]; k++)
                IMPC_AT(wk.As, k) = (IMPC_AT(wk.As, k) * IMPC_AT(Et, sy.Ai[k])) * dj;
            IMPC_AT(wk.qs, j) = dj * IMPC_AT(wk.qs, j);
            IMPC_AT(wk.D, j) = IMPC_AT(wk.D, j) * dj;
        }
        for (int32_t i = 0; i < m; i++) IMPC_AT(wk.E, i) = IMPC_AT(wk.E, i) * IMPC_AT(Et, i);
        // cost normalisation: c_t = 1 / max(mean colnorm_sym(P), ||q||_inf), limited
        for (int32_t j = 0; j < n; j++) IMPC_AT(Dt, j) = 0.0;
        for (int32_t j = 0; j < n; j++)
            for (int32_t k = sy.Pp[j]; k < sy.Pp[j + 1]; k++) {
                int32_t i = sy.Pi[k];
                double a = fabs(IMPC_AT(wk.Ps, k));
                IMPC_AT(Dt, j) = dmax(a, IMPC_AT(Dt, j));
                if (i != j) IMPC_AT(Dt, i) = dmax(a, IMPC_AT(Dt, i));
            }
        double ct = 0.0, qn = 0.0;
        for (int32_t j = 0; j < n; j++) ct += IMPC_AT(Dt, j);
        ct = ct / (double)n;
        for (int32_t j = 0; j < n; j++) qn = dmax(fabs(IMPC_AT(wk.qs, j)), qn);
        qn = qn < kMinScaling ? 1.0 : qn;
        qn = qn > kMaxScaling ? kMaxScaling : qn;
        ct = dmax(ct, qn);
        ct = ct < kMinScaling ? 1.0 : ct;
        ct = ct > kMaxScaling ? kMaxScaling : ct;
        ct = 1. / ct;
        for (int32_t k = 0; k < sy.nnzP; k++) IMPC_AT(wk.Ps, k) *= ct;
        for (int32_t j = 0; j < n; j++) IMPC_AT(wk.qs, j) *= ct;
        c *= ct;
    }
    IMPC_AT(wk.scal, SC_C) = c;
    IMPC_AT(wk.scal, SC_CINV) = 1. / c;
    for (int32_t j = 0; j < n; j++) IMPC_AT(wk.Dinv, j) = 1. / IMPC_AT(wk.D, j);
    for (int32_t i = 0; i < m; i++) {
        double e = IMPC_AT(wk.E, i);
        IMPC_AT(wk.Einv, i) = 1. / e;
        IMPC_AT(wk.ls, i) = e * IMPC_AT(wk.ls, i);
        IMPC_AT(wk.us, i) = e * IMPC_AT(wk.us, i);
    }
    double rho = dmin(dmax(st.rho, kRhoMin), kRhoMax);
    IMPC_AT(wk.scal, SC_RHO) = rho;
    set_rho_vec(sy, wk, rho, lane);
    int err = assemble_and_factor(sy, wk, st, lane) ? IMPC_NONCVX_ERROR : 0;
    IMPC_AT(wk.scal, SC_SETUP_ERR) = (double)err;
    // iterates: zero (osqp_setup cold_start), then osqp_warm_start when requested
    for (int32_t j = 0; j < n; j++) IMPC_AT(wk.x, j) = 0.0;
    for (int32_t i = 0; i < m; i++) {
        IMPC_AT(wk.z, i) = 0.0;
        IMPC_AT(wk.y, i) = 0.0;
    }
    if (has_ws) apply_warm_start(sy, wk, st, c, lane);
    refresh_v(sy, wk, lane);
    return err;
}

// ---------------------------------------------------------------------- osqp_solve state
struct InfoState {
    // residuals and the norms the tolerances / rho estimate need (update_info)
    double pri_res, dua_res;
    double pri_norm_u, dua_norm_u;  // unscaled-termination norms (max(||Einv z||, ||Einv Ax||), cinv * max(...))
    double pri_norm_s, dua_norm_s;  // scaled-space norms (max(||z||, ||Ax||), max(||q||, ||A'y||, ||Px||))
    double pri_plain, dua_plain;    // ||Ax - z||, ||Px + q + A'y|| in the scaled space
    int64_t iter;
};

// Px for the upper-triangular P (mat_vec + mat_tpose_vec skip_diag) into out[n].
IMPC_HD void sym_p_times(const DevSym &sy, const DevWork &wk, const double *vin, double *out, int lane) {
    const int64_t S = wk.S;
    for (int32_t j = 0; j < sy.n; j++) IMPC_AT(out, j) = 0.0;
    for (int32_t j = 0; j < sy.n; j++)
        for (int32_t k = sy.Pp[j]; k < sy.Pp[j + 1]; k++)
            IMPC_AT(out, sy.Pi[k]) += IMPC_AT(wk.Ps, k) * IMPC_AT(vin, j);
    for (int32_t j = 0; j < sy.n; j++)
        for (int32_t k = sy.Pp[j]; k < sy.Pp[j + 1]; k++) {
            int32_t i = sy.Pi[k];
            IMPC_AT(out, j) += i == j ? 0 : IMPC_AT(wk.Ps, k) * IMPC_AT(vin, i);
        }
}

// update_info (auxil.h:122): residuals of the current iterate.
IMPC_HD void update_info(const DevSym &sy, const DevWork &wk, const DevSettings &st, InfoState &inf, int64_t iter,
                         double cinv, int lane) {
    const int64_t S = wk.S;
    const bool unsc = st.scaling > 0 && !st.scaled_termination;
    inf.iter = iter;
    double pr_u = 0, z_u = 0, ax_u = 0, pr_p = 0, z_p = 0, ax_p = 0;
    for (int32_t i = 0; i < sy.m; i++) {
        double ax = 0.0;
        for (int32_t k = sy.Arp[i]; k < sy.Arp[i + 1]; k++)
            ax += IMPC_AT(wk.As, sy.Arpos[k]) * IMPC_AT(wk.x, sy.Arcol[k]);
        double zi = IMPC_AT(wk.z, i);
        double r = ax + -1 * zi;
        double ei = IMPC_AT(wk.Einv, i);
        pr_p = dmax(pr_p, fabs(r));
        z_p = dmax(z_p, fabs(zi));
        ax_p = dmax(ax_p, fabs(ax));
        pr_u = dmax(pr_u, fabs(ei * r));
        z_u = dmax(z_u, fabs(ei * zi));
        ax_u = dmax(ax_u, fabs(ei * ax));
    }
    sym_p_times(sy, wk, wk.x, wk.tn1, lane);
    double dr_u = 0, q_u = 0, aty_u = 0, px_u = 0, dr_p = 0, q_p = 0, aty_p = 0, px_p = 0;
    for (int32_t j = 0; j < sy.n; j++) {
        double aty = 0.0;
        for (int32_t k = sy.Ap[j]; k < sy.Ap[j + 1]; k++) aty += IMPC_AT(wk.As, k) * IMPC_AT(wk.y, sy.Ai[k]);
        double qj = IMPC_AT(wk.qs, j), px = IMPC_AT(wk.tn1, j);
        double r = qj + 1 * px;
        r = r + 1 * aty;
        double di = IMPC_AT(wk.Dinv, j);
        dr_p = dmax(dr_p, fabs(r));
        q_p = dmax(q_p, fabs(qj));
        aty_p = dmax(aty_p, fabs(aty));
        px_p = dmax(px_p, fabs(px));
        dr_u = dmax(dr_u, fabs(di * r));
        q_u = dmax(q_u, fabs(di * qj));
        aty_u = dmax(aty_u, fabs(di * aty));
        px_u = dmax(px_u, fabs(di * px));
    }
    inf.pri_plain = pr_p;
    inf.dua_plain = dr_p;
    inf.pri_norm_s = dmax(z_p, ax_p);
    inf.dua_norm_s = dmax(dmax(q_p, aty_p), px_p);
    if (unsc) {
        inf.pri_res = sy.m == 0 ? 0.0 : pr_u;
        inf.dua_res = cinv * dr_u;
        inf.pri_norm_u = dmax(z_u, ax_u);
        inf.dua_norm_u = dmax(dmax(q_u, aty_u), px_u) * cinv;
    } else {
        inf.pri_res = sy.m == 0 ? 0.0 : pr_p;
        inf.dua_res = dr_p;
        inf.pri_norm_u = inf.pri_norm_s;
        inf.dua_norm_u = inf.dua_norm_s;
    }
}

// is_primal_infeasible (auxil.c); projects wk.dy in place like the reference.
IMPC_HD int primal_infeasible(const DevSym &sy, const DevWork &wk, const DevSettings &st, double eps, int lane) {
    const int64_t S = wk.S;
    const bool unsc = st.scaling > 0 && !st.scaled_termination;
    double nrm = 0.0;
    for (int32_t i = 0; i < sy.m; i++) {
        double d = IMPC_AT(wk.dy, i), ui = IMPC_AT(wk.us, i), li = IMPC_AT(wk.ls, i);
        if (ui > kInf * kMinScaling) {
            d = (li < -kInf * kMinScaling) ? 0.0 : dmin(d, 0.0);
        } else if (li < -kInf * kMinScaling) {
            d = dmax(d, 0.0);
        }
        IMPC_AT(wk.dy, i) = d;
        nrm = dmax(nrm, fabs(unsc ? IMPC_AT(wk.E, i) * d : d));
    }
    if (nrm > kDivTol) {
        double lhs = 0.0;
        for (int32_t i = 0; i < sy.m; i++) {
            double d = IMPC_AT(wk.dy, i);
            lhs += IMPC_AT(wk.us, i) * dmax(d, 0) + IMPC_AT(wk.ls, i) * dmin(d, 0);
        }
        if (lhs < eps * nrm) {
            double mx = 0.0;
            for (int32_t j = 0; j < sy.n; j++) {
                double s = 0.0;
                for (int32_t k = sy.Ap[j]; k < sy.Ap[j + 1]; k++) s += IMPC_AT(wk.As, k) * IMPC_AT(wk.dy, sy.Ai[k]);
                if (unsc) s = IMPC_AT(wk.Dinv, j) * s;
                mx = dmax(mx, fabs(s));
            }
            return mx < eps * nrm;
        }
    }
    return 0;
}

// is_dual_infeasible (auxil.c).
IMPC_HD int dual_infeasible(const DevSym &sy, const DevWork &wk, const DevSettings &st, double eps, double c,
                            int lane) {
    const int64_t S = wk.S;
    const bool unsc = st.scaling > 0 && !st.scaled_termination;
    double nrm = 0.0, cs = unsc ? c : 1.0;
    for (int32_t j = 0; j < sy.n; j++) {
        double d = IMPC_AT(wk.dx, j);
        nrm = dmax(nrm, fabs(unsc ? IMPC_AT(wk.D, j) * d : d));
    }
    if (nrm > kDivTol) {
        double qdx = 0.0;
        for (int32_t j = 0; j < sy.n; j++) qdx += IMPC_AT(wk.qs, j) * IMPC_AT(wk.dx, j);
        if (qdx < cs * eps * nrm) {
            sym_p_times(sy, wk, wk.dx, wk.tn1, lane);
            double mx = 0.0;
            for (int32_t j = 0; j < sy.n; j++) {
                double pv = IMPC_AT(wk.tn1, j);
                if (unsc) pv = IMPC_AT(wk.Dinv, j) * pv;
                mx = dmax(mx, fabs(pv));
            }
            if (mx < cs * eps * nrm) {
                for (int32_t i = 0; i < sy.m; i++) {
                    double s = 0.0;
                    for (int32_t k = sy.Arp[i]; k < sy.Arp[i + 1]; k++)
                        s += IMPC_AT(wk.As, sy.Arpos[k]) * IMPC_AT(wk.dx, sy.Arcol[k]);
                    if (unsc) s = IMPC_AT(wk.Einv, i) * s;
                    if (((IMPC_AT(wk.us, i) < kInf * kMinScaling) && (s > eps * nrm)) ||
                        ((IMPC_AT(wk.ls, i) > -kInf * kMinScaling) && (s < -eps * nrm)))
                        return 0;
                }
                return 1;
            }
        }
    }
    return 0;
}

// check_termination (auxil.h:153).  Returns 1 when a final status was set.
IMPC_HD int check_termination(const DevSym &sy, const DevWork &wk, const DevSettings &st, const InfoState &inf,
                              int approximate, double c, int64_t &status, double &obj, int lane) {
    const int64_t S = wk.S;
    if ((inf.pri_res > kInf) || (inf.dua_res > kInf)) {
        status = IMPC_NON_CVX;
        obj = kNan;
        return 1;
    }
    double eps_abs = st.eps_abs, eps_rel = st.eps_rel, eps_pinf = st.eps_prim_inf, eps_dinf = st.eps_dual_inf;
    if (approximate) {
        eps_abs *= 10;
        eps_rel *= 10;
        eps_pinf *= 10;
        eps_dinf *= 10;
    }
    int prim_ok = 0, dual_ok = 0, prim_inf = 0, dual_inf = 0;
    if (sy.m == 0) {
        prim_ok = 1;
    } else {
        double eps_prim = eps_abs + eps_rel * inf.pri_norm_u;
        if (inf.pri_res < eps_prim)
            prim_ok = 1;
        else
            prim_inf = primal_infeasible(sy, wk, st, eps_pinf, lane);
    }
    double eps_dual = eps_abs + eps_rel * inf.dua_norm_u;
    if (inf.dua_res < eps_dual)
        dual_ok = 1;
    else
        dual_inf = dual_infeasible(sy, wk, st, eps_dinf, c, lane);
    (void)S;
    if (prim_ok && dual_ok) {
        status = approximate ? IMPC_SOLVED_INACCURATE : IMPC_SOLVED;
        return 1;
    } else if (prim_inf) {
        status = approximate ? IMPC_PRIMAL_INFEASIBLE_INACCURATE : IMPC_PRIMAL_INFEASIBLE;
        obj = kInf;
        return 1;
    } else if (dual_inf) {
        status = approximate ? IMPC_DUAL_INFEASIBLE_INACCURATE : IMPC_DUAL_INFEASIBLE;
        obj = -kInf;
        return 1;
    }
    return 0;
}

// compute_rho_estimate (auxil.h:21) from the last update_info.
IMPC_HD double rho_estimate(const InfoState &inf, double rho) {
    double pri = inf.pri_plain / (inf.pri_norm_s + kDivTol);
    double dua = inf.dua_plain / (inf.dua_norm_s + kDivTol);
    double est = rho * sqrt(pri / (dua + kDivTol));
    return dmin(dmax(est, kRhoMin), kRhoMax);
}

// osqp_update_rho (osqp.h:264): new rho on inequality / equality rows, refactor, refresh v.
IMPC_HD int update_rho(const DevSym &sy, const DevWork &wk, const DevSettings &st, double rho_new, int lane) {
    const int64_t S = wk.S;
    double rho = dmin(dmax(rho_new, kRhoMin), kRhoMax);
    IMPC_AT(wk.scal, SC_RHO) = rho;
    for (int32_t i = 0; i < sy.m; i++) {
        double t = IMPC_AT(wk.ctype, i);
        if (t == 0.0) {
            IMPC_AT(wk.rho, i) = rho;
            IMPC_AT(wk.rhoinv, i) = 1. / rho;
        } else if (t == 1.0) {
            double r = kRhoEqOverIneq * rho;
            IMPC_AT(wk.rho, i) = r;
            IMPC_AT(wk.rhoinv, i) = 1. / r;
        }
    }
    int bad = assemble_and_factor(sy, wk, st, lane);
    refresh_v(sy, wk, lane);
    return bad;
}

// the device's constant-rate clock (s_memrealtime); its rate comes from
// hipDeviceAttributeWallClockRate (DevSettings::tick_s), never assumed
IMPC_HD uint64_t device_clock() {
#ifdef __HIP_DEVICE_COMPILE__
    return wall_clock64();
#else
    return 0;
#endif
}

// ---------------------------------------------------------------------------- osqp_solve
// Runs the ADMM loop from the current iterates, sets the info record and the interleaved
// unscaled outputs xo / yo (store_solution + unscale_solution).
// first_run: the first solve after qp_setup -- as OSQP 0.6.2's osqp_solve, its time limit counts
// setup_time + the solve's own time (later solves: the solve's own time)
IMPC_HD void qp_solve(const DevSym &sy, const DevWork &wk, const DevSettings &st, int lane, int64_t qp_index,
                      int64_t rho_updates0, int first_run = 0) {
    const int64_t S = wk.S;
    const int32_t n = sy.n, m = sy.m;
    impc_info &out = wk.info[qp_index];
    const double c = IMPC_AT(wk.scal, SC_C), cinv = IMPC_AT(wk.scal, SC_CINV);
    const bool scaled = st.scaling > 0;
    double rho = IMPC_AT(wk.scal, SC_RHO);
    int64_t status = IMPC_UNSOLVED, rho_updates = rho_updates0;
    double obj = 0.0, rho_est = rho;
    InfoState inf;
    inf.pri_res = inf.dua_res = inf.pri_norm_u = inf.dua_norm_u = inf.pri_norm_s = inf.dua_norm_s = 0.0;
    inf.pri_plain = inf.dua_plain = 0.0;
    inf.iter = 0;
    if ((int)IMPC_AT(wk.scal, SC_SETUP_ERR) != 0) {
        out.iter = 0;
        out.status_val = IMPC_NON_CVX;
        out.rho_updates = 0;
        out.setup_exitflag = (int64_t)IMPC_AT(wk.scal, SC_SETUP_ERR);
        out.obj_val = kNan;
        out.pri_res = out.dua_res = 0.0;
        out.rho_estimate = rho;
        for (int32_t j = 0; j < n; j++) IMPC_AT(wk.xo, j) = kNan;
        for (int32_t i = 0; i < m; i++) IMPC_AT(wk.yo, i) = kNan;
        return;
    }
    if (!st.warm_start) {  // cold_start
        for (int32_t j = 0; j < n; j++) IMPC_AT(wk.x, j) = 0.0;
        for (int32_t i = 0; i < m; i++) {
            IMPC_AT(wk.z, i) = 0.0;
            IMPC_AT(wk.y, i) = 0.0;
        }
        refresh_v(sy, wk, lane);
    }
    const double alpha = st.alpha, oma = (double)1.0 - st.alpha, sigma = st.sigma;
    const int32_t chk = st.check_termination;
    const double tl = wk.tlim ? wk.tlim[qp_index] : st.time_limit;
    const uint64_t t0 = device_clock() - (first_run ? (uint64_t)IMPC_AT(wk.scal, SC_TSETUP) : 0);
    int can_check = 0;
    int64_t iter;
    for (iter = 1; iter <= st.max_iter; iter++) {
        const int need_delta = (chk && iter % chk == 0) || iter == st.max_iter ||
                               (st.adaptive_rho && st.rho_interval && iter % st.rho_interval == 0) ||
                               tl > 0;
        // ---- update_xz_tilde: rhs (factor order) then the LDL^T solve
        for (int32_t p = 0; p < n; p++) {
            int32_t j = sy.perm[p];
            double r = sigma * IMPC_AT(wk.x, j) - IMPC_AT(wk.qs, j);
            for (int32_t k = sy.Ap[j]; k < sy.Ap[j + 1]; k++) r += IMPC_AT(wk.As, k) * IMPC_AT(wk.v, sy.Ai[k]);
            IMPC_AT(wk.w, p) = r;
        }
        ldl_solve(sy, wk, lane);
        // ---- update_x
        for (int32_t j = 0; j < n; j++) {
            double xp = IMPC_AT(wk.x, j);
            double xn = alpha * IMPC_AT(wk.w, sy.iperm[j]) + oma * xp;
            if (need_delta) IMPC_AT(wk.dx, j) = xn - xp;
            IMPC_AT(wk.x, j) = xn;
        }
        // ---- update_z (+ project) and update_y, fused per constraint row
        for (int32_t i = 0; i < m; i++) {
            double zt = 0.0;
            for (int32_t k = sy.Arp[i]; k < sy.Arp[i + 1]; k++)
                zt += IMPC_AT(wk.As, sy.Arpos[k]) * IMPC_AT(wk.w, sy.Arcolf[k]);
            double zp = IMPC_AT(wk.z, i), yi = IMPC_AT(wk.y, i), ri = IMPC_AT(wk.rho, i);
            double zr = alpha * zt + oma * zp;
            double zn = dmin(dmax(zr + IMPC_AT(wk.rhoinv, i) * yi, IMPC_AT(wk.ls, i)), IMPC_AT(wk.us, i));
            double dyi = ri * (zr - zn);
            yi += dyi;
            if (need_delta) IMPC_AT(wk.dy, i) = dyi;
            IMPC_AT(wk.z, i) = zn;
            IMPC_AT(wk.y, i) = yi;
            IMPC_AT(wk.v, i) = ri * zn - yi;
        }
        // osqp_solve (PROFILING build): after the ADMM steps, before can_check is recomputed, so
        // can_check keeps the previous iteration's value when the limit fires
        if (tl > 0 && (double)(device_clock() - t0) * st.tick_s >= tl) {
            status = IMPC_TIME_LIMIT_REACHED;
            break;
        }
        can_check = chk && (iter % chk == 0);
        if (can_check) {
            update_info(sy, wk, st, inf, iter, cinv, lane);
            if (check_termination(sy, wk, st, inf, 0, c, status, obj, lane)) break;
        }
        if (st.adaptive_rho && st.rho_interval && (iter % st.rho_interval == 0)) {
            if (!can_check) update_info(sy, wk, st, inf, iter, cinv, lane);
            double rn = rho_estimate(inf, rho);
            rho_est = rn;
            if ((rn > rho * st.adaptive_rho_tolerance) || (rn < rho / st.adaptive_rho_tolerance)) {
                const int bad = update_rho(sy, wk, st, rn, lane);
                rho = IMPC_AT(wk.scal, SC_RHO);
                rho_updates += 1;
                if (bad) {  // osqp_solve exits with exitflag 1: status UNSOLVED, no stored solution
                    out.iter = inf.iter;
                    out.status_val = IMPC_UNSOLVED;
                    out.rho_updates = rho_updates;
                    out.setup_exitflag = 0;
                    out.pri_res = inf.pri_res;
                    out.dua_res = inf.dua_res;
                    out.rho_estimate = rho_est;
                    return;
                }
            }
        }
    }
    // post-loop update_info / check (may turn TIME_LIMIT_REACHED into SOLVED), as osqp_solve
    if (!can_check) {
        update_info(sy, wk, st, inf, iter - 1, cinv, lane);
        check_termination(sy, wk, st, inf, 0, c, status, obj, lane);
    }
    const bool has_sol = status != IMPC_PRIMAL_INFEASIBLE && status != IMPC_PRIMAL_INFEASIBLE_INACCURATE &&
                         status != IMPC_DUAL_INFEASIBLE && status != IMPC_DUAL_INFEASIBLE_INACCURATE &&
                         status != IMPC_NON_CVX;
    if (has_sol) {  // compute_obj_val: quad_form(P, x) + q'x, times cinv
        double qf = 0.0;
        for (int32_t j = 0; j < n; j++)
            for (int32_t k = sy.Pp[j]; k < sy.Pp[j + 1]; k++) {
                int32_t i = sy.Pi[k];
                if (i == j)
                    qf += (double).5 * IMPC_AT(wk.Ps, k) * IMPC_AT(wk.x, i) * IMPC_AT(wk.x, i);
                else
                    qf += IMPC_AT(wk.Ps, k) * IMPC_AT(wk.x, i) * IMPC_AT(wk.x, j);
            }
        double qx = 0.0;
        for (int32_t j = 0; j < n; j++) qx += IMPC_AT(wk.qs, j) * IMPC_AT(wk.x, j);
        obj = qf + qx;
        if (scaled) obj *= cinv;
    }
    if (status == IMPC_UNSOLVED) {
        if (!check_termination(sy, wk, st, inf, 1, c, status, obj, lane)) status = IMPC_MAX_ITER_REACHED;
    }
    rho_est = rho_estimate(inf, rho);
    const bool has_sol2 = status != IMPC_PRIMAL_INFEASIBLE && status != IMPC_PRIMAL_INFEASIBLE_INACCURATE &&
                          status != IMPC_DUAL_INFEASIBLE && status != IMPC_DUAL_INFEASIBLE_INACCURATE &&
                          status != IMPC_NON_CVX;
    if (has_sol2) {
        for (int32_t j = 0; j < n; j++)
            IMPC_AT(wk.xo, j) = scaled ? IMPC_AT(wk.D, j) * IMPC_AT(wk.x, j) : IMPC_AT(wk.x, j);
        for (int32_t i = 0; i < m; i++) {
            double yi = IMPC_AT(wk.y, i);
            if (scaled) {
                yi = IMPC_AT(wk.E, i) * yi;  // unscale_solution: y = E y / c
                yi *= cinv;
            }
            IMPC_AT(wk.yo, i) = yi;
        }
    } else {
        for (int32_t j = 0; j < n; j++) IMPC_AT(wk.xo, j) = kNan;
        for (int32_t i = 0; i < m; i++) IMPC_AT(wk.yo, i) = kNan;
        for (int32_t j = 0; j < n; j++) IMPC_AT(wk.x, j) = 0.0;  // cold_start for the next solve
        for (int32_t i = 0; i < m; i++) {
            IMPC_AT(wk.z, i) = 0.0;
            IMPC_AT(wk.y, i) = 0.0;
        }
        refresh_v(sy, wk, lane);
    }
    out.iter = inf.iter;
    out.status_val = status;
    out.rho_updates = rho_updates;
    out.setup_exitflag = 0;
    out.obj_val = obj;
    out.pri_res = inf.pri_res;
    out.dua_res = inf.dua_res;
    out.rho_estimate = rho_est;
}

}  // namespace impc
