/*
 * osqp_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity oracle).
 *
 * A plain-C, single-threaded-per-QP restatement of the OSQP 0.6.2 ADMM solver that the
 * reference calls through OsqpEigen 0.7.0 from trajPlanner::mpcPlanner::solveTraj
 * (reference: trajectory_planner/include/trajectory_planner/mpcPlanner.cpp:436-527).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline.  The product (libimpc_qp.so) never
 * links or calls it.
 *
 * Provenance / parity status
 * --------------------------
 * OSQP's C sources are NOT vendored in /root/reference (only its headers and a prebuilt
 * x86 libosqp.so, which this build never loads or runs).  The algorithm below restates
 * the published OSQP 0.6.2 design, function by function, using the constants, struct
 * layouts and prototypes the reference does vendor:
 *   third_party/osqp/constants.h:12   (OSQP_VERSION "0.6.2")
 *   third_party/osqp/constants.h:59-119 (RHO, SIGMA, MAX_ITER, EPS_*, ALPHA, RHO_MIN/MAX,
 *                                       RHO_EQ_OVER_RHO_INEQ, RHO_TOL, CHECK_TERMINATION,
 *                                       SCALING, MIN/MAX_SCALING, OSQP_NAN, OSQP_INFTY,
 *                                       ADAPTIVE_RHO_*)
 *   third_party/osqp/types.h:139-176  (OSQPSettings field order, mirrored by ora_settings)
 *   third_party/osqp/auxil.h:21-172   (compute_rho_estimate, adapt_rho, set_rho_vec,
 *                                       update_rho_vec, update_xz_tilde, update_x/z/y,
 *                                       compute_obj_val, has_solution, store_solution,
 *                                       update_info, check_termination, validate_*)
 *   third_party/osqp/scaling.h:21-38  (scale_data, unscale_solution)
 *   third_party/osqp/lin_alg.h:17-208 (vector / csc kernels)
 *   third_party/osqp/osqp.h:32-178    (osqp_setup / solve / warm_start / update_*)
 * The KKT factorisation follows QDLDL's published up-looking LDL^T (etree + numeric
 * factor + L/D/L^T solves) on the quasi-definite KKT [[P+sigma I, A'],[A, -diag(1/rho)]],
 * as OSQP 0.6.2's default linear-system solver does; the fill-reducing ordering is an
 * exact minimum-degree ordering instead of SuiteSparse AMD (a different ordering changes
 * only rounding, ~1e-13 relative, per SURVEY.md 8c probe).
 *
 * No reference test or fixture pins an OSQP output for this path, and
 * the vendored binary may not be executed here, so this oracle is PARITY UNPINNED against
 * the reference itself.  It is pinned instead against analytic known-answer QPs
 * (tests/test_oracle.py) and serves as the independent checker for the HIP path.
 *
 * Deliberate, documented deviation: adaptive_rho_interval == 0 ("automatic") makes the
 * reference's rho-update cadence wall-clock dependent (solve time vs 0.4*setup time).  On
 * the reference's CPU that trigger fires within the first ~10-15 iterations for every
 * N=20..40 MPC QP, which c_roundmultiple() resolves to check_termination (25).  The oracle
 * (and the HIP path) therefore resolve interval 0 to check_termination (or 25 when
 * termination checking is disabled) deterministically.  time_limit is not modelled.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <pthread.h>

typedef long long c_int;
typedef double c_float;

/* constants.h:18-30, 59-119 */
#define OSQP_DUAL_INFEASIBLE_INACCURATE (4)
#define OSQP_PRIMAL_INFEASIBLE_INACCURATE (3)
#define OSQP_SOLVED_INACCURATE (2)
#define OSQP_SOLVED (1)
#define OSQP_MAX_ITER_REACHED (-2)
#define OSQP_PRIMAL_INFEASIBLE (-3)
#define OSQP_DUAL_INFEASIBLE (-4)
#define OSQP_NON_CVX (-7)
#define OSQP_UNSOLVED (-10)

#define OSQP_DATA_VALIDATION_ERROR 1
#define OSQP_SETTINGS_VALIDATION_ERROR 2
#define OSQP_LINSYS_SOLVER_INIT_ERROR 4
#define OSQP_NONCVX_ERROR 5
#define OSQP_MEM_ALLOC_ERROR 6
#define OSQP_WORKSPACE_NOT_INIT_ERROR 7

#define RHO_MIN (1e-06)
#define RHO_MAX (1e06)
#define RHO_EQ_OVER_RHO_INEQ (1e03)
#define RHO_TOL (1e-04)
#define CHECK_TERMINATION (25)
#define MIN_SCALING (1e-04)
#define MAX_SCALING (1e+04)
#define OSQP_NAN ((c_float)0x7fc00000UL)
#define OSQP_INFTY ((c_float)1e30)
#define OSQP_DIVISION_TOL ((c_float)1.0 / OSQP_INFTY)

/* Mirror of OSQPSettings, types.h:139-176 (PROFILING build, enum stored as c_int). */
typedef struct {
    c_float rho;
    c_float sigma;
    c_int scaling;
    c_int adaptive_rho;
    c_int adaptive_rho_interval;
    c_float adaptive_rho_tolerance;
    c_float adaptive_rho_fraction;
    c_int max_iter;
    c_float eps_abs;
    c_float eps_rel;
    c_float eps_prim_inf;
    c_float eps_dual_inf;
    c_float alpha;
    c_int linsys_solver;
    c_float delta;
    c_int polish;
    c_int polish_refine_iter;
    c_int verbose;
    c_int scaled_termination;
    c_int check_termination;
    c_int warm_start;
    c_float time_limit;
} ora_settings;

/* Subset of OSQPInfo (types.h:66-89) that the parity tests compare. */
typedef struct {
    c_int iter;
    c_int status_val;
    c_int rho_updates;
    c_int setup_exitflag; /* osqp_setup()'s return value (0 = ok) */
    c_float obj_val;
    c_float pri_res;
    c_float dua_res;
    c_float rho_estimate;
} ora_info;

typedef struct {
    c_int m, n;
    c_int *p, *i;
    c_float *x;
} ocsc;

/* ---------------------------------------------------------------- csc helpers */
static ocsc *csc_alloc(c_int m, c_int n, c_int nnz) {
    ocsc *A = (ocsc *)calloc(1, sizeof(ocsc));
    A->m = m;
    A->n = n;
    A->p = (c_int *)calloc((size_t)n + 1, sizeof(c_int));
    A->i = (c_int *)calloc((size_t)(nnz > 0 ? nnz : 1), sizeof(c_int));
    A->x = (c_float *)calloc((size_t)(nnz > 0 ? nnz : 1), sizeof(c_float));
    return A;
}
static void csc_free(ocsc *A) {
    if (!A) return;
    free(A->p);
    free(A->i);
    free(A->x);
    free(A);
}
static ocsc *csc_copy(c_int m, c_int n, const c_int *p, const c_int *i, const c_float *x) {
    c_int nnz = p[n];
    ocsc *A = csc_alloc(m, n, nnz);
    memcpy(A->p, p, sizeof(c_int) * (size_t)(n + 1));
    if (nnz) {
        memcpy(A->i, i, sizeof(c_int) * (size_t)nnz);
        memcpy(A->x, x, sizeof(c_float) * (size_t)nnz);
    }
    return A;
}

/* lin_alg.h:150 mat_vec (plus_eq = 0 / 1) */
static void mat_vec(const ocsc *A, const c_float *x, c_float *y, int plus_eq) {
    c_int i, j;
    if (!plus_eq)
        for (i = 0; i < A->m; i++) y[i] = 0;
    if (A->p[A->n] == 0) return;
    for (j = 0; j < A->n; j++)
        for (i = A->p[j]; i < A->p[j + 1]; i++) y[A->i[i]] += A->x[i] * x[j];
}
/* lin_alg.h:162 mat_tpose_vec (plus_eq = 0 / 1) */
static void mat_tpose_vec(const ocsc *A, const c_float *x, c_float *y, int plus_eq, int skip_diag) {
    c_int i, j, k;
    if (!plus_eq)
        for (i = 0; i < A->n; i++) y[i] = 0;
    if (A->p[A->n] == 0) return;
    if (skip_diag) {
        for (j = 0; j < A->n; j++)
            for (k = A->p[j]; k < A->p[j + 1]; k++) {
                i = A->i[k];
                y[j] += i == j ? 0 : A->x[k] * x[i];
            }
    } else {
        for (j = 0; j < A->n; j++)
            for (k = A->p[j]; k < A->p[j + 1]; k++) y[j] += A->x[k] * x[A->i[k]];
    }
}
static c_float vec_norm_inf(const c_float *v, c_int l) {
    c_float mx = 0.0;
    for (c_int i = 0; i < l; i++) {
        c_float a = fabs(v[i]);
        if (a > mx) mx = a;
    }
    return mx;
}
static c_float vec_scaled_norm_inf(const c_float *S, const c_float *v, c_int l) {
    c_float mx = 0.0;
    for (c_int i = 0; i < l; i++) {
        c_float a = fabs(S[i] * v[i]);
        if (a > mx) mx = a;
    }
    return mx;
}
static c_float vec_prod(const c_float *a, const c_float *b, c_int n) {
    c_float s = 0.0;
    for (c_int i = 0; i < n; i++) s += a[i] * b[i];
    return s;
}
static void limit_scaling(c_float *D, c_int n) {
    for (c_int i = 0; i < n; i++) {
        D[i] = D[i] < MIN_SCALING ? 1.0 : D[i];
        D[i] = D[i] > MAX_SCALING ? MAX_SCALING : D[i];
    }
}
/* lin_alg.h:197 mat_inf_norm_cols_sym_triu */
static void mat_inf_norm_cols_sym_triu(const ocsc *M, c_float *E) {
    c_int i, j, ptr;
    c_float abs_x;
    for (j = 0; j < M->n; j++) E[j] = 0.;
    for (j = 0; j < M->n; j++)
        for (ptr = M->p[j]; ptr < M->p[j + 1]; ptr++) {
            i = M->i[ptr];
            abs_x = fabs(M->x[ptr]);
            E[j] = abs_x > E[j] ? abs_x : E[j];
            if (i != j) E[i] = abs_x > E[i] ? abs_x : E[i];
        }
}
/* lin_alg.h:177 mat_inf_norm_cols */
static void mat_inf_norm_cols(const ocsc *M, c_float *E) {
    for (c_int j = 0; j < M->n; j++) {
        E[j] = 0.;
        for (c_int ptr = M->p[j]; ptr < M->p[j + 1]; ptr++) {
            c_float a = fabs(M->x[ptr]);
            E[j] = a > E[j] ? a : E[j];
        }
    }
}
/* lin_alg.h:186 mat_inf_norm_rows */
static void mat_inf_norm_rows(const ocsc *M, c_float *E) {
    for (c_int j = 0; j < M->m; j++) E[j] = 0.;
    for (c_int j = 0; j < M->n; j++)
        for (c_int ptr = M->p[j]; ptr < M->p[j + 1]; ptr++) {
            c_int i = M->i[ptr];
            c_float a = fabs(M->x[ptr]);
            E[i] = a > E[i] ? a : E[i];
        }
}
/* lin_alg.h:208 quad_form (upper-triangular P) */
static c_float quad_form(const ocsc *P, const c_float *x) {
    c_float qf = 0.;
    for (c_int j = 0; j < P->n; j++)
        for (c_int ptr = P->p[j]; ptr < P->p[j + 1]; ptr++) {
            c_int i = P->i[ptr];
            if (i == j)
                qf += (c_float).5 * P->x[ptr] * x[i] * x[i];
            else if (i < j)
                qf += P->x[ptr] * x[i] * x[j];
        }
    return qf;
}

/* ------------------------------------------------ minimum-degree ordering (AMD stand-in) */
/* Exact minimum-degree elimination on the symmetric pattern of an upper-CSC matrix.
 * Returns perm (perm[k] = original index eliminated k-th).  Ties -> lowest index. */
static void min_degree_order(const ocsc *K, c_int *perm) {
    c_int N = K->n, W = (N + 63) / 64;
    uint64_t *adj = (uint64_t *)calloc((size_t)N * (size_t)W, sizeof(uint64_t));
    c_int *deg = (c_int *)calloc((size_t)N, sizeof(c_int));
    char *alive = (char *)malloc((size_t)N);
    uint64_t *nb = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)W);
    memset(alive, 1, (size_t)N);
    for (c_int j = 0; j < N; j++)
        for (c_int k = K->p[j]; k < K->p[j + 1]; k++) {
            c_int i = K->i[k];
            if (i == j) continue;
            adj[i * W + j / 64] |= 1ULL << (j % 64);
            adj[j * W + i / 64] |= 1ULL << (i % 64);
        }
    for (c_int i = 0; i < N; i++) {
        c_int d = 0;
        for (c_int w = 0; w < W; w++) d += __builtin_popcountll(adj[i * W + w]);
        deg[i] = d;
    }
    for (c_int step = 0; step < N; step++) {
        c_int best = -1;
        for (c_int i = 0; i < N; i++)
            if (alive[i] && (best < 0 || deg[i] < deg[best])) best = i;
        perm[step] = best;
        alive[best] = 0;
        memcpy(nb, adj + best * W, sizeof(uint64_t) * (size_t)W);
        for (c_int w = 0; w < W; w++) {
            uint64_t bits = nb[w];
            while (bits) {
                int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                c_int u = w * 64 + b;
                uint64_t *ru = adj + u * W;
                for (c_int v = 0; v < W; v++) ru[v] |= nb[v];
                ru[u / 64] &= ~(1ULL << (u % 64));
                ru[best / 64] &= ~(1ULL << (best % 64));
                c_int d = 0;
                for (c_int v = 0; v < W; v++) d += __builtin_popcountll(ru[v]);
                deg[u] = d;
            }
        }
    }
    free(adj);
    free(deg);
    free(alive);
    free(nb);
}

/* C = upper(P A P') for an upper-CSC A, pinv[old] = new (CSparse cs_symperm semantics). */
static ocsc *csc_symperm_upper(const ocsc *A, const c_int *pinv) {
    c_int n = A->n, nz = A->p[n];
    ocsc *C = csc_alloc(n, n, nz);
    c_int *w = (c_int *)calloc((size_t)n, sizeof(c_int));
    for (c_int j = 0; j < n; j++) {
        c_int j2 = pinv[j];
        for (c_int p = A->p[j]; p < A->p[j + 1]; p++) {
            c_int i = A->i[p];
            if (i > j) continue;
            c_int i2 = pinv[i];
            w[i2 > j2 ? i2 : j2]++;
        }
    }
    C->p[0] = 0;
    for (c_int j = 0; j < n; j++) C->p[j + 1] = C->p[j] + w[j];
    for (c_int j = 0; j < n; j++) w[j] = C->p[j];
    for (c_int j = 0; j < n; j++) {
        c_int j2 = pinv[j];
        for (c_int p = A->p[j]; p < A->p[j + 1]; p++) {
            c_int i = A->i[p];
            if (i > j) continue;
            c_int i2 = pinv[i];
            c_int col = i2 > j2 ? i2 : j2, row = i2 < j2 ? i2 : j2;
            c_int q = w[col]++;
            C->i[q] = row;
            C->x[q] = A->x[p];
        }
    }
    free(w);
    /* sort row indices inside each column (QDLDL does not require it, kept for determinism) */
    for (c_int j = 0; j < n; j++)
        for (c_int a = C->p[j] + 1; a < C->p[j + 1]; a++) {
            c_int ri = C->i[a];
            c_float rx = C->x[a];
            c_int b = a - 1;
            while (b >= C->p[j] && C->i[b] > ri) {
                C->i[b + 1] = C->i[b];
                C->x[b + 1] = C->x[b];
                b--;
            }
            C->i[b + 1] = ri;
            C->x[b + 1] = rx;
        }
    return C;
}

/* ------------------------------------------------ QDLDL-style LDL^T (published algorithm) */
typedef struct {
    c_int n;
    c_int *etree, *Lnz, *Lp, *Li;
    c_float *Lx, *D, *Dinv;
    c_int *iwork;
    char *bwork;
    c_float *fwork;
} ldl_t;

static c_int ldl_etree(c_int n, const c_int *Ap, const c_int *Ai, c_int *work, c_int *Lnz, c_int *etree) {
    c_int sumLnz = 0;
    for (c_int i = 0; i < n; i++) {
        work[i] = 0;
        Lnz[i] = 0;
        etree[i] = -1;
    }
    for (c_int j = 0; j < n; j++) {
        work[j] = j;
        for (c_int p = Ap[j]; p < Ap[j + 1]; p++) {
            c_int i = Ai[p];
            if (i > j) return -1;
            while (work[i] != j) {
                if (etree[i] == -1) etree[i] = j;
                Lnz[i]++;
                work[i] = j;
                i = etree[i];
            }
        }
    }
    for (c_int i = 0; i < n; i++) sumLnz += Lnz[i];
    return sumLnz;
}

/* returns number of positive pivots, or -1 on a zero pivot */
static c_int ldl_factor(ldl_t *f, const c_int *Ap, const c_int *Ai, const c_float *Ax) {
    c_int n = f->n, positive = 0;
    c_int *yIdx = f->iwork, *elimBuffer = f->iwork + n, *LNext = f->iwork + 2 * n;
    char *yMarkers = f->bwork;
    c_float *yVals = f->fwork;
    f->Lp[0] = 0;
    for (c_int i = 0; i < n; i++) {
        f->Lp[i + 1] = f->Lp[i] + f->Lnz[i];
        yMarkers[i] = 0;
        yVals[i] = 0.0;
        f->D[i] = 0.0;
        LNext[i] = f->Lp[i];
    }
    f->D[0] = Ax[0];
    if (f->D[0] == 0.0) return -1;
    if (f->D[0] > 0.0) positive++;
    f->Dinv[0] = 1 / f->D[0];
    for (c_int k = 1; k < n; k++) {
        c_int nnzY = 0;
        for (c_int i = Ap[k]; i < Ap[k + 1]; i++) {
            c_int bidx = Ai[i];
            if (bidx == k) {
                f->D[k] = Ax[i];
                continue;
            }
            yVals[bidx] = Ax[i];
            c_int next = bidx;
            if (yMarkers[next] == 0) {
                yMarkers[next] = 1;
                elimBuffer[0] = next;
                c_int nnzE = 1;
                next = f->etree[bidx];
                while (next != -1 && next < k) {
                    if (yMarkers[next] == 1) break;
                    yMarkers[next] = 1;
                    elimBuffer[nnzE++] = next;
                    next = f->etree[next];
                }
                while (nnzE) yIdx[nnzY++] = elimBuffer[--nnzE];
            }
        }
        for (c_int i = nnzY - 1; i >= 0; i--) {
            c_int cidx = yIdx[i];
            c_int tmp = LNext[cidx];
            c_float yv = yVals[cidx];
            for (c_int j = f->Lp[cidx]; j < tmp; j++) yVals[f->Li[j]] -= f->Lx[j] * yv;
            f->Li[tmp] = k;
            f->Lx[tmp] = yv * f->Dinv[cidx];
            f->D[k] -= yv * f->Lx[tmp];
            LNext[cidx]++;
            yVals[cidx] = 0.0;
            yMarkers[cidx] = 0;
        }
        if (f->D[k] == 0.0) return -1;
        if (f->D[k] > 0.0) positive++;
        f->Dinv[k] = 1 / f->D[k];
    }
    return positive;
}
static void ldl_solve(const ldl_t *f, c_float *x) {
    c_int n = f->n;
    for (c_int i = 0; i < n; i++) {
        c_float v = x[i];
        for (c_int j = f->Lp[i]; j < f->Lp[i + 1]; j++) x[f->Li[j]] -= f->Lx[j] * v;
    }
    for (c_int i = 0; i < n; i++) x[i] *= f->Dinv[i];
    for (c_int i = n - 1; i >= 0; i--) {
        c_float v = x[i];
        for (c_int j = f->Lp[i]; j < f->Lp[i + 1]; j++) v -= f->Lx[j] * x[f->Li[j]];
        x[i] = v;
    }
}

/* --------------------------------------------------------------- workspace */
typedef struct {
    c_int n, m;
    ocsc *P, *A;
    c_float *q, *l, *u;
    ora_settings st;
    /* scaling (types.h:45-51) */
    int scaled;
    c_float c, cinv;
    c_float *D, *Dinv, *E, *Einv, *D_temp, *D_temp_A, *E_temp;
    /* rho */
    c_float *rho_vec, *rho_inv_vec;
    c_int *constr_type;
    /* iterates (types.h:211-251) */
    c_float *x, *y, *z, *xz_tilde, *x_prev, *z_prev;
    c_float *Ax, *Px, *Aty, *delta_y, *Atdelta_y, *delta_x, *Pdelta_x, *Adelta_x;
    /* linear system: permuted upper KKT + LDL^T */
    c_int nK;
    c_int *perm, *pinv;
    ldl_t ldl;
    c_float *bp, *sol;
    /* info */
    ora_info info;
    c_float *sol_x, *sol_y;
} ora_ws;

static void *xcalloc(c_int n, size_t sz) { return calloc((size_t)(n > 0 ? n : 1), sz); }

/* form_KKT (upper): cols 0..n-1: triu(P) + sigma on the diagonal; cols n..n+m-1: A' rows
 * then -1/rho_i on the diagonal.  Mirrors OSQP kkt.h form_KKT for QDLDL. */
static ocsc *form_kkt(const ora_ws *w) {
    c_int n = w->n, m = w->m, nK = n + m;
    c_int nnzP = w->P->p[n], nnzA = w->A->p[n];
    ocsc *K = csc_alloc(nK, nK, nnzP + n + nnzA + m);
    c_int z = 0;
    for (c_int j = 0; j < n; j++) {
        K->p[j] = z;
        int has_diag = 0;
        for (c_int k = w->P->p[j]; k < w->P->p[j + 1]; k++) {
            c_int i = w->P->i[k];
            if (i == j) {
                has_diag = 1;
                K->i[z] = i;
                K->x[z++] = w->P->x[k] + w->st.sigma;
            } else {
                K->i[z] = i;
                K->x[z++] = w->P->x[k];
            }
        }
        if (!has_diag) {
            K->i[z] = j;
            K->x[z++] = w->st.sigma;
        }
    }
    /* A' : column n+r holds row r of A; build row lists of A */
    c_int *cnt = (c_int *)xcalloc(m + 1, sizeof(c_int));
    for (c_int k = 0; k < nnzA; k++) cnt[w->A->i[k] + 1]++;
    for (c_int r = 0; r < m; r++) cnt[r + 1] += cnt[r];
    c_int *rp = (c_int *)xcalloc(m + 1, sizeof(c_int));
    memcpy(rp, cnt, sizeof(c_int) * (size_t)(m + 1));
    c_int *rj = (c_int *)xcalloc(nnzA, sizeof(c_int));
    c_float *rx = (c_float *)xcalloc(nnzA, sizeof(c_float));
    for (c_int j = 0; j < n; j++)
        for (c_int k = w->A->p[j]; k < w->A->p[j + 1]; k++) {
            c_int r = w->A->i[k];
            c_int q = rp[r]++;
            rj[q] = j;
            rx[q] = w->A->x[k];
        }
    for (c_int r = 0; r < m; r++) {
        K->p[n + r] = z;
        for (c_int q = cnt[r]; q < cnt[r + 1]; q++) {
            K->i[z] = rj[q];
            K->x[z++] = rx[q];
        }
        K->i[z] = n + r;
        K->x[z++] = -w->rho_inv_vec[r];
    }
    K->p[nK] = z;
    free(cnt);
    free(rp);
    free(rj);
    free(rx);
    return K;
}

static int linsys_factor(ora_ws *w) {
    ocsc *K = form_kkt(w);
    ocsc *KP = csc_symperm_upper(K, w->pinv);
    csc_free(K);
    c_int sumLnz = ldl_etree(w->nK, KP->p, KP->i, w->ldl.iwork, w->ldl.Lnz, w->ldl.etree);
    if (sumLnz < 0) {
        csc_free(KP);
        return -1;
    }
    free(w->ldl.Li);
    free(w->ldl.Lx);
    w->ldl.Li = (c_int *)xcalloc(sumLnz, sizeof(c_int));
    w->ldl.Lx = (c_float *)xcalloc(sumLnz, sizeof(c_float));
    c_int pos = ldl_factor(&w->ldl, KP->p, KP->i, KP->x);
    csc_free(KP);
    if (pos < 0 || pos != w->n) return -1; /* KKT not quasi-definite */
    return 0;
}

static int linsys_init(ora_ws *w) {
    c_int nK = w->n + w->m;
    w->nK = nK;
    w->perm = (c_int *)xcalloc(nK, sizeof(c_int));
    w->pinv = (c_int *)xcalloc(nK, sizeof(c_int));
    ocsc *K = form_kkt(w);
    min_degree_order(K, w->perm);
    csc_free(K);
    for (c_int k = 0; k < nK; k++) w->pinv[w->perm[k]] = k;
    w->ldl.n = nK;
    w->ldl.etree = (c_int *)xcalloc(nK, sizeof(c_int));
    w->ldl.Lnz = (c_int *)xcalloc(nK, sizeof(c_int));
    w->ldl.Lp = (c_int *)xcalloc(nK + 1, sizeof(c_int));
    w->ldl.D = (c_float *)xcalloc(nK, sizeof(c_float));
    w->ldl.Dinv = (c_float *)xcalloc(nK, sizeof(c_float));
    w->ldl.iwork = (c_int *)xcalloc(3 * nK, sizeof(c_int));
    w->ldl.bwork = (char *)xcalloc(nK, 1);
    w->ldl.fwork = (c_float *)xcalloc(nK, sizeof(c_float));
    w->ldl.Li = NULL;
    w->ldl.Lx = NULL;
    w->bp = (c_float *)xcalloc(nK, sizeof(c_float));
    w->sol = (c_float *)xcalloc(nK, sizeof(c_float));
    return linsys_factor(w);
}

/* qdldl_interface solve: sol = KKT^{-1} b; b[0:n] <- sol[0:n]; b[n+j] += rho_inv_j sol[n+j] */
static void linsys_solve(ora_ws *w, c_float *b) {
    c_int nK = w->nK;
    for (c_int j = 0; j < nK; j++) w->bp[j] = b[w->perm[j]];
    ldl_solve(&w->ldl, w->bp);
    for (c_int j = 0; j < nK; j++) w->sol[w->perm[j]] = w->bp[j];
    for (c_int j = 0; j < w->n; j++) b[j] = w->sol[j];
    for (c_int j = 0; j < w->m; j++) b[j + w->n] += w->rho_inv_vec[j] * w->sol[j + w->n];
}

/* ----------------------------------------------------------------- scaling.h */
static void scale_data(ora_ws *w) {
    c_int n = w->n, m = w->m;
    w->c = 1.0;
    for (c_int i = 0; i < n; i++) w->D[i] = w->Dinv[i] = 1.;
    for (c_int i = 0; i < m; i++) w->E[i] = w->Einv[i] = 1.;
    for (c_int it = 0; it < w->st.scaling; it++) {
        /* compute_inf_norm_cols_KKT */
        mat_inf_norm_cols_sym_triu(w->P, w->D_temp);
        mat_inf_norm_cols(w->A, w->D_temp_A);
        for (c_int i = 0; i < n; i++) w->D_temp[i] = w->D_temp[i] > w->D_temp_A[i] ? w->D_temp[i] : w->D_temp_A[i];
        mat_inf_norm_rows(w->A, w->E_temp);
        limit_scaling(w->D_temp, n);
        limit_scaling(w->E_temp, m);
        for (c_int i = 0; i < n; i++) w->D_temp[i] = sqrt(w->D_temp[i]);
        for (c_int i = 0; i < m; i++) w->E_temp[i] = sqrt(w->E_temp[i]);
        for (c_int i = 0; i < n; i++) w->D_temp[i] = 1.0 / w->D_temp[i];
        for (c_int i = 0; i < m; i++) w->E_temp[i] = 1.0 / w->E_temp[i];
        /* P <- D P D (mat_premult_diag then mat_postmult_diag) */
        for (c_int j = 0; j < n; j++)
            for (c_int k = w->P->p[j]; k < w->P->p[j + 1]; k++) w->P->x[k] *= w->D_temp[w->P->i[k]];
        for (c_int j = 0; j < n; j++)
            for (c_int k = w->P->p[j]; k < w->P->p[j + 1]; k++) w->P->x[k] *= w->D_temp[j];
        /* A <- E A D */
        for (c_int j = 0; j < n; j++)
            for (c_int k = w->A->p[j]; k < w->A->p[j + 1]; k++) w->A->x[k] *= w->E_temp[w->A->i[k]];
        for (c_int j = 0; j < n; j++)
            for (c_int k = w->A->p[j]; k < w->A->p[j + 1]; k++) w->A->x[k] *= w->D_temp[j];
        for (c_int i = 0; i < n; i++) w->q[i] = w->D_temp[i] * w->q[i];
        for (c_int i = 0; i < n; i++) w->D[i] = w->D[i] * w->D_temp[i];
        for (c_int i = 0; i < m; i++) w->E[i] = w->E[i] * w->E_temp[i];
        /* cost normalisation */
        mat_inf_norm_cols_sym_triu(w->P, w->D_temp);
        c_float c_temp = 0.0;
        for (c_int i = 0; i < n; i++) c_temp += w->D_temp[i];
        c_temp = c_temp / (c_float)n; /* vec_mean */
        c_float inf_norm_q = vec_norm_inf(w->q, n);
        limit_scaling(&inf_norm_q, 1);
        c_temp = c_temp > inf_norm_q ? c_temp : inf_norm_q;
        limit_scaling(&c_temp, 1);
        c_temp = 1. / c_temp;
        for (c_int k = 0; k < w->P->p[n]; k++) w->P->x[k] *= c_temp;
        for (c_int i = 0; i < n; i++) w->q[i] *= c_temp;
        w->c *= c_temp;
    }
    w->cinv = 1. / w->c;
    for (c_int i = 0; i < n; i++) w->Dinv[i] = 1. / w->D[i];
    for (c_int i = 0; i < m; i++) w->Einv[i] = 1. / w->E[i];
    for (c_int i = 0; i < m; i++) w->l[i] = w->E[i] * w->l[i];
    for (c_int i = 0; i < m; i++) w->u[i] = w->E[i] * w->u[i];
}

/* auxil.h:34 set_rho_vec */
static void set_rho_vec(ora_ws *w) {
    w->st.rho = fmin(fmax(w->st.rho, RHO_MIN), RHO_MAX);
    for (c_int i = 0; i < w->m; i++) {
        if ((w->l[i] < -OSQP_INFTY * MIN_SCALING) && (w->u[i] > OSQP_INFTY * MIN_SCALING)) {
            w->constr_type[i] = -1;
            w->rho_vec[i] = RHO_MIN;
        } else if (w->u[i] - w->l[i] < RHO_TOL) {
            w->constr_type[i] = 1;
            w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->st.rho;
        } else {
            w->constr_type[i] = 0;
            w->rho_vec[i] = w->st.rho;
        }
        w->rho_inv_vec[i] = 1. / w->rho_vec[i];
    }
}

/* auxil.h:43 update_rho_vec (called by osqp_update_bounds) */
static int update_rho_vec(ora_ws *w) {
    int changed = 0;
    for (c_int i = 0; i < w->m; i++) {
        if ((w->l[i] < -OSQP_INFTY * MIN_SCALING) && (w->u[i] > OSQP_INFTY * MIN_SCALING)) {
            if (w->constr_type[i] != -1) {
                w->constr_type[i] = -1;
                w->rho_vec[i] = RHO_MIN;
                w->rho_inv_vec[i] = 1. / RHO_MIN;
                changed = 1;
            }
        } else if (w->u[i] - w->l[i] < RHO_TOL) {
            if (w->constr_type[i] != 1) {
                w->constr_type[i] = 1;
                w->rho_vec[i] = w->st.rho * RHO_EQ_OVER_RHO_INEQ;
                w->rho_inv_vec[i] = 1. / w->rho_vec[i];
                changed = 1;
            }
        } else {
            if (w->constr_type[i] != 0) {
                w->constr_type[i] = 0;
                w->rho_vec[i] = w->st.rho;
                w->rho_inv_vec[i] = 1. / w->st.rho;
                changed = 1;
            }
        }
    }
    if (changed) return linsys_factor(w);
    return 0;
}

/* osqp.h:264 osqp_update_rho */
static int update_rho(ora_ws *w, c_float rho_new) {
    if (rho_new <= 0) return 1;
    w->st.rho = fmin(fmax(rho_new, RHO_MIN), RHO_MAX);
    for (c_int i = 0; i < w->m; i++) {
        if (w->constr_type[i] == 0) {
            w->rho_vec[i] = w->st.rho;
            w->rho_inv_vec[i] = 1. / w->st.rho;
        } else if (w->constr_type[i] == 1) {
            w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->st.rho;
            w->rho_inv_vec[i] = 1. / w->rho_vec[i];
        }
    }
    return linsys_factor(w);
}

/* ------------------------------------------------------------------ auxil.h */
static void cold_start(ora_ws *w) {
    memset(w->x, 0, sizeof(c_float) * (size_t)w->n);
    memset(w->z, 0, sizeof(c_float) * (size_t)w->m);
    memset(w->y, 0, sizeof(c_float) * (size_t)w->m);
}
static void update_xz_tilde(ora_ws *w) {
    c_int n = w->n, m = w->m;
    for (c_int i = 0; i < n; i++) w->xz_tilde[i] = w->st.sigma * w->x_prev[i] - w->q[i];
    for (c_int i = 0; i < m; i++) w->xz_tilde[i + n] = w->z_prev[i] - w->rho_inv_vec[i] * w->y[i];
    linsys_solve(w, w->xz_tilde);
}
static void update_x(ora_ws *w) {
    c_float a = w->st.alpha;
    for (c_int i = 0; i < w->n; i++) w->x[i] = a * w->xz_tilde[i] + ((c_float)1.0 - a) * w->x_prev[i];
    for (c_int i = 0; i < w->n; i++) w->delta_x[i] = w->x[i] - w->x_prev[i];
}
static void update_z(ora_ws *w) {
    c_float a = w->st.alpha;
    c_int n = w->n;
    for (c_int i = 0; i < w->m; i++) {
        w->z[i] = a * w->xz_tilde[i + n] + ((c_float)1.0 - a) * w->z_prev[i] + w->rho_inv_vec[i] * w->y[i];
    }
    /* project(): z = min(max(z, l), u) */
    for (c_int i = 0; i < w->m; i++) w->z[i] = fmin(fmax(w->z[i], w->l[i]), w->u[i]);
}
static void update_y(ora_ws *w) {
    c_float a = w->st.alpha;
    c_int n = w->n;
    for (c_int i = 0; i < w->m; i++) {
        w->delta_y[i] = w->rho_vec[i] * (a * w->xz_tilde[i + n] + ((c_float)1.0 - a) * w->z_prev[i] - w->z[i]);
        w->y[i] += w->delta_y[i];
    }
}
static c_float compute_obj_val(ora_ws *w, const c_float *x) {
    c_float obj = quad_form(w->P, x) + vec_prod(w->q, x, w->n);
    if (w->scaled) obj *= w->cinv;
    return obj;
}
static c_float compute_pri_res(ora_ws *w, const c_float *x, const c_float *z) {
    mat_vec(w->A, x, w->Ax, 0);
    for (c_int i = 0; i < w->m; i++) w->z_prev[i] = w->Ax[i] + -1 * z[i]; /* vec_add_scaled(.., -1) */
    if (w->scaled && !w->st.scaled_termination) return vec_scaled_norm_inf(w->Einv, w->z_prev, w->m);
    return vec_norm_inf(w->z_prev, w->m);
}
static c_float compute_pri_tol(ora_ws *w, c_float eps_abs, c_float eps_rel) {
    c_float mx, t;
    if (w->scaled && !w->st.scaled_termination) {
        mx = vec_scaled_norm_inf(w->Einv, w->z, w->m);
        t = vec_scaled_norm_inf(w->Einv, w->Ax, w->m);
    } else {
        mx = vec_norm_inf(w->z, w->m);
        t = vec_norm_inf(w->Ax, w->m);
    }
    mx = mx > t ? mx : t;
    return eps_abs + eps_rel * mx;
}
static c_float compute_dua_res(ora_ws *w, const c_float *x, const c_float *y) {
    c_int n = w->n;
    memcpy(w->x_prev, w->q, sizeof(c_float) * (size_t)n);
    mat_vec(w->P, x, w->Px, 0);
    mat_tpose_vec(w->P, x, w->Px, 1, 1);
    for (c_int i = 0; i < n; i++) w->x_prev[i] = w->x_prev[i] + 1 * w->Px[i];
    if (w->m > 0) {
        mat_tpose_vec(w->A, y, w->Aty, 0, 0);
        for (c_int i = 0; i < n; i++) w->x_prev[i] = w->x_prev[i] + 1 * w->Aty[i];
    }
    if (w->scaled && !w->st.scaled_termination) return w->cinv * vec_scaled_norm_inf(w->Dinv, w->x_prev, n);
    return vec_norm_inf(w->x_prev, n);
}
static c_float compute_dua_tol(ora_ws *w, c_float eps_abs, c_float eps_rel) {
    c_float mx, t;
    if (w->scaled && !w->st.scaled_termination) {
        mx = vec_scaled_norm_inf(w->Dinv, w->q, w->n);
        t = vec_scaled_norm_inf(w->Dinv, w->Aty, w->n);
        mx = mx > t ? mx : t;
        t = vec_scaled_norm_inf(w->Dinv, w->Px, w->n);
        mx = mx > t ? mx : t;
        mx *= w->cinv;
    } else {
        mx = vec_norm_inf(w->q, w->n);
        t = vec_norm_inf(w->Aty, w->n);
        mx = mx > t ? mx : t;
        t = vec_norm_inf(w->Px, w->n);
        mx = mx > t ? mx : t;
    }
    return eps_abs + eps_rel * mx;
}
static int is_primal_infeasible(ora_ws *w, c_float eps) {
    c_float norm_dy, ineq_lhs = 0.0;
    for (c_int i = 0; i < w->m; i++) {
        if (w->u[i] > OSQP_INFTY * MIN_SCALING) {
            if (w->l[i] < -OSQP_INFTY * MIN_SCALING)
                w->delta_y[i] = 0.0;
            else
                w->delta_y[i] = fmin(w->delta_y[i], 0.0);
        } else if (w->l[i] < -OSQP_INFTY * MIN_SCALING) {
            w->delta_y[i] = fmax(w->delta_y[i], 0.0);
        }
    }
    if (w->scaled && !w->st.scaled_termination) {
        for (c_int i = 0; i < w->m; i++) w->Adelta_x[i] = w->E[i] * w->delta_y[i];
        norm_dy = vec_norm_inf(w->Adelta_x, w->m);
    } else {
        norm_dy = vec_norm_inf(w->delta_y, w->m);
    }
    if (norm_dy > OSQP_DIVISION_TOL) {
        for (c_int i = 0; i < w->m; i++)
            ineq_lhs += w->u[i] * fmax(w->delta_y[i], 0) + w->l[i] * fmin(w->delta_y[i], 0);
        if (ineq_lhs < eps * norm_dy) {
            mat_tpose_vec(w->A, w->delta_y, w->Atdelta_y, 0, 0);
            if (w->scaled && !w->st.scaled_termination)
                for (c_int i = 0; i < w->n; i++) w->Atdelta_y[i] = w->Dinv[i] * w->Atdelta_y[i];
            return vec_norm_inf(w->Atdelta_y, w->n) < eps * norm_dy;
        }
    }
    return 0;
}
static int is_dual_infeasible(ora_ws *w, c_float eps) {
    c_float norm_dx, cost_scaling;
    if (w->scaled && !w->st.scaled_termination) {
        norm_dx = vec_scaled_norm_inf(w->D, w->delta_x, w->n);
        cost_scaling = w->c;
    } else {
        norm_dx = vec_norm_inf(w->delta_x, w->n);
        cost_scaling = 1.0;
    }
    if (norm_dx > OSQP_DIVISION_TOL) {
        if (vec_prod(w->q, w->delta_x, w->n) < cost_scaling * eps * norm_dx) {
            mat_vec(w->P, w->delta_x, w->Pdelta_x, 0);
            mat_tpose_vec(w->P, w->delta_x, w->Pdelta_x, 1, 1);
            if (w->scaled && !w->st.scaled_termination)
                for (c_int i = 0; i < w->n; i++) w->Pdelta_x[i] = w->Dinv[i] * w->Pdelta_x[i];
            if (vec_norm_inf(w->Pdelta_x, w->n) < cost_scaling * eps * norm_dx) {
                mat_vec(w->A, w->delta_x, w->Adelta_x, 0);
                if (w->scaled && !w->st.scaled_termination)
                    for (c_int i = 0; i < w->m; i++) w->Adelta_x[i] = w->Einv[i] * w->Adelta_x[i];
                for (c_int i = 0; i < w->m; i++) {
                    if (((w->u[i] < OSQP_INFTY * MIN_SCALING) && (w->Adelta_x[i] > eps * norm_dx)) ||
                        ((w->l[i] > -OSQP_INFTY * MIN_SCALING) && (w->Adelta_x[i] < -eps * norm_dx)))
                        return 0;
                }
                return 1;
            }
        }
    }
    return 0;
}
static int has_solution(const ora_info *info) {
    return (info->status_val != OSQP_PRIMAL_INFEASIBLE) && (info->status_val != OSQP_PRIMAL_INFEASIBLE_INACCURATE) &&
           (info->status_val != OSQP_DUAL_INFEASIBLE) && (info->status_val != OSQP_DUAL_INFEASIBLE_INACCURATE) &&
           (info->status_val != OSQP_NON_CVX);
}
static void update_info(ora_ws *w, c_int iter) {
    w->info.iter = iter;
    if (w->m == 0)
        w->info.pri_res = 0.;
    else
        w->info.pri_res = compute_pri_res(w, w->x, w->z);
    w->info.dua_res = compute_dua_res(w, w->x, w->y);
}
static int check_termination(ora_ws *w, int approximate) {
    c_float eps_prim, eps_dual;
    int prim_res_check = 0, dual_res_check = 0, prim_inf_check = 0, dual_inf_check = 0;
    c_float eps_abs = w->st.eps_abs, eps_rel = w->st.eps_rel;
    c_float eps_prim_inf = w->st.eps_prim_inf, eps_dual_inf = w->st.eps_dual_inf;
    if ((w->info.pri_res > OSQP_INFTY) || (w->info.dua_res > OSQP_INFTY)) {
        w->info.status_val = OSQP_NON_CVX;
        w->info.obj_val = OSQP_NAN;
        return 1;
    }
    if (approximate) {
        eps_abs *= 10;
        eps_rel *= 10;
        eps_prim_inf *= 10;
        eps_dual_inf *= 10;
    }
    if (w->m == 0) {
        prim_res_check = 1;
    } else {
        eps_prim = compute_pri_tol(w, eps_abs, eps_rel);
        if (w->info.pri_res < eps_prim)
            prim_res_check = 1;
        else
            prim_inf_check = is_primal_infeasible(w, eps_prim_inf);
    }
    eps_dual = compute_dua_tol(w, eps_abs, eps_rel);
    if (w->info.dua_res < eps_dual)
        dual_res_check = 1;
    else
        dual_inf_check = is_dual_infeasible(w, eps_dual_inf);

    if (prim_res_check && dual_res_check) {
        w->info.status_val = approximate ? OSQP_SOLVED_INACCURATE : OSQP_SOLVED;
        return 1;
    } else if (prim_inf_check) {
        w->info.status_val = approximate ? OSQP_PRIMAL_INFEASIBLE_INACCURATE : OSQP_PRIMAL_INFEASIBLE;
        if (w->scaled && !w->st.scaled_termination)
            for (c_int i = 0; i < w->m; i++) w->delta_y[i] = w->E[i] * w->delta_y[i];
        w->info.obj_val = OSQP_INFTY;
        return 1;
    } else if (dual_inf_check) {
        w->info.status_val = approximate ? OSQP_DUAL_INFEASIBLE_INACCURATE : OSQP_DUAL_INFEASIBLE;
        if (w->scaled && !w->st.scaled_termination)
            for (c_int i = 0; i < w->n; i++) w->delta_x[i] = w->D[i] * w->delta_x[i];
        w->info.obj_val = -OSQP_INFTY;
        return 1;
    }
    return 0;
}
static c_float compute_rho_estimate(ora_ws *w) {
    c_int n = w->n, m = w->m;
    c_float pri_res = vec_norm_inf(w->z_prev, m);
    c_float dua_res = vec_norm_inf(w->x_prev, n);
    c_float pn = vec_norm_inf(w->z, m), t = vec_norm_inf(w->Ax, m);
    pn = pn > t ? pn : t;
    pri_res /= (pn + OSQP_DIVISION_TOL);
    c_float dn = vec_norm_inf(w->q, n);
    t = vec_norm_inf(w->Aty, n);
    dn = dn > t ? dn : t;
    t = vec_norm_inf(w->Px, n);
    dn = dn > t ? dn : t;
    dua_res /= (dn + OSQP_DIVISION_TOL);
    c_float est = w->st.rho * sqrt(pri_res / (dua_res + OSQP_DIVISION_TOL));
    return fmin(fmax(est, RHO_MIN), RHO_MAX);
}
static int adapt_rho(ora_ws *w) {
    int exitflag = 0;
    c_float rho_new = compute_rho_estimate(w);
    w->info.rho_estimate = rho_new;
    if ((rho_new > w->st.rho * w->st.adaptive_rho_tolerance) || (rho_new < w->st.rho / w->st.adaptive_rho_tolerance)) {
        exitflag = update_rho(w, rho_new);
        w->info.rho_updates += 1;
    }
    return exitflag;
}
static void store_solution(ora_ws *w) {
    if (has_solution(&w->info)) {
        memcpy(w->sol_x, w->x, sizeof(c_float) * (size_t)w->n);
        memcpy(w->sol_y, w->y, sizeof(c_float) * (size_t)w->m);
        if (w->scaled) {
            for (c_int i = 0; i < w->n; i++) w->sol_x[i] = w->D[i] * w->sol_x[i];
            for (c_int i = 0; i < w->m; i++) w->sol_y[i] = w->E[i] * w->sol_y[i]; /* y = E y / c */
            for (c_int i = 0; i < w->m; i++) w->sol_y[i] *= w->cinv;
        }
    } else {
        for (c_int i = 0; i < w->n; i++) w->sol_x[i] = OSQP_NAN;
        for (c_int i = 0; i < w->m; i++) w->sol_y[i] = OSQP_NAN;
        cold_start(w);
    }
}

/* -------------------------------------------------------------- public API */
void ora_default_settings(ora_settings *s) {
    /* osqp.h:32 osqp_set_default_settings (constants.h:59-119) */
    s->rho = 0.1;
    s->sigma = 1e-06;
    s->scaling = 10;
    s->adaptive_rho = 1;
    s->adaptive_rho_interval = 0;
    s->adaptive_rho_tolerance = 5;
    s->adaptive_rho_fraction = 0.4;
    s->max_iter = 4000;
    s->eps_abs = 1e-3;
    s->eps_rel = 1e-3;
    s->eps_prim_inf = 1e-4;
    s->eps_dual_inf = 1e-4;
    s->alpha = 1.6;
    s->linsys_solver = 0;
    s->delta = 1e-6;
    s->polish = 0;
    s->polish_refine_iter = 3;
    s->verbose = 1;
    s->scaled_termination = 0;
    s->check_termination = 25;
    s->warm_start = 1;
    s->time_limit = 0;
}

static int validate_settings(const ora_settings *s) {
    if (s->rho <= 0.0 || s->sigma <= 0.0 || s->scaling < 0 || (s->adaptive_rho != 0 && s->adaptive_rho != 1) ||
        s->adaptive_rho_interval < 0 || s->adaptive_rho_fraction <= 0 || s->adaptive_rho_tolerance < 1.0 ||
        s->max_iter <= 0 || s->eps_abs < 0 || s->eps_rel < 0 || (s->eps_abs == 0 && s->eps_rel == 0) ||
        s->eps_prim_inf <= 0 || s->eps_dual_inf <= 0 || s->alpha <= 0 || s->alpha >= 2 || s->delta <= 0 ||
        (s->polish != 0 && s->polish != 1) || s->polish_refine_iter < 0 || (s->verbose != 0 && s->verbose != 1) ||
        (s->scaled_termination != 0 && s->scaled_termination != 1) || s->check_termination < 0 ||
        (s->warm_start != 0 && s->warm_start != 1) || s->time_limit < 0)
        return 1;
    return 0;
}

void ora_cleanup(ora_ws *w);

/* osqp.h:58 osqp_setup.  Returns 0 or an osqp_error_type. */
int ora_setup(ora_ws **wp, c_int n, c_int m, const c_int *Pp, const c_int *Pi, const c_float *Px, const c_float *q,
              const c_int *Ap, const c_int *Ai, const c_float *Ax, const c_float *l, const c_float *u,
              const ora_settings *s) {
    *wp = NULL;
    /* validate_data (auxil.h:164) */
    if (n <= 0 || m < 0) return OSQP_DATA_VALIDATION_ERROR;
    for (c_int j = 0; j < n; j++)
        for (c_int k = Pp[j]; k < Pp[j + 1]; k++)
            if (Pi[k] > j) return OSQP_DATA_VALIDATION_ERROR; /* P not upper triangular */
    for (c_int i = 0; i < m; i++)
        if (l[i] > u[i]) return OSQP_DATA_VALIDATION_ERROR;
    if (validate_settings(s)) return OSQP_SETTINGS_VALIDATION_ERROR;

    ora_ws *w = (ora_ws *)calloc(1, sizeof(ora_ws));
    w->n = n;
    w->m = m;
    w->st = *s;
    w->P = csc_copy(n, n, Pp, Pi, Px);
    w->A = csc_copy(m, n, Ap, Ai, Ax);
    w->q = (c_float *)xcalloc(n, sizeof(c_float));
    w->l = (c_float *)xcalloc(m, sizeof(c_float));
    w->u = (c_float *)xcalloc(m, sizeof(c_float));
    memcpy(w->q, q, sizeof(c_float) * (size_t)n);
    for (c_int i = 0; i < m; i++) {
        w->l[i] = fmin(fmax(l[i], -OSQP_INFTY), OSQP_INFTY);
        w->u[i] = fmin(fmax(u[i], -OSQP_INFTY), OSQP_INFTY);
    }
#define ALN(v, k) w->v = (c_float *)xcalloc(k, sizeof(c_float))
    ALN(rho_vec, m);
    ALN(rho_inv_vec, m);
    w->constr_type = (c_int *)xcalloc(m, sizeof(c_int));
    ALN(x, n);
    ALN(z, m);
    ALN(xz_tilde, n + m);
    ALN(x_prev, n);
    ALN(z_prev, m);
    ALN(y, m);
    ALN(Ax, m);
    ALN(Px, n);
    ALN(Aty, n);
    ALN(delta_y, m);
    ALN(Atdelta_y, n);
    ALN(delta_x, n);
    ALN(Pdelta_x, n);
    ALN(Adelta_x, m);
    ALN(D, n);
    ALN(Dinv, n);
    ALN(E, m);
    ALN(Einv, m);
    ALN(D_temp, n);
    ALN(D_temp_A, n);
    ALN(E_temp, m);
    ALN(sol_x, n);
    ALN(sol_y, m);
#undef ALN
    cold_start(w);
    w->c = w->cinv = 1.0;
    if (s->scaling) {
        w->scaled = 1;
        scale_data(w);
    } else {
        w->scaled = 0;
    }
    set_rho_vec(w);
    if (linsys_init(w)) {
        ora_cleanup(w);
        return OSQP_NONCVX_ERROR;
    }
    w->info.status_val = OSQP_UNSOLVED;
    w->info.rho_updates = 0;
    w->info.rho_estimate = w->st.rho;
    *wp = w;
    return 0;
}

/* osqp.h:157 osqp_warm_start */
int ora_warm_start(ora_ws *w, const c_float *x, const c_float *y) {
    if (!w) return OSQP_WORKSPACE_NOT_INIT_ERROR;
    if (!w->st.warm_start) w->st.warm_start = 1;
    memcpy(w->x, x, sizeof(c_float) * (size_t)w->n);
    memcpy(w->y, y, sizeof(c_float) * (size_t)w->m);
    if (w->scaled) {
        for (c_int i = 0; i < w->n; i++) w->x[i] = w->Dinv[i] * w->x[i];
        for (c_int i = 0; i < w->m; i++) w->y[i] = w->Einv[i] * w->y[i];
        for (c_int i = 0; i < w->m; i++) w->y[i] *= w->c;
    }
    mat_vec(w->A, w->x, w->z, 0);
    return 0;
}

/* osqp.h:114 osqp_update_lin_cost */
int ora_update_lin_cost(ora_ws *w, const c_float *q_new) {
    memcpy(w->q, q_new, sizeof(c_float) * (size_t)w->n);
    if (w->scaled) {
        for (c_int i = 0; i < w->n; i++) w->q[i] = w->D[i] * w->q[i];
        for (c_int i = 0; i < w->n; i++) w->q[i] *= w->c;
    }
    w->info.status_val = OSQP_UNSOLVED;
    w->info.rho_updates = 0;
    return 0;
}

/* osqp.h:125 osqp_update_bounds (bounds clamped to +-OSQP_INFTY as at setup) */
int ora_update_bounds(ora_ws *w, const c_float *l_new, const c_float *u_new) {
    for (c_int i = 0; i < w->m; i++)
        if (l_new[i] > u_new[i]) return 1;
    for (c_int i = 0; i < w->m; i++) {
        w->l[i] = fmin(fmax(l_new[i], -OSQP_INFTY), OSQP_INFTY);
        w->u[i] = fmin(fmax(u_new[i], -OSQP_INFTY), OSQP_INFTY);
    }
    if (w->scaled) {
        for (c_int i = 0; i < w->m; i++) w->l[i] = w->E[i] * w->l[i];
        for (c_int i = 0; i < w->m; i++) w->u[i] = w->E[i] * w->u[i];
    }
    w->info.status_val = OSQP_UNSOLVED;
    w->info.rho_updates = 0;
    return update_rho_vec(w);
}

/* scaling.h:40 unscale_data: P, q, A, l, u back to the problem's own units */
static void unscale_data(ora_ws *w) {
    c_int n = w->n, m = w->m;
    for (c_int k = 0; k < w->P->p[n]; k++) w->P->x[k] *= w->cinv;                       /* mat_mult_scalar */
    for (c_int j = 0; j < n; j++)                                                        /* mat_premult_diag */
        for (c_int k = w->P->p[j]; k < w->P->p[j + 1]; k++) w->P->x[k] *= w->Dinv[w->P->i[k]];
    for (c_int j = 0; j < n; j++)                                                        /* mat_postmult_diag */
        for (c_int k = w->P->p[j]; k < w->P->p[j + 1]; k++) w->P->x[k] *= w->Dinv[j];
    for (c_int i = 0; i < n; i++) w->q[i] *= w->cinv;
    for (c_int i = 0; i < n; i++) w->q[i] = w->Dinv[i] * w->q[i];
    for (c_int j = 0; j < n; j++)
        for (c_int k = w->A->p[j]; k < w->A->p[j + 1]; k++) w->A->x[k] *= w->Einv[w->A->i[k]];
    for (c_int j = 0; j < n; j++)
        for (c_int k = w->A->p[j]; k < w->A->p[j + 1]; k++) w->A->x[k] *= w->Dinv[j];
    for (c_int i = 0; i < m; i++) w->l[i] = w->Einv[i] * w->l[i];
    for (c_int i = 0; i < m; i++) w->u[i] = w->Einv[i] * w->u[i];
}

/* osqp.h:137 / :147 osqp_update_P / osqp_update_A with every value (Px_new_idx = OSQP_NULL):
 * unscale_data, the new values, scale_data, update_matrices (refactor with the current rho_vec),
 * reset_info.  The iterates x, z, y stay as they are (scaled with the old scaling). */
static int update_matrix(ora_ws *w, const c_float *Px_new, const c_float *Ax_new) {
    if (!w) return OSQP_WORKSPACE_NOT_INIT_ERROR;
    if (w->scaled) unscale_data(w);
    if (Px_new) memcpy(w->P->x, Px_new, sizeof(c_float) * (size_t)w->P->p[w->n]);
    if (Ax_new) memcpy(w->A->x, Ax_new, sizeof(c_float) * (size_t)w->A->p[w->n]);
    if (w->scaled) scale_data(w);
    if (linsys_factor(w)) return OSQP_NONCVX_ERROR;
    w->info.status_val = OSQP_UNSOLVED;
    w->info.rho_updates = 0;
    return 0;
}
/* Study variant (tools / tests only, not OSQP): replace P, q, A, l, u by raw values and scale them
 * afresh from the problem's own units -- no unscale round trip of the old scaled data -- keeping
 * rho and the scaled iterates; the row types follow the new scaled bounds. */
int ora_rescale_raw(ora_ws *w, const c_float *Px, const c_float *q, const c_float *Ax, const c_float *l,
                    const c_float *u) {
    if (!w) return OSQP_WORKSPACE_NOT_INIT_ERROR;
    memcpy(w->P->x, Px, sizeof(c_float) * (size_t)w->P->p[w->n]);
    memcpy(w->A->x, Ax, sizeof(c_float) * (size_t)w->A->p[w->n]);
    memcpy(w->q, q, sizeof(c_float) * (size_t)w->n);
    for (c_int i = 0; i < w->m; i++) {
        w->l[i] = fmin(fmax(l[i], -OSQP_INFTY), OSQP_INFTY);
        w->u[i] = fmin(fmax(u[i], -OSQP_INFTY), OSQP_INFTY);
    }
    if (w->scaled) scale_data(w);
    update_rho_vec(w);
    if (linsys_factor(w)) return OSQP_NONCVX_ERROR;
    w->info.status_val = OSQP_UNSOLVED;
    w->info.rho_updates = 0;
    return 0;
}
int ora_update_P(ora_ws *w, const c_float *Px_new) { return update_matrix(w, Px_new, NULL); }
int ora_update_A(ora_ws *w, const c_float *Ax_new) { return update_matrix(w, NULL, Ax_new); }
int ora_update_P_A(ora_ws *w, const c_float *Px_new, const c_float *Ax_new) { return update_matrix(w, Px_new, Ax_new); }

/* osqp.h:78 osqp_solve */
int ora_solve_ws(ora_ws *w) {
    int exitflag = 0, can_check_termination = 0;
    c_int iter;
    if (!w) return OSQP_WORKSPACE_NOT_INIT_ERROR;
    if (!w->st.warm_start) cold_start(w);
    c_int rho_interval = w->st.adaptive_rho_interval;
    if (w->st.adaptive_rho && rho_interval == 0)
        rho_interval = w->st.check_termination ? w->st.check_termination : CHECK_TERMINATION;
    for (iter = 1; iter <= w->st.max_iter; iter++) {
        c_float *t = w->x;
        w->x = w->x_prev;
        w->x_prev = t;
        t = w->z;
        w->z = w->z_prev;
        w->z_prev = t;
        update_xz_tilde(w);
        update_x(w);
        update_z(w);
        update_y(w);
        can_check_termination = w->st.check_termination && (iter % w->st.check_termination == 0);
        if (can_check_termination) {
            update_info(w, iter);
            if (check_termination(w, 0)) break;
        }
        if (w->st.adaptive_rho && rho_interval && (iter % rho_interval == 0)) {
            if (!can_check_termination) update_info(w, iter);
            if (adapt_rho(w)) {
                exitflag = 1;
                return exitflag;
            }
        }
    }
    if (!can_check_termination) {
        update_info(w, iter - 1);
        check_termination(w, 0);
    }
    if (has_solution(&w->info)) w->info.obj_val = compute_obj_val(w, w->x);
    if (w->info.status_val == OSQP_UNSOLVED) {
        if (!check_termination(w, 1)) w->info.status_val = OSQP_MAX_ITER_REACHED;
    }
    w->info.rho_estimate = compute_rho_estimate(w);
    store_solution(w);
    return exitflag;
}

void ora_get(const ora_ws *w, c_float *x, c_float *y, ora_info *info) {
    if (x) memcpy(x, w->sol_x, sizeof(c_float) * (size_t)w->n);
    if (y) memcpy(y, w->sol_y, sizeof(c_float) * (size_t)w->m);
    if (info) *info = w->info;
}

/* Unscaled (x, y) iterates, for the persistent-workspace tests. */
void ora_get_iterates(const ora_ws *w, c_float *x, c_float *y) {
    for (c_int i = 0; i < w->n; i++) x[i] = w->scaled ? w->D[i] * w->x[i] : w->x[i];
    for (c_int i = 0; i < w->m; i++) y[i] = w->scaled ? w->E[i] * w->y[i] * w->cinv : w->y[i];
}

/* Test-only state transfer (not an OSQP call): the workspace's SCALED iterates work->x, z, y and
 * settings->rho (types.h:182-289).  ora_set_state loads another solver's persisted state -- the
 * device's persistent workspace (impc_batch_get_persistent) -- into this workspace before the next
 * update / solve, as osqp_update_rho (osqp.h:264) would set rho: rho_vec by constraint type and a
 * refactorisation.  The closed-loop parity tests re-synchronise the oracle with it at every step,
 * so each step is compared from the same starting point. */
void ora_get_state(const ora_ws *w, c_float *rho, c_float *x, c_float *z, c_float *y) {
    if (rho) *rho = w->st.rho;
    if (x) memcpy(x, w->x, sizeof(c_float) * (size_t)w->n);
    if (z) memcpy(z, w->z, sizeof(c_float) * (size_t)w->m);
    if (y) memcpy(y, w->y, sizeof(c_float) * (size_t)w->m);
}
int ora_set_state(ora_ws *w, c_float rho, const c_float *x, const c_float *z, const c_float *y) {
    if (!w) return OSQP_WORKSPACE_NOT_INIT_ERROR;
    memcpy(w->x, x, sizeof(c_float) * (size_t)w->n);
    memcpy(w->z, z, sizeof(c_float) * (size_t)w->m);
    memcpy(w->y, y, sizeof(c_float) * (size_t)w->m);
    if (rho != w->st.rho) return update_rho(w, rho) ? OSQP_NONCVX_ERROR : 0;
    return 0;
}

/* The state osqp_setup leaves in the workspace (types.h:182-289): rho_vec, constr_type, the
 * scaling vectors D, E and the cost scale c -- compared in tests/test_oracle.py with the facts the
 * survey's probe read from the reference libosqp.so's OSQPWorkspace after osqp_setup (SURVEY.md
 * 8a row a9). */
void ora_get_setup(const ora_ws *w, c_float *rho_vec, c_int *constr_type, c_float *D, c_float *E, c_float *c) {
    if (rho_vec) memcpy(rho_vec, w->rho_vec, sizeof(c_float) * (size_t)w->m);
    if (constr_type) memcpy(constr_type, w->constr_type, sizeof(c_int) * (size_t)w->m);
    for (c_int i = 0; D && i < w->n; i++) D[i] = w->scaled ? w->D[i] : 1.0;
    for (c_int i = 0; E && i < w->m; i++) E[i] = w->scaled ? w->E[i] : 1.0;
    if (c) *c = w->scaled ? w->c : 1.0;
}

void ora_cleanup(ora_ws *w) {
    if (!w) return;
    csc_free(w->P);
    csc_free(w->A);
    void *ptrs[] = {w->q, w->l, w->u, w->D, w->Dinv, w->E, w->Einv, w->D_temp, w->D_temp_A, w->E_temp,
                    w->rho_vec, w->rho_inv_vec, w->constr_type, w->x, w->y, w->z, w->xz_tilde, w->x_prev,
                    w->z_prev, w->Ax, w->Px, w->Aty, w->delta_y, w->Atdelta_y, w->delta_x, w->Pdelta_x,
                    w->Adelta_x, w->perm, w->pinv, w->ldl.etree, w->ldl.Lnz, w->ldl.Lp, w->ldl.Li, w->ldl.Lx,
                    w->ldl.D, w->ldl.Dinv, w->ldl.iwork, w->ldl.bwork, w->ldl.fwork, w->bp, w->sol, w->sol_x,
                    w->sol_y};
    for (size_t k = 0; k < sizeof(ptrs) / sizeof(ptrs[0]); k++) free(ptrs[k]);
    free(w);
}

/* One QP, the reference's per-call pattern (mpcPlanner.cpp:436-527):
 * osqp_setup -> [osqp_warm_start(x_ws, y_ws)] -> osqp_solve -> read solution -> cleanup. */
int ora_solve(c_int n, c_int m, const c_int *Pp, const c_int *Pi, const c_float *Px, const c_float *q,
              const c_int *Ap, const c_int *Ai, const c_float *Ax, const c_float *l, const c_float *u,
              const ora_settings *s, const c_float *x_ws, const c_float *y_ws, c_float *x_out, c_float *y_out,
              ora_info *info) {
    ora_ws *w = NULL;
    int e = ora_setup(&w, n, m, Pp, Pi, Px, q, Ap, Ai, Ax, l, u, s);
    if (e) {
        if (info) {
            memset(info, 0, sizeof(*info));
            info->setup_exitflag = e;
            info->status_val = OSQP_UNSOLVED;
        }
        return e;
    }
    if (x_ws && y_ws) ora_warm_start(w, x_ws, y_ws);
    int ef = ora_solve_ws(w);
    ora_get(w, x_out, y_out, info);
    ora_cleanup(w);
    return ef;
}

/* ----------------------------------------------------------- batch driver */
typedef struct {
    c_int n, m;
    const c_int *Pp, *Pi, *Ap, *Ai;
    const c_float *Px, *q, *Ax, *l, *u, *xw, *yw;
    const ora_settings *s;
    c_float *xo, *yo;
    ora_info *info;
    c_int nnzP, nnzA, b0, b1;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *j = (batch_job *)arg;
    for (c_int b = j->b0; b < j->b1; b++) {
        ora_solve(j->n, j->m, j->Pp, j->Pi, j->Px + b * j->nnzP, j->q + b * j->n, j->Ap, j->Ai, j->Ax + b * j->nnzA,
                  j->l + b * j->m, j->u + b * j->m, j->s, j->xw ? j->xw + b * j->n : NULL,
                  j->yw ? j->yw + b * j->m : NULL, j->xo + b * j->n, j->yo + b * j->m, j->info + b);
    }
    return NULL;
}

/* Batch of QPs sharing one sparsity pattern; per-QP arrays QP-major (QP b at offset b*len).
 * Solved one QP at a time per thread with the reference's per-call pattern. */
int ora_solve_batch(c_int nb, c_int n, c_int m, const c_int *Pp, const c_int *Pi, const c_float *Px, const c_float *q,
                    const c_int *Ap, const c_int *Ai, const c_float *Ax, const c_float *l, const c_float *u,
                    const ora_settings *s, const c_float *x_ws, const c_float *y_ws, c_float *x_out, c_float *y_out,
                    ora_info *info, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > nb) nthreads = (int)(nb > 0 ? nb : 1);
    pthread_t th[256];
    batch_job jobs[256];
    if (nthreads > 256) nthreads = 256;
    c_int per = (nb + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        batch_job *j = &jobs[t];
        j->n = n;
        j->m = m;
        j->Pp = Pp;
        j->Pi = Pi;
        j->Ap = Ap;
        j->Ai = Ai;
        j->Px = Px;
        j->q = q;
        j->Ax = Ax;
        j->l = l;
        j->u = u;
        j->xw = x_ws;
        j->yw = y_ws;
        j->s = s;
        j->xo = x_out;
        j->yo = y_out;
        j->info = info;
        j->nnzP = Pp[n];
        j->nnzA = Ap[n];
        j->b0 = t * per;
        j->b1 = (t + 1) * per < nb ? (t + 1) * per : nb;
        if (j->b0 > j->b1) j->b0 = j->b1;
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    batch_worker(&jobs[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    return 0;
}
