/*
 * OsqpEigen/OsqpEigen.h -- OsqpEigen-compatible C++ front end of libimpc_qp.so (header only).
 *
 * Lets the reference's caller compile unchanged against the MI355X solver: mpcPlanner.h includes
 * <trajectory_planner/third_party/OsqpEigen/OsqpEigen.h> (reference mpcPlanner.h:22); pointing that
 * include at this header keeps every call in mpcPlanner::solveTraj
 * (mpcPlanner.cpp:436-527) as it is.  Mirrors the OsqpEigen 0.7 surface the reference uses:
 *
 *   OsqpEigen::Settings  (Settings.hpp:25-202)  setVerbosity, setWarmStart, setTimeLimit, ... ->
 *                                               impc_settings (OSQPSettings mirror)
 *   OsqpEigen::Data      (Data.hpp:44-151)      setNumberOf*, setHessianMatrix (upper triangle,
 *                                               Data.tpp:38), setGradient, setLinearConstraints-
 *                                               Matrix, setLower/UpperBound, getGradient,
 *                                               getData (OSQP's OSQPData view)
 *   OsqpEigen::Solver    (Solver.hpp:87-249)    initSolver, setWarmStart, solveProblem, getStatus,
 *                                               getSolution, getDualSolution, clearSolver,
 *                                               clearSolverVariables, updateGradient /
 *                                               updateLower|UpperBound / updateBounds,
 *                                               updateHessianMatrix / updateLinearConstraintsMatrix,
 *                                               set|getPrimalVariable, set|getDualVariable
 *   Status / ErrorExitFlag values               (Constants.hpp:14-56, OSQP constants.h:18-51)
 *
 * Each Solver owns a one-QP batch on a process-wide context (device IMPC_DEVICE, default 0); the
 * context belongs to the thread that first initialises a solver (the reference's single mpc
 * worker thread, mpcNavigation.cpp:177-178).  The batch comes from the context's workspace pool
 * (impc_batch_acquire / impc_batch_release): solveTraj builds a new Solver on every call
 * (mpcPlanner.cpp:436, :527), and a Solver on a pattern the process has seen before takes a
 * released batch's device buffers and analysis instead of allocating and analysing again
 * (IMPC_SHIM_NOPOOL=1 creates and destroys a batch per Solver instead, for comparison).  Differences from OsqpEigen, all benign for the
 * reference's call pattern: Data copies vectors when they are set (OsqpEigen keeps the caller's
 * pointer until initSolver); osqp_setup's numeric work runs on the device at the first solve, so
 * a non-convex P surfaces as ErrorExitFlag::NonCvxError from solveProblem instead of a failed
 * initSolver; the update* calls keep OSQP's workspace semantics on both kernels (scaling, rho,
 * factor and iterates carried over: the structured kernel through a persistent workspace,
 * impc_batch_set_persistent, the generic kernel in place).  An update before the first solve
 * (on either kernel), or on a structured batch whose settings exceed the persistent workspace's
 * 20 Ruiz passes, re-runs setup from the new data instead, warm-started from the last solution.
 * The argument types are the reference declarations' (Eigen::Ref, SparseCompressedBase, the
 * fixed-size Matrix<T, n, 1> templates of Solver.hpp:217-231); this repository compiles the
 * header against a test-only Eigen stand-in (tests/native/mock_eigen), since Eigen 3.3 is not in
 * the image -- real-Eigen template deduction is therefore unverified here.
 *
 * Requires Eigen's <Eigen/Dense> and <Eigen/Sparse> (the reference's own dependency) and
 * linking against intent-mpc_amd/lib/libimpc_qp.so.
 */
#ifndef IMPC_OSQPEIGEN_SHIM_H
#define IMPC_OSQPEIGEN_SHIM_H

#include <Eigen/Dense>
#include <Eigen/Sparse>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <utility>
#include <vector>

#include "../impc_qp.h"

/* OSQP 0.6.2's public data types (osqp/include/types.h, glob_opts.h with DLONG / no DFLOAT), the
 * return type of Data::getData(); skipped when the real osqp.h came first. */
#ifndef OSQP_TYPES_H
typedef long long c_int;
typedef double c_float;
typedef struct {
    c_int nzmax;
    c_int m;
    c_int n;
    c_int *p;
    c_int *i;
    c_float *x;
    c_int nz;
} csc;
typedef struct {
    c_int n;
    c_int m;
    csc *P;
    csc *A;
    c_float *q;
    c_float *l;
    c_float *u;
} OSQPData;
#endif
static_assert(sizeof(c_int) == sizeof(int64_t), "OSQPData views the shim's int64 index arrays");

namespace OsqpEigen {

constexpr double INFTY = 1e30; /* OSQP_INFTY */

enum class Status : int {
    DualInfeasibleInaccurate = IMPC_DUAL_INFEASIBLE_INACCURATE,
    PrimalInfeasibleInaccurate = IMPC_PRIMAL_INFEASIBLE_INACCURATE,
    SolvedInaccurate = IMPC_SOLVED_INACCURATE,
    Solved = IMPC_SOLVED,
    MaxIterReached = IMPC_MAX_ITER_REACHED,
    PrimalInfeasible = IMPC_PRIMAL_INFEASIBLE,
    DualInfeasible = IMPC_DUAL_INFEASIBLE,
    Sigint = -5,
    TimeLimitReached = IMPC_TIME_LIMIT_REACHED,
    NonCvx = IMPC_NON_CVX,
    Unsolved = IMPC_UNSOLVED
};

enum class ErrorExitFlag : int {
    NoError = 0,
    DataValidationError = IMPC_DATA_VALIDATION_ERROR,
    SettingsValidationError = IMPC_SETTINGS_VALIDATION_ERROR,
    LinsysSolverLoadError = 3,
    LinsysSolverInitError = IMPC_LINSYS_SOLVER_INIT_ERROR,
    NonCvxError = IMPC_NONCVX_ERROR,
    MemAllocError = IMPC_MEM_ALLOC_ERROR,
    WorkspaceNotInitError = IMPC_WORKSPACE_NOT_INIT_ERROR
};

namespace detail {

inline void debug(const char *what) { std::fprintf(stderr, "[OsqpEigen/impc] %s\n", what); }

inline void debug_impc(const char *what, int rc) {
    std::fprintf(stderr, "[OsqpEigen/impc] %s failed (%d): %s\n", what, rc, impc_last_error());
}

/* Workspace pool off (IMPC_SHIM_NOPOOL=1): a batch is created and destroyed per Solver. */
inline bool no_pool() {
    static const bool off = [] {
        const char *e = std::getenv("IMPC_SHIM_NOPOOL");
        return e && e[0] == '1';
    }();
    return off;
}

/* Process-wide context, created on first use. */
inline impc_ctx context() {
    static impc_ctx ctx = [] {
        impc_ctx c = nullptr;
        const char *dev = std::getenv("IMPC_DEVICE");
        int rc = impc_ctx_create(dev ? std::atoi(dev) : 0, &c);
        if (rc) debug_impc("impc_ctx_create", rc);
        return rc ? nullptr : c;
    }();
    return ctx;
}

/* CSC copy of an Eigen sparse matrix (stored entries, explicit zeros kept, rows sorted), optionally
 * only the upper triangle (OsqpEigen Data.tpp:38, SparseMatrixHelper.tpp:11-58). */
template <typename Derived>
void to_csc(const Derived &M, bool upper, std::vector<int64_t> &p, std::vector<int64_t> &i, std::vector<double> &x) {
    const int64_t cols = (int64_t)M.cols();
    std::vector<std::vector<std::pair<int64_t, double>>> colv((size_t)cols);
    for (int64_t k = 0; k < (int64_t)M.outerSize(); ++k)
        for (typename Derived::InnerIterator it(M, k); it; ++it) {
            const int64_t r = (int64_t)it.row(), c = (int64_t)it.col();
            if (upper && r > c) continue;
            colv[(size_t)c].emplace_back(r, (double)it.value());
        }
    p.assign(1, 0);
    i.clear();
    x.clear();
    for (auto &cv : colv) {
        std::sort(cv.begin(), cv.end(), [](const std::pair<int64_t, double> &a, const std::pair<int64_t, double> &b) {
            return a.first < b.first;
        });
        for (auto &e : cv) {
            i.push_back(e.first);
            x.push_back(e.second);
        }
        p.push_back((int64_t)i.size());
    }
}

template <typename V>
bool copy_vec(const V &v, int64_t n, std::vector<double> &out) {
    if ((int64_t)v.size() != n) return false;
    out.resize((size_t)n);
    for (int64_t k = 0; k < n; ++k) out[(size_t)k] = (double)v((int)k);
    return true;
}

}  // namespace detail

class Settings {
    impc_settings m_s;

public:
    Settings() { resetDefaultSettings(); }
    void resetDefaultSettings() { impc_default_settings(&m_s); }
    void setRho(const double v) { m_s.rho = v; }
    void setSigma(const double v) { m_s.sigma = v; }
    void setScaling(const int v) { m_s.scaling = v; }
    void setAdaptiveRho(const bool v) { m_s.adaptive_rho = v ? 1 : 0; }
    void setAdaptiveRhoInterval(const int v) { m_s.adaptive_rho_interval = v; }
    void setAdaptiveRhoTolerance(const double v) { m_s.adaptive_rho_tolerance = v; }
    void setAdaptiveRhoFraction(const double v) { m_s.adaptive_rho_fraction = v; }
    void setMaxIteration(const int v) { m_s.max_iter = v; }
    void setMaxIteraction(const int v) { m_s.max_iter = v; }
    void setAbsoluteTolerance(const double v) { m_s.eps_abs = v; }
    void setRelativeTolerance(const double v) { m_s.eps_rel = v; }
    void setPrimalInfeasibilityTolerance(const double v) { m_s.eps_prim_inf = v; }
    void setPrimalInfeasibilityTollerance(const double v) { m_s.eps_prim_inf = v; }
    void setDualInfeasibilityTolerance(const double v) { m_s.eps_dual_inf = v; }
    void setDualInfeasibilityTollerance(const double v) { m_s.eps_dual_inf = v; }
    void setAlpha(const double v) { m_s.alpha = v; }
    void setLinearSystemSolver(const int v) { m_s.linsys_solver = v; }
    void setDelta(const double v) { m_s.delta = v; }
    void setPolish(const bool v) { m_s.polish = v ? 1 : 0; }
    void setPolishRefineIter(const int v) { m_s.polish_refine_iter = v; }
    void setVerbosity(const bool v) { m_s.verbose = v ? 1 : 0; }
    void setScaledTerimination(const bool v) { m_s.scaled_termination = v ? 1 : 0; }
    void setCheckTermination(const int v) { m_s.check_termination = v; }
    void setWarmStart(const bool v) { m_s.warm_start = v ? 1 : 0; }
    void setTimeLimit(const double v) { m_s.time_limit = v; }
    const impc_settings &getSettings() const { return m_s; }
};

/* Data.hpp:44-151: same member names and argument types (setGradient / set*Bound take
 * Eigen::Ref<VectorXd> by value, the matrices an Eigen::SparseCompressedBase).  getData() returns
 * OSQP 0.6.2's public OSQPData (the types below, osqp/include/types.h with DLONG: c_int = long
 * long) viewing this object's arrays: P upper triangular CSC, A CSC, q, l, u. */
class Data {
    int64_t m_n = 0, m_m = 0;
    bool m_hasP = false, m_hasA = false, m_hasq = false, m_hasl = false, m_hasu = false;
    ::csc m_P{}, m_A{};
    ::OSQPData m_view{};
    ::OSQPData *m_viewp = &m_view;

public:
    std::vector<int64_t> Pp, Pi, Ap, Ai;
    std::vector<double> Px, Ax, q, l, u;

    Data() = default;
    Data(int n, int m) : m_n(n), m_m(m) {}
    void setNumberOfVariables(int n) { m_n = n; }
    void setNumberOfConstraints(int m) { m_m = m; }
    int64_t numberOfVariables() const { return m_n; }
    int64_t numberOfConstraints() const { return m_m; }
    void clearHessianMatrix() { m_hasP = false; Pp.clear(); Pi.clear(); Px.clear(); }
    void clearLinearConstraintsMatrix() { m_hasA = false; Ap.clear(); Ai.clear(); Ax.clear(); }

    template <typename Derived>
    bool setHessianMatrix(const Eigen::SparseCompressedBase<Derived> &hessianMatrix) {
        if (m_hasP) { detail::debug("the Hessian matrix was already set"); return false; }
        if ((int64_t)hessianMatrix.rows() != m_n || (int64_t)hessianMatrix.cols() != m_n) {
            detail::debug("the Hessian matrix has to be n x n");
            return false;
        }
        detail::to_csc(hessianMatrix.derived(), true, Pp, Pi, Px);
        return m_hasP = true;
    }
    template <typename Derived>
    bool setLinearConstraintsMatrix(const Eigen::SparseCompressedBase<Derived> &linearConstraintsMatrix) {
        if (m_hasA) { detail::debug("the constraint matrix was already set"); return false; }
        if ((int64_t)linearConstraintsMatrix.rows() != m_m || (int64_t)linearConstraintsMatrix.cols() != m_n) {
            detail::debug("the constraint matrix has to be m x n");
            return false;
        }
        detail::to_csc(linearConstraintsMatrix.derived(), false, Ap, Ai, Ax);
        return m_hasA = true;
    }
    bool setGradient(Eigen::Ref<Eigen::Matrix<double, Eigen::Dynamic, 1>> gradientVector) {
        if (!detail::copy_vec(gradientVector, m_n, q)) { detail::debug("the gradient has to be n x 1"); return false; }
        return m_hasq = true;
    }
    bool setLowerBound(Eigen::Ref<Eigen::Matrix<double, Eigen::Dynamic, 1>> lowerBoundVector) {
        if (!detail::copy_vec(lowerBoundVector, m_m, l)) { detail::debug("the lower bound has to be m x 1"); return false; }
        return m_hasl = true;
    }
    bool setUpperBound(Eigen::Ref<Eigen::Matrix<double, Eigen::Dynamic, 1>> upperBoundVector) {
        if (!detail::copy_vec(upperBoundVector, m_m, u)) { detail::debug("the upper bound has to be m x 1"); return false; }
        return m_hasu = true;
    }
    bool setBounds(Eigen::Ref<Eigen::Matrix<double, Eigen::Dynamic, 1>> lowerBound,
                   Eigen::Ref<Eigen::Matrix<double, Eigen::Dynamic, 1>> upperBound) {
        return setLowerBound(lowerBound) && setUpperBound(upperBound);
    }
    bool isSet() const { return m_n > 0 && m_hasP && m_hasA && m_hasq && m_hasl && m_hasu; }
    // Data.hpp:99 -- the gradient as a vector (a copy)
    Eigen::Matrix<double, Eigen::Dynamic, 1> getGradient() {
        Eigen::Matrix<double, Eigen::Dynamic, 1> g;
        g.setZero(m_n);
        for (int64_t i = 0; i < (int64_t)q.size() && i < m_n; i++) g(i) = q[i];
        return g;
    }
    // Data.hpp:145 -- the problem data in OSQP's struct, pointing into this object (valid until the
    // next set* / clear* call); a matrix not set yet has nullptr arrays
    ::OSQPData *const &getData() const {
        auto *self = const_cast<Data *>(this);
        auto fill = [](::csc &c, int64_t rows, int64_t cols, std::vector<int64_t> &p, std::vector<int64_t> &i,
                       std::vector<double> &x) {
            c.m = (c_int)rows;
            c.n = (c_int)cols;
            c.nzmax = (c_int)x.size();
            c.p = p.empty() ? nullptr : (c_int *)p.data();
            c.i = i.empty() ? nullptr : (c_int *)i.data();
            c.x = x.empty() ? nullptr : x.data();
            c.nz = -1;  // compressed column form
        };
        fill(self->m_P, m_n, m_n, self->Pp, self->Pi, self->Px);
        fill(self->m_A, m_m, m_n, self->Ap, self->Ai, self->Ax);
        self->m_view.n = (c_int)m_n;
        self->m_view.m = (c_int)m_m;
        self->m_view.P = m_hasP ? &self->m_P : nullptr;
        self->m_view.A = m_hasA ? &self->m_A : nullptr;
        self->m_view.q = m_hasq ? self->q.data() : nullptr;
        self->m_view.l = m_hasl ? self->l.data() : nullptr;
        self->m_view.u = m_hasu ? self->u.data() : nullptr;
        return m_viewp;
    }
};

/* Solver.hpp:87-249: same member names and signatures (Solver.hpp:196-231 templates included). */
class Solver {
    using VecRef = Eigen::Ref<const Eigen::Matrix<double, Eigen::Dynamic, 1>>;
    std::unique_ptr<Settings> m_settings;
    std::unique_ptr<Data> m_data;
    impc_batch m_batch = nullptr;
    bool m_solved = false;
    impc_info m_info{};
    Eigen::Matrix<double, Eigen::Dynamic, 1> m_x, m_y;
    // the iterate the next solve starts from, as far as the host knows (last solution or last warm
    // start, unscaled): osqp_warm_start_x / _y replace one half and keep the other
    std::vector<double> m_wx, m_wy;
    bool m_persistent = false;     // structured batch with a persistent workspace
    bool m_setup_current = false;  // the device workspace is set up on the current data

    void release() {
        if (m_batch) (detail::no_pool() ? impc_batch_destroy : impc_batch_release)(m_batch);
        m_batch = nullptr;
    }
    bool structured() const {
        impc_batch_stats st{};
        return m_batch && impc_batch_get_stats(m_batch, &st) == IMPC_OK && st.kernel == IMPC_KERNEL_STRUCTURED;
    }
    // osqp_update_* applies to the set-up workspace in place: a persistent structured batch or a
    // generic batch, once a solve has set it up on the current data
    bool in_place() const { return m_setup_current && (m_persistent || !structured()); }
    bool warm_start_raw(const std::vector<double> &x, const std::vector<double> &y) {
        int rc = impc_batch_warm_start(m_batch, x.data(), y.data());
        if (rc) { detail::debug_impc("impc_batch_warm_start", rc); return false; }
        m_wx = x;
        m_wy = y;
        return true;
    }
    // osqp_setup again from the current data, warm-started from the last solution (what OsqpEigen
    // does when an update cannot be applied in place: clearSolver, initSolver, set*Variable)
    bool resetup_from_data() {
        const Data &d = *m_data;
        int rc = impc_batch_set_values(m_batch, d.Px.data(), d.q.data(), d.Ax.data(), d.l.data(), d.u.data());
        if (rc) { detail::debug_impc("impc_batch_set_values", rc); return false; }
        m_setup_current = false;
        if (m_solved) return warm_start_raw(m_wx, m_wy);
        return true;
    }
    template <typename Derived>
    bool update_matrix(const Eigen::SparseCompressedBase<Derived> &M, bool hessian) {
        if (!m_batch) { detail::debug("the solver has not been initialized"); return false; }
        Data &d = *m_data;
        const int64_t rows = hessian ? d.numberOfVariables() : d.numberOfConstraints();
        if ((int64_t)M.rows() != rows || (int64_t)M.cols() != d.numberOfVariables()) {
            detail::debug(hessian ? "the hessian matrix has to be a nxn matrix" : "the constraint matrix has to be m x n");
            return false;
        }
        std::vector<int64_t> p, i;
        std::vector<double> x;
        detail::to_csc(M.derived(), hessian, p, i, x);
        if (p != (hessian ? d.Pp : d.Ap) || i != (hessian ? d.Pi : d.Ai)) {
            // new sparsity pattern: a new batch (OsqpEigen: clearSolver + initSolver + warm start)
            std::vector<double> wx = m_wx, wy = m_wy;
            const bool had = m_solved;
            if (hessian) { d.Pp = p; d.Pi = i; d.Px = x; } else { d.Ap = p; d.Ai = i; d.Ax = x; }
            clearSolver();
            if (!initSolver()) return false;
            return had ? warm_start_raw(wx, wy) : true;
        }
        std::vector<double> &dst = hessian ? d.Px : d.Ax;
        if (in_place() && structured()) {  // osqp_update_P / osqp_update_A on the kept workspace
            int rc = impc_batch_update_matrices(m_batch, hessian ? x.data() : nullptr, hessian ? nullptr : x.data());
            if (rc) { detail::debug_impc("impc_batch_update_matrices", rc); return false; }
            dst = x;
            return true;
        }
        std::vector<double> old = dst;
        dst = x;
        if (resetup_from_data()) return true;
        dst = old;
        return false;
    }

public:
    Solver() : m_settings(new Settings()), m_data(new Data()) {}
    ~Solver() { clearSolver(); }
    Solver(const Solver &) = delete;
    Solver &operator=(const Solver &) = delete;

    const std::unique_ptr<Settings> &settings() const { return m_settings; }
    const std::unique_ptr<Data> &data() const { return m_data; }

    bool isInitialized() { return m_batch != nullptr; }

    bool initSolver() {
        if (m_batch) { detail::debug("the solver is already initialized"); return false; }
        if (!m_data->isSet()) { detail::debug("some data are not set"); return false; }
        impc_ctx ctx = detail::context();
        if (!ctx) return false;
        const Data &d = *m_data;
        int rc = (detail::no_pool() ? impc_batch_create : impc_batch_acquire)(
            ctx, d.numberOfVariables(), d.numberOfConstraints(), d.Pp.data(), d.Pi.data(), d.Ap.data(), d.Ai.data(), 1,
            &m_batch);
        if (rc) { detail::debug_impc("impc_batch_acquire", rc); m_batch = nullptr; return false; }
        rc = impc_batch_set_settings(m_batch, &m_settings->getSettings());
        if (!rc) rc = impc_batch_set_values(m_batch, d.Px.data(), d.q.data(), d.Ax.data(), d.l.data(), d.u.data());
        if (rc) {
            detail::debug_impc("osqp_setup equivalent", rc);
            release();
            return false;
        }
        // updateGradient / updateBounds between solves keep the solver state, as osqp_update_*
        // does; scaling > 20 passes is refused (IMPC_UNSUPPORTED) and falls back to re-setup
        m_persistent = structured() && impc_batch_set_persistent(m_batch, 1) == IMPC_OK;
        m_x.setZero(d.numberOfVariables());
        m_y.setZero(d.numberOfConstraints());
        m_wx.assign((size_t)d.numberOfVariables(), 0.0);
        m_wy.assign((size_t)d.numberOfConstraints(), 0.0);
        m_solved = false;
        m_setup_current = false;
        return true;
    }

    void clearSolver() {
        release();
        m_solved = false;
        m_persistent = false;
        m_setup_current = false;
    }

    bool clearSolverVariables() {
        if (!m_batch) return false;
        // osqp cold start: zero iterates (a persistent workspace would otherwise resume from its own)
        std::vector<double> x((size_t)m_data->numberOfVariables(), 0.0), y((size_t)m_data->numberOfConstraints(), 0.0);
        if (m_persistent) return warm_start_raw(x, y);
        m_wx = x;
        m_wy = y;
        return impc_batch_warm_start(m_batch, nullptr, nullptr) == IMPC_OK;
    }

    template <typename T, int n, int m>
    bool setWarmStart(const Eigen::Matrix<T, n, 1> &primalVariable, const Eigen::Matrix<T, m, 1> &dualVariable) {
        if (!m_batch) { detail::debug("the solver is not initialized"); return false; }
        std::vector<double> x, y;
        if (!detail::copy_vec(primalVariable, m_data->numberOfVariables(), x) ||
            !detail::copy_vec(dualVariable, m_data->numberOfConstraints(), y)) {
            detail::debug("warm start has the wrong size");
            return false;
        }
        return warm_start_raw(x, y);
    }

    /* osqp_warm_start_x: x replaced, y kept */
    template <typename T, int n>
    bool setPrimalVariable(const Eigen::Matrix<T, n, 1> &primalVariable) {
        if (!m_batch) { detail::debug("the solver is not initialized"); return false; }
        std::vector<double> x;
        if (!detail::copy_vec(primalVariable, m_data->numberOfVariables(), x)) {
            detail::debug("the size of the primal variable vector has to be equal to the number of variables");
            return false;
        }
        return warm_start_raw(x, m_wy);
    }

    /* osqp_warm_start_y: y replaced, x kept */
    template <typename T, int m>
    bool setDualVariable(const Eigen::Matrix<T, m, 1> &dualVariable) {
        if (!m_batch) { detail::debug("the solver is not initialized"); return false; }
        std::vector<double> y;
        if (!detail::copy_vec(dualVariable, m_data->numberOfConstraints(), y)) {
            detail::debug("the size of the dual variable vector has to be equal to the number of constraints");
            return false;
        }
        return warm_start_raw(m_wx, y);
    }

    /* Returns the unscaled iterate the next solve starts from (OsqpEigen copies OSQP's scaled
     * internal work->x / work->y here; no reference caller reads it). */
    template <typename T, int n>
    bool getPrimalVariable(Eigen::Matrix<T, n, 1> &primalVariable) {
        if (!m_batch) { detail::debug("the solver is not initialized"); return false; }
        const int64_t nv = m_data->numberOfVariables();
        if (n == Eigen::Dynamic) primalVariable.resize(nv, 1);
        else if (n != nv) { detail::debug("the size of the vector has to be equal to the number of variables"); return false; }
        for (int64_t k = 0; k < nv; ++k) primalVariable((Eigen::Index)k) = (T)m_wx[(size_t)k];
        return true;
    }
    template <typename T, int m>
    bool getDualVariable(Eigen::Matrix<T, m, 1> &dualVariable) {
        if (!m_batch) { detail::debug("the solver is not initialized"); return false; }
        const int64_t mc = m_data->numberOfConstraints();
        if (m == Eigen::Dynamic) dualVariable.resize(mc, 1);
        else if (m != mc) { detail::debug("the size of the vector has to be equal to the number of constraints"); return false; }
        for (int64_t k = 0; k < mc; ++k) dualVariable((Eigen::Index)k) = (T)m_wy[(size_t)k];
        return true;
    }

    ErrorExitFlag solveProblem() {
        if (!m_batch) return ErrorExitFlag::WorkspaceNotInitError;
        int rc = impc_batch_set_settings(m_batch, &m_settings->getSettings());
        if (!rc) rc = impc_batch_solve(m_batch, nullptr);
        if (rc) {
            detail::debug_impc("impc_batch_solve", rc);
            return rc == IMPC_SETTINGS_VALIDATION_ERROR || rc == IMPC_UNSUPPORTED ? ErrorExitFlag::SettingsValidationError
                                                                                   : ErrorExitFlag::WorkspaceNotInitError;
        }
        std::vector<double> x((size_t)m_data->numberOfVariables()), y((size_t)m_data->numberOfConstraints());
        rc = impc_batch_get(m_batch, x.data(), y.data(), &m_info);
        if (rc) { detail::debug_impc("impc_batch_get", rc); return ErrorExitFlag::WorkspaceNotInitError; }
        for (size_t k = 0; k < x.size(); ++k) m_x((Eigen::Index)k) = x[k];
        for (size_t k = 0; k < y.size(); ++k) m_y((Eigen::Index)k) = y[k];
        m_wx = x;
        m_wy = y;
        m_solved = true;
        m_setup_current = true;
        if (m_info.setup_exitflag == IMPC_NONCVX_ERROR) return ErrorExitFlag::NonCvxError;
        return ErrorExitFlag::NoError;
    }

    /* deprecated OsqpEigen API: true when solved to full accuracy */
    bool solve() { return solveProblem() == ErrorExitFlag::NoError && getStatus() == Status::Solved; }

    Status getStatus() const { return m_solved ? (Status)m_info.status_val : Status::Unsolved; }
    const Eigen::Matrix<double, Eigen::Dynamic, 1> &getSolution() { return m_x; }
    const Eigen::Matrix<double, Eigen::Dynamic, 1> &getDualSolution() { return m_y; }
    double getObjValue() const { return m_info.obj_val; }
    int64_t getIterations() const { return m_info.iter; }

    /* osqp_update_lin_cost; before the workspace is set up (no solve yet, or after a re-setup)
     * the new vector is taken by a fresh setup.  Data keeps the old vector if the update fails. */
    bool updateGradient(const VecRef &gradient) {
        if (!m_batch) { detail::debug("the solver has not been initialized"); return false; }
        std::vector<double> q;
        if (!detail::copy_vec(gradient, m_data->numberOfVariables(), q)) { detail::debug("the gradient has to be n x 1"); return false; }
        if (!in_place()) {
            std::vector<double> old = m_data->q;
            m_data->q = q;
            if (resetup_from_data()) return true;
            m_data->q = old;
            return false;
        }
        int rc = impc_batch_update_lin_cost(m_batch, q.data());
        if (rc) { detail::debug_impc("impc_batch_update_lin_cost", rc); return false; }
        m_data->q = q;
        return true;
    }
    /* osqp_update_bounds, with the same fallback */
    bool updateBounds(const VecRef &lowerBound, const VecRef &upperBound) {
        if (!m_batch) { detail::debug("the solver has not been initialized"); return false; }
        const int64_t m = m_data->numberOfConstraints();
        std::vector<double> l, u;
        if (!detail::copy_vec(lowerBound, m, l) || !detail::copy_vec(upperBound, m, u)) {
            detail::debug("the bounds have to be m x 1");
            return false;
        }
        if (!in_place()) {
            std::vector<double> ol = m_data->l, ou = m_data->u;
            m_data->l = l;
            m_data->u = u;
            if (resetup_from_data()) return true;
            m_data->l = ol;
            m_data->u = ou;
            return false;
        }
        int rc = impc_batch_update_bounds(m_batch, l.data(), u.data());
        if (rc) { detail::debug_impc("impc_batch_update_bounds", rc); return false; }
        m_data->l = l;
        m_data->u = u;
        return true;
    }
    bool updateLowerBound(const VecRef &lowerBound) {
        Eigen::Matrix<double, Eigen::Dynamic, 1> u((Eigen::Index)m_data->numberOfConstraints());
        for (int64_t k = 0; k < m_data->numberOfConstraints(); ++k) u((Eigen::Index)k) = m_data->u[(size_t)k];
        return updateBounds(lowerBound, u);
    }
    bool updateUpperBound(const VecRef &upperBound) {
        Eigen::Matrix<double, Eigen::Dynamic, 1> l((Eigen::Index)m_data->numberOfConstraints());
        for (int64_t k = 0; k < m_data->numberOfConstraints(); ++k) l((Eigen::Index)k) = m_data->l[(size_t)k];
        return updateBounds(l, upperBound);
    }

    /* Solver.tpp:15-113 / :116-212.  Same pattern on the persistent structured workspace (the
     * mpcPlanner QP): osqp_update_P / osqp_update_A -- the next solve re-runs the scaling on the new
     * data, refactors with the kept rho and continues from the kept scaled iterates, as OSQP 0.6.2
     * does (impc_batch_update_matrices).  Same pattern on the generic kernel (any other QP), or
     * before the first solve: the new values are set up afresh and the solve resumes from the last
     * solution, unscaled (a documented deviation: the same fixed point, a different first
     * iteration).  New pattern: a new batch, warm-started, as OsqpEigen re-initialises its solver.
     * No reference caller updates P or A. */
    template <typename Derived>
    bool updateHessianMatrix(const Eigen::SparseCompressedBase<Derived> &hessianMatrix) {
        return update_matrix(hessianMatrix, true);
    }
    template <typename Derived>
    bool updateLinearConstraintsMatrix(const Eigen::SparseCompressedBase<Derived> &linearConstraintsMatrix) {
        return update_matrix(linearConstraintsMatrix, false);
    }
};

}  // namespace OsqpEigen

#endif
