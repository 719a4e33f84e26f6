// TEST INFRASTRUCTURE ONLY -- drives include/OsqpEigen/OsqpEigen.h with the call sequence of
// mpcPlanner::solveTraj (reference mpcPlanner.cpp:436-527), against the Eigen stand-in.
//   shim_test cpu : conversion checks + graceful failure without a device (exit 0 = pass)
//   shim_test gpu : OSQP demo QP through the shim on the GPU (x*, y*, status), then a
//                   stage-structured mpcPlanner QP (impc_mpc_build_*) through the shim's
//                   solve -> updateGradient -> solve -> updateBounds -> solve sequence against
//                   a direct persistent batch of the C-ABI (exit 0 = pass)
//   shim_test replay <in> <out> : the solveTraj call sequence (new Solver per QP, settings,
//                   set*, initSolver, setWarmStart(x, y = 0), solveProblem, get*) over the QPs of
//                   <in>, optionally followed by updateGradient -> solveProblem -> updateBounds ->
//                   solveProblem; results to <out> for tests/test_shim.py to check against the
//                   oracle (not against the C-ABI)
//   shim_test bench <in> <calls> : the per-call cost of the drop-in path -- host wall time of the
//                   whole solveTraj sequence (Solver construction -> settings -> set* -> initSolver
//                   -> setWarmStart -> solveProblem -> getSolution -> clearSolver) over <calls>
//                   calls cycling through the QPs of <in>, next to the device time of the same
//                   QPs solved alone on a direct one-QP batch (HIP events around the launch, and
//                   the kernel's own dequeue-to-results latency); one JSON line
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <OsqpEigen/OsqpEigen.h>
#include <impc_mpc.h>
#include <vector>

static int fails = 0;
#define CHECK(c)                                                   \
    do {                                                           \
        if (!(c)) {                                                \
            std::printf("CHECK failed line %d: %s\n", __LINE__, #c); \
            fails++;                                               \
        }                                                          \
    } while (0)

// One live-config mpcPlanner QP (N = 20, 2 dynamic obstacles ahead of the drone), through the
// shim and through a direct persistent structured batch: the shim's update* calls must carry the
// workspace over exactly as impc_batch_update_* on a persistent batch do (same iteration counts,
// primal to 1e-9).
static void structured_case() {
    impc_mpc_params p{};
    p.horizon = 20, p.num_half_space = 0, p.ts = 0.1, p.max_vel = 5.0, p.max_acc = 20.0;
    p.y_range_min = -5.0, p.y_range_max = 5.0, p.z_range_min = 0.5, p.z_range_max = 4.5;
    p.static_safety_dist = 0.8, p.dynamic_safety_dist = 1.5, p.static_slack = 0.01, p.dynamic_slack = 0.2;
    p.position_weight = 1000.0, p.velocity_weight = 0.0, p.acceleration_weight = 10.0;
    const int N = 20, K = 2, L = 20;
    impc_qp_dims dm{};
    CHECK(impc_mpc_dims(&p, 0, K, &dm) == IMPC_OK);
    const int64_t n = dm.n, m = dm.m;
    std::vector<int64_t> Pp(n + 1), Pi(dm.nnzP), Ap(n + 1), Ai(dm.nnzA);
    CHECK(impc_mpc_build_pattern(&p, 0, K, Pp.data(), Pi.data(), Ap.data(), Ai.data()) == IMPC_OK);
    double pos[3] = {0.0, 0.0, 1.2}, vel[3] = {1.0, 0.1, 0.0};
    std::vector<double> xref((size_t)N * 8, 0.0), dpos((size_t)K * L * 3), dsize((size_t)K * L * 3, 0.6);
    for (int j = 0; j < N; j++) {
        xref[(size_t)j * 8 + 0] = 0.15 * j;
        xref[(size_t)j * 8 + 2] = 1.2;
        xref[(size_t)j * 8 + 3] = 1.5;
    }
    for (int k = 0; k < K; k++)
        for (int j = 0; j < L; j++) {
            double *d = &dpos[((size_t)k * L + j) * 3];
            d[0] = 2.0 + 0.8 * k - 0.05 * j;
            d[1] = (k ? -0.4 : 0.5) + 0.02 * j;
            d[2] = 1.2;
        }
    std::vector<double> Px(dm.nnzP), q(n), Ax(dm.nnzA), l(m), u(m);
    CHECK(impc_mpc_build_values(&p, 1, pos, vel, xref.data(), nullptr, 0, nullptr, nullptr, nullptr, K, L, dpos.data(),
                                dsize.data(), Px.data(), q.data(), Ax.data(), l.data(), u.data()) == IMPC_OK);
    Eigen::SparseMatrix<double> P((Eigen::Index)n, (Eigen::Index)n), A((Eigen::Index)m, (Eigen::Index)n);
    for (int64_t j = 0; j < n; j++) {
        for (int64_t k = Pp[j]; k < Pp[j + 1]; k++) P.insert(Pi[k], j) = Px[k];
        for (int64_t k = Ap[j]; k < Ap[j + 1]; k++) A.insert(Ai[k], j) = Ax[k];
    }
    auto vec = [](const std::vector<double> &v) {
        Eigen::VectorXd e((Eigen::Index)v.size());
        for (size_t k = 0; k < v.size(); k++) e((Eigen::Index)k) = v[k];
        return e;
    };
    // the update sequence: a shifted reference (q), then the y band narrowed (l / u)
    std::vector<double> q2(q), l3(l), u3(u);
    for (int64_t j = 0; j < n; j++) q2[j] = q[j] * 1.05 + (j % 8 == 1 ? 0.3 : 0.0);
    for (int64_t i = 0; i < m; i++)
        if (std::isfinite(l3[i]) && std::isfinite(u3[i]) && u3[i] - l3[i] > 0.1) l3[i] += 0.01, u3[i] -= 0.01;

    OsqpEigen::Solver solver;
    solver.settings()->setVerbosity(false);
    solver.settings()->setWarmStart(true);
    solver.data()->setNumberOfVariables((int)n);
    solver.data()->setNumberOfConstraints((int)m);
    Eigen::VectorXd qv = vec(q), lv = vec(l), uv = vec(u);  // Data's setters take Ref<VectorXd>: lvalues
    CHECK(solver.data()->setHessianMatrix(P));
    CHECK(solver.data()->setGradient(qv));
    CHECK(solver.data()->setLinearConstraintsMatrix(A));
    CHECK(solver.data()->setLowerBound(lv));
    CHECK(solver.data()->setUpperBound(uv));
    CHECK(solver.initSolver());

    impc_ctx ctx = nullptr;
    impc_batch b = nullptr;
    CHECK(impc_ctx_create(0, &ctx) == IMPC_OK);
    CHECK(impc_batch_create(ctx, n, m, Pp.data(), Pi.data(), Ap.data(), Ai.data(), 1, &b) == IMPC_OK);
    impc_settings st;
    impc_default_settings(&st);
    st.verbose = 0;
    st.warm_start = 1;
    impc_batch_stats bs{};
    CHECK(impc_batch_get_stats(b, &bs) == IMPC_OK && bs.kernel == IMPC_KERNEL_STRUCTURED);
    CHECK(impc_batch_set_settings(b, &st) == IMPC_OK);
    CHECK(impc_batch_set_values(b, Px.data(), q.data(), Ax.data(), l.data(), u.data()) == IMPC_OK);
    CHECK(impc_batch_set_persistent(b, 1) == IMPC_OK);
    std::vector<double> xd(n), yd(m);
    impc_info info{};
    for (int step = 0; step < 3; step++) {
        if (step == 1) {
            CHECK(solver.updateGradient(vec(q2)));  // Ref<const VectorXd>: temporaries bind
            CHECK(impc_batch_update_lin_cost(b, q2.data()) == IMPC_OK);
        } else if (step == 2) {
            CHECK(solver.updateBounds(vec(l3), vec(u3)));
            CHECK(impc_batch_update_bounds(b, l3.data(), u3.data()) == IMPC_OK);
        }
        CHECK(solver.solveProblem() == OsqpEigen::ErrorExitFlag::NoError);
        CHECK(impc_batch_solve(b, nullptr) == IMPC_OK);
        CHECK(impc_batch_get(b, xd.data(), yd.data(), &info) == IMPC_OK);
        const Eigen::VectorXd &xs = solver.getSolution();
        double dx = 0.0, xm = 1e-12;
        for (int64_t j = 0; j < n; j++) {
            dx = std::fmax(dx, std::fabs(xs((Eigen::Index)j) - xd[j]));
            xm = std::fmax(xm, std::fabs(xd[j]));
        }
        std::printf("structured step %d: status %d iters %lld (direct %lld) max|dx| %.3e\n", step,
                    (int)solver.getStatus(), (long long)solver.getIterations(), (long long)info.iter, dx);
        CHECK((int64_t)solver.getStatus() == info.status_val);
        CHECK(solver.getIterations() == info.iter);
        CHECK(dx <= 1e-9 * xm);
    }
    impc_batch_destroy(b);
    impc_ctx_destroy(ctx);
}

// Replay file layout (little-endian): int64 header {n, m, nnzP, nnzA, nqp, flags} (flags bit 0:
// warm start x per QP, bit 1: update sequence q2 / l3 / u3 per QP, bit 2 (with bit 1): then
// updateHessianMatrix(P4) -> solve -> updateLinearConstraintsMatrix(A4) -> solve), int64 Pp[n+1]
// Pi Ap[n+1] Ai, then per QP double Px q Ax l u [x_ws] [q2 l3 u3] [P4 A4].  Output per QP and step: double status, iter,
// obj, x[n], y[m].  P is inserted with both triangles (as an Eigen user holding the full symmetric
// matrix does); the shim keeps the upper one (OsqpEigen Data.tpp:38-39).
static int replay(const char *in, const char *out) {
    FILE *f = std::fopen(in, "rb");
    if (!f) return 2;
    int64_t h[6];
    if (std::fread(h, sizeof h, 1, f) != 1) return 2;
    const int64_t n = h[0], m = h[1], nnzP = h[2], nnzA = h[3], nqp = h[4], flags = h[5];
    auto rd = [&](auto &v, size_t k) { v.resize(k); return std::fread(v.data(), sizeof(v[0]), k, f) == k; };
    std::vector<int64_t> Pp, Pi, Ap, Ai;
    if (!rd(Pp, n + 1) || !rd(Pi, nnzP) || !rd(Ap, n + 1) || !rd(Ai, nnzA)) return 2;
    FILE *o = std::fopen(out, "wb");
    if (!o) return 2;
    auto vec = [](const std::vector<double> &v) {
        Eigen::VectorXd e((Eigen::Index)v.size());
        for (size_t k = 0; k < v.size(); k++) e((Eigen::Index)k) = v[k];
        return e;
    };
    for (int64_t qp = 0; qp < nqp; qp++) {
        std::vector<double> Px, q, Ax, l, u, xw, q2, l3, u3, P4, A4;
        if (!rd(Px, nnzP) || !rd(q, n) || !rd(Ax, nnzA) || !rd(l, m) || !rd(u, m)) return 2;
        if ((flags & 1) && !rd(xw, n)) return 2;
        if ((flags & 2) && (!rd(q2, n) || !rd(l3, m) || !rd(u3, m))) return 2;
        if ((flags & 4) && (!rd(P4, nnzP) || !rd(A4, nnzA))) return 2;
        // the Eigen matrices a user holds: P with both triangles, A full
        auto mats = [&](const std::vector<double> &pv, const std::vector<double> &av, Eigen::SparseMatrix<double> &P,
                        Eigen::SparseMatrix<double> &A) {
            for (int64_t j = 0; j < n; j++) {
                for (int64_t k = Pp[j]; k < Pp[j + 1]; k++) {
                    P.insert(Pi[k], j) = pv[k];
                    if (Pi[k] != j) P.insert(j, Pi[k]) = pv[k];
                }
                for (int64_t k = Ap[j]; k < Ap[j + 1]; k++) A.insert(Ai[k], j) = av[k];
            }
        };
        Eigen::SparseMatrix<double> P((Eigen::Index)n, (Eigen::Index)n), A((Eigen::Index)m, (Eigen::Index)n);
        mats(Px, Ax, P, A);
        OsqpEigen::Solver solver;  // mpcPlanner.cpp:436-527
        solver.settings()->setVerbosity(false);
        solver.settings()->setWarmStart(true);
        solver.data()->setNumberOfVariables((int)n);
        solver.data()->setNumberOfConstraints((int)m);
        Eigen::VectorXd qv = vec(q), lv = vec(l), uv = vec(u);
        CHECK(solver.data()->setHessianMatrix(P));
        CHECK(solver.data()->setGradient(qv));
        CHECK(solver.data()->setLinearConstraintsMatrix(A));
        CHECK(solver.data()->setLowerBound(lv));
        CHECK(solver.data()->setUpperBound(uv));
        CHECK(solver.initSolver());
        if (flags & 1) {
            Eigen::VectorXd x0 = vec(xw), y0;
            y0.setZero((Eigen::Index)m);
            CHECK(solver.setWarmStart(x0, y0));
        }
        const int steps = (flags & 2) ? ((flags & 4) ? 5 : 3) : 1;
        for (int step = 0; step < steps; step++) {
            if (step == 1) CHECK(solver.updateGradient(vec(q2)));
            if (step == 2) CHECK(solver.updateBounds(vec(l3), vec(u3)));
            if (step >= 3) {  // Solver.tpp:15-212, same sparsity pattern
                Eigen::SparseMatrix<double> P4m((Eigen::Index)n, (Eigen::Index)n), A4m((Eigen::Index)m, (Eigen::Index)n);
                mats(P4, A4, P4m, A4m);
                if (step == 3) CHECK(solver.updateHessianMatrix(P4m));
                if (step == 4) CHECK(solver.updateLinearConstraintsMatrix(A4m));
            }
            CHECK(solver.solveProblem() == OsqpEigen::ErrorExitFlag::NoError);
            double hdr[3] = {(double)solver.getStatus(), (double)solver.getIterations(), solver.getObjValue()};
            std::fwrite(hdr, sizeof(double), 3, o);
            const Eigen::VectorXd &x = solver.getSolution();
            const Eigen::VectorXd &y = solver.getDualSolution();
            CHECK(x.size() == n && y.size() == m);
            std::fwrite(x.data(), sizeof(double), (size_t)n, o);
            std::fwrite(y.data(), sizeof(double), (size_t)m, o);
        }
        solver.clearSolver();
    }
    std::fclose(f);
    std::fclose(o);
    std::printf("replay: %lld QP(s), %d failure(s)\n", (long long)nqp, fails);
    return fails ? 1 : 0;
}

static double pct(std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[(size_t)std::min<double>((double)v.size() - 1, p * (double)(v.size() - 1) + 0.5)];
}

static int bench(const char *in, long calls) {
    FILE *f = std::fopen(in, "rb");
    if (!f) return 2;
    int64_t h[6];
    if (std::fread(h, sizeof h, 1, f) != 1) return 2;
    const int64_t n = h[0], m = h[1], nnzP = h[2], nnzA = h[3], nqp = h[4], flags = h[5];
    auto rd = [&](auto &v, size_t k) { v.resize(k); return std::fread(v.data(), sizeof(v[0]), k, f) == k; };
    std::vector<int64_t> Pp, Pi, Ap, Ai;
    if (!rd(Pp, n + 1) || !rd(Pi, nnzP) || !rd(Ap, n + 1) || !rd(Ai, nnzA)) return 2;
    struct QP {
        std::vector<double> Px, q, Ax, l, u, xw;
        Eigen::SparseMatrix<double> P, A;
    };
    std::vector<QP> qps((size_t)nqp);
    for (QP &Q : qps) {
        if (!rd(Q.Px, nnzP) || !rd(Q.q, n) || !rd(Q.Ax, nnzA) || !rd(Q.l, m) || !rd(Q.u, m)) return 2;
        if ((flags & 1) && !rd(Q.xw, n)) return 2;
        Q.P = Eigen::SparseMatrix<double>((Eigen::Index)n, (Eigen::Index)n);
        Q.A = Eigen::SparseMatrix<double>((Eigen::Index)m, (Eigen::Index)n);
        for (int64_t j = 0; j < n; j++) {
            for (int64_t k = Pp[j]; k < Pp[j + 1]; k++) Q.P.insert(Pi[k], j) = Q.Px[k];
            for (int64_t k = Ap[j]; k < Ap[j + 1]; k++) Q.A.insert(Ai[k], j) = Q.Ax[k];
        }
    }
    std::fclose(f);
    auto vec = [](const std::vector<double> &v) {
        Eigen::VectorXd e((Eigen::Index)v.size());
        for (size_t k = 0; k < v.size(); k++) e((Eigen::Index)k) = v[k];
        return e;
    };
    // the drop-in path, timed per call on the host clock (the first call of each QP shape also
    // creates the context / pool entry: warm-up calls are not timed)
    std::vector<double> wall;
    const long warm = std::min<long>(8, calls);
    for (long c = 0; c < calls + warm; c++) {
        const QP &Q = qps[(size_t)(c % nqp)];
        const auto t0 = std::chrono::steady_clock::now();
        {
            OsqpEigen::Solver solver;  // mpcPlanner.cpp:436-527
            solver.settings()->setVerbosity(false);
            solver.settings()->setWarmStart(true);
            solver.data()->setNumberOfVariables((int)n);
            solver.data()->setNumberOfConstraints((int)m);
            Eigen::VectorXd qv = vec(Q.q), lv = vec(Q.l), uv = vec(Q.u);
            bool ok = solver.data()->setHessianMatrix(Q.P) && solver.data()->setGradient(qv) &&
                      solver.data()->setLinearConstraintsMatrix(Q.A) && solver.data()->setLowerBound(lv) &&
                      solver.data()->setUpperBound(uv) && solver.initSolver();
            Eigen::VectorXd x0 = (flags & 1) ? vec(Q.xw) : Eigen::VectorXd(), y0;
            if (!(flags & 1)) x0.setZero((Eigen::Index)n);
            y0.setZero((Eigen::Index)m);
            ok = ok && solver.setWarmStart(x0, y0) && solver.solveProblem() == OsqpEigen::ErrorExitFlag::NoError;
            const Eigen::VectorXd &x = solver.getSolution();
            ok = ok && x.size() == n;
            solver.clearSolver();
            if (!ok) {
                std::printf("bench: call %ld failed\n", c);
                return 1;
            }
        }
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (c >= warm) wall.push_back(ms);
    }
    // the same QPs alone on a direct one-QP batch: HIP-event time of the solve call (queue order +
    // kernel) and the kernel's dequeue-to-results latency
    impc_ctx ctx = nullptr;
    if (impc_ctx_create(0, &ctx)) return 1;
    impc_batch b = nullptr;
    if (impc_batch_create(ctx, n, m, Pp.data(), Pi.data(), Ap.data(), Ai.data(), 1, &b)) return 1;
    impc_settings st;
    impc_default_settings(&st);
    st.verbose = 0;
    impc_batch_set_settings(b, &st);
    impc_batch_set_profiling(b, 1);
    std::vector<double> ev_ms, lat_ms;
    const long dev_calls = std::min<long>(calls, 256);
    for (long c = 0; c < dev_calls + warm; c++) {
        const QP &Q = qps[(size_t)(c % nqp)];
        if (impc_batch_set_values(b, Q.Px.data(), Q.q.data(), Q.Ax.data(), Q.l.data(), Q.u.data())) return 1;
        std::vector<double> x0 = (flags & 1) ? Q.xw : std::vector<double>((size_t)n, 0.0);
        if (impc_batch_warm_start(b, x0.data(), nullptr) || impc_batch_solve(b, nullptr)) return 1;
        double su = 0, so = 0, ou = 0, lat = 0;
        if (impc_batch_get_timings(b, &su, &so, &ou) || impc_batch_get_qp_latency(b, &lat)) return 1;
        if (c >= warm) {
            ev_ms.push_back(so);
            lat_ms.push_back(lat);
        }
    }
    impc_batch_destroy(b);
    impc_ctx_destroy(ctx);
    std::printf("{\"calls\": %ld, \"qps\": %lld, \"n\": %lld, \"m\": %lld, \"pool\": %s, "
                "\"host_wall_ms\": {\"p50\": %.4f, \"p90\": %.4f, \"mean\": %.4f}, "
                "\"device_event_ms\": {\"p50\": %.4f, \"p90\": %.4f}, \"kernel_latency_ms\": {\"p50\": %.4f, "
                "\"p90\": %.4f}, \"overhead_p50_ms\": %.4f}\n",
                (long)wall.size(), (long long)nqp, (long long)n, (long long)m, OsqpEigen::detail::no_pool() ? "false" : "true",
                pct(wall, 0.5), pct(wall, 0.9), [&] { double s = 0; for (double v : wall) s += v; return s / (double)wall.size(); }(),
                pct(ev_ms, 0.5), pct(ev_ms, 0.9), pct(lat_ms, 0.5), pct(lat_ms, 0.9), pct(wall, 0.5) - pct(ev_ms, 0.5));
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 3 && std::strcmp(argv[1], "replay") == 0) return replay(argv[2], argv[3]);
    if (argc > 3 && std::strcmp(argv[1], "bench") == 0) return bench(argv[2], std::atol(argv[3]));
    const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
    // OSQP demo problem: P = [[4,1],[1,2]] (both triangles inserted, as Eigen users do),
    // q = (1,1), A = [[1,1],[1,0],[0,1]], l = (1,0,0), u = (1,0.7,0.7); x* = (0.3,0.7), y* = (-2.9,0,0.2)
    Eigen::SparseMatrix<double> P(2, 2), A(3, 2);
    P.insert(0, 0) = 4.0;
    P.insert(1, 0) = 1.0;
    P.insert(0, 1) = 1.0;
    P.insert(1, 1) = 2.0;
    A.insert(0, 0) = 1.0;
    A.insert(1, 0) = 1.0;
    A.insert(0, 1) = 1.0;
    A.insert(2, 1) = 1.0;
    Eigen::VectorXd q(2), l(3), u(3);
    q(0) = q(1) = 1.0;
    l(0) = 1.0, l(1) = 0.0, l(2) = 0.0;
    u(0) = 1.0, u(1) = 0.7, u(2) = 0.7;

    OsqpEigen::Solver solver;
    solver.settings()->setVerbosity(false);
    solver.settings()->setWarmStart(true);
    solver.settings()->setTimeLimit(0.05);
    solver.data()->setNumberOfVariables(2);
    solver.data()->setNumberOfConstraints(3);
    CHECK(solver.data()->setHessianMatrix(P));
    CHECK(solver.data()->setGradient(q));
    CHECK(solver.data()->setLinearConstraintsMatrix(A));
    CHECK(solver.data()->setLowerBound(l));
    CHECK(solver.data()->setUpperBound(u));
    // upper triangle, CSC, rows sorted (Data.tpp:38)
    const auto &d = *solver.data();
    CHECK(d.Pp.size() == 3 && d.Pp[0] == 0 && d.Pp[1] == 1 && d.Pp[2] == 3);
    CHECK(d.Pi.size() == 3 && d.Pi[0] == 0 && d.Pi[1] == 0 && d.Pi[2] == 1);
    CHECK(d.Px.size() == 3 && d.Px[0] == 4.0 && d.Px[1] == 1.0 && d.Px[2] == 2.0);
    CHECK(d.Ap.size() == 3 && d.Ap[2] == 4 && d.Ai[0] == 0 && d.Ai[1] == 1 && d.Ai[2] == 0 && d.Ai[3] == 2);
    // Data.hpp:99 / :145 accessors: the gradient, and OSQP's OSQPData view of the stored problem
    CHECK(solver.data()->getGradient().size() == 2 && solver.data()->getGradient()(1) == 1.0);
    {
        OSQPData *const &od = solver.data()->getData();
        CHECK(od && od->n == 2 && od->m == 3 && od->P && od->A && od->q && od->l && od->u);
        CHECK(od->P->n == 2 && od->P->nzmax == 3 && od->P->p[2] == 3 && od->P->i[2] == 1 && od->P->x[2] == 2.0);
        CHECK(od->A->m == 3 && od->A->p[2] == 4 && od->A->i[3] == 2 && od->A->nz == -1);
        CHECK(od->q[0] == 1.0 && od->l[0] == 1.0 && od->u[1] == 0.7);
    }
    // size errors are reported, not accepted
    Eigen::VectorXd bad(5);
    CHECK(!solver.data()->setGradient(bad));

    if (!gpu) {
        CHECK(!solver.initSolver());  // no device here: fails loudly, no CPU fallback
        CHECK(solver.solveProblem() == OsqpEigen::ErrorExitFlag::WorkspaceNotInitError);
        CHECK(solver.getStatus() == OsqpEigen::Status::Unsolved);
    } else {
        CHECK(solver.initSolver());
        CHECK(!solver.initSolver());  // already initialised
        Eigen::VectorXd x0, y0;
        x0.setZero(2);
        y0.setZero(3);
        CHECK(solver.setWarmStart(x0, y0));
        CHECK(solver.solveProblem() == OsqpEigen::ErrorExitFlag::NoError);
        CHECK(solver.getStatus() == OsqpEigen::Status::Solved);
        const Eigen::VectorXd &x = solver.getSolution();
        const Eigen::VectorXd &y = solver.getDualSolution();
        std::printf("x = (%.6f, %.6f) y = (%.6f, %.6f, %.6f) obj %.6f iters %lld\n", x(0), x(1), y(0), y(1), y(2),
                    solver.getObjValue(), (long long)solver.getIterations());
        CHECK(std::fabs(x(0) - 0.3) < 2e-3 && std::fabs(x(1) - 0.7) < 2e-3);
        CHECK(std::fabs(y(0) + 2.9) < 2e-2 && std::fabs(y(2) - 0.2) < 2e-2);
        // persistent update path: shift the bounds, re-solve
        Eigen::VectorXd l2(3), u2(3);
        l2(0) = 1.0, l2(1) = 0.0, l2(2) = 0.0;
        u2(0) = 1.0, u2(1) = 0.7, u2(2) = 0.6;
        CHECK(solver.updateBounds(l2, u2));
        CHECK(solver.solveProblem() == OsqpEigen::ErrorExitFlag::NoError);
        CHECK(solver.getStatus() == OsqpEigen::Status::Solved);
        CHECK(std::fabs(solver.getSolution()(1) - 0.6) < 2e-3);
        // reference-declared accessors: the iterate the next solve starts from, fixed-size templates
        Eigen::Matrix<double, 2, 1> xp;
        Eigen::Matrix<double, Eigen::Dynamic, 1> yd;
        CHECK(solver.getPrimalVariable(xp) && std::fabs(xp(1) - 0.6) < 2e-3);
        CHECK(solver.getDualVariable(yd) && yd.size() == 3);
        Eigen::Matrix<double, 3, 1> y3;
        y3(0) = y3(1) = y3(2) = 0.0;
        CHECK(solver.setDualVariable(y3));  // osqp_warm_start_y: x kept
        CHECK(solver.getPrimalVariable(xp) && std::fabs(xp(1) - 0.6) < 2e-3);
        // same-pattern Hessian update: P = [[4,1],[1,2]] -> [[8,2],[2,4]] with q doubled is the same QP
        // up to a factor 2 in the objective: x* unchanged
        Eigen::SparseMatrix<double> P2(2, 2);
        P2.insert(0, 0) = 8.0;
        P2.insert(1, 0) = 2.0;
        P2.insert(0, 1) = 2.0;
        P2.insert(1, 1) = 4.0;
        Eigen::VectorXd q2(2);
        q2(0) = q2(1) = 2.0;
        CHECK(solver.updateHessianMatrix(P2));
        CHECK(solver.updateGradient(q2));
        CHECK(solver.solveProblem() == OsqpEigen::ErrorExitFlag::NoError);
        CHECK(std::fabs(solver.getSolution()(1) - 0.6) < 2e-3);
        solver.clearSolver();
        CHECK(!solver.isInitialized());
        // an update before the first solve on the generic kernel (the demo QP's pattern is not
        // stage-structured): taken by the setup, as OsqpEigen's update after initSolver
        OsqpEigen::Solver s2;
        s2.settings()->setVerbosity(false);
        s2.data()->setNumberOfVariables(2);
        s2.data()->setNumberOfConstraints(3);
        CHECK(s2.data()->setHessianMatrix(P));
        CHECK(s2.data()->setGradient(q));
        CHECK(s2.data()->setLinearConstraintsMatrix(A));
        CHECK(s2.data()->setLowerBound(l));
        CHECK(s2.data()->setUpperBound(u));
        CHECK(s2.initSolver());
        CHECK(s2.updateBounds(l2, u2));
        CHECK(s2.updateGradient(q));
        CHECK(s2.solveProblem() == OsqpEigen::ErrorExitFlag::NoError);
        CHECK(s2.getStatus() == OsqpEigen::Status::Solved);
        CHECK(std::fabs(s2.getSolution()(1) - 0.6) < 2e-3);
        // a wrongly sized update is refused and leaves the data as it was
        Eigen::VectorXd bad2(4);
        CHECK(!s2.updateGradient(bad2));
        CHECK(s2.data()->q.size() == 2 && s2.data()->q[0] == 1.0);
        structured_case();
    }
    std::printf("%s: %d failure(s)\n", gpu ? "gpu" : "cpu", fails);
    return fails ? 1 : 0;
}
