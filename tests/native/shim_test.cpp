// TEST INFRASTRUCTURE ONLY -- drives include/OsqpEigen/OsqpEigen.h with the call sequence of
// mpcPlanner::solveTraj (reference mpcPlanner.cpp:436-527), against the Eigen stand-in.
//   shim_test cpu : conversion checks + graceful failure without a device (exit 0 = pass)
//   shim_test gpu : OSQP demo QP through the shim on the GPU (x*, y*, status) (exit 0 = pass)
#include <cmath>
#include <cstdio>
#include <cstring>

#include <OsqpEigen/OsqpEigen.h>

static int fails = 0;
#define CHECK(c)                                                   \
    do {                                                           \
        if (!(c)) {                                                \
            std::printf("CHECK failed line %d: %s\n", __LINE__, #c); \
            fails++;                                               \
        }                                                          \
    } while (0)

int main(int argc, char **argv) {
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
        solver.clearSolver();
        CHECK(!solver.isInitialized());
    }
    std::printf("%s: %d failure(s)\n", gpu ? "gpu" : "cpu", fails);
    return fails ? 1 : 0;
}
