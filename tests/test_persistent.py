"""Persistent workspaces (osqp_update_lin_cost / osqp_update_bounds between solves, as a persistent
OsqpEigen::Solver does, polyTrajSolver.cpp:183-237): both kernels against the oracle's persistent
workspace (oracle/osqp_oracle.c ora_update_*, osqp.h:114,125) over a sequence setup+solve ->
update q -> solve -> update bounds -> solve.  Identical statuses and iteration counts, primal
within 1e-5 relative at every step."""
import numpy as np
import pytest

import impc
from impc import scenarios
from oracle import osqp_oracle as ora

pytestmark = pytest.mark.gpu

KERNELS = pytest.mark.parametrize("kernel", [impc.KERNEL_GENERIC, impc.KERNEL_STRUCTURED],
                                  ids=["generic", "structured"])


def check(x, info, ref, rtol=1e-5):
    xr, _, ir = ref
    assert info["status_val"] == ir["status_val"] and info["iter"] == ir["iter"], (info, ir)
    if ir["status_val"] in (1, 2):
        assert np.abs(x - xr).max() <= rtol * max(np.abs(xr).max(), 1e-12)


@KERNELS
@pytest.mark.parametrize("warm", [1, 0], ids=["warm", "cold"])
def test_update_sequence_matches_persistent_oracle(ctx, kernel, warm):
    """warm = 0: every osqp_solve cold-starts its iterates (osqp.c osqp_solve, oracle
    ora_solve :1140) but keeps the scaling, rho and factor of the workspace."""
    cfg = scenarios.static_config(N=20, K=4, batch=12, identical=False, seed=515)
    pat, v = cfg["pattern"], cfg["values"]
    B = v["q"].shape[0]
    s = impc.default_settings(verbose=0, adaptive_rho_interval=25, warm_start=warm)
    rng = np.random.default_rng(9)
    q2 = v["q"] * (1 + 0.05 * rng.standard_normal(v["q"].shape))
    # bounds update: shift the finite box bounds of the states a little
    l3, u3 = v["l"].copy(), v["u"].copy()
    fin = np.isfinite(l3) & np.isfinite(u3) & (u3 - l3 > 1e-3)
    l3[fin] -= 0.05
    u3[fin] += 0.05
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    try:
        b.set_kernel(kernel)
        b.set_settings(s)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        if kernel == impc.KERNEL_STRUCTURED:
            b.set_persistent(True)
        b.solve()
        r1 = b.get()
        b.update_lin_cost(q2)
        b.solve()
        r2 = b.get()
        b.update_bounds(l3, u3)
        b.solve()
        r3 = b.get()
    finally:
        b.close()
    os_ = ora.settings_from(s)
    for i in range(B):
        w = ora.Workspace(pat, v["Px"][i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], os_)
        check(r1[0][i], r1[2][i], w.solve())
        w.update_lin_cost(q2[i])
        check(r2[0][i], r2[2][i], w.solve())
        w.update_bounds(l3[i], u3[i])
        check(r3[0][i], r3[2][i], w.solve())
        w.close()


def test_structured_updates_need_persistence(ctx):
    cfg = scenarios.static_config(N=20, K=2, batch=4, identical=False, seed=516)
    pat, v = cfg["pattern"], cfg["values"]
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], 4)
    try:
        b.set_kernel(impc.KERNEL_STRUCTURED)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.solve()
        with pytest.raises(impc.ImpcError):
            b.update_lin_cost(v["q"])
    finally:
        b.close()


@KERNELS
def test_explicit_warm_start_between_updates(ctx, kernel):
    """osqp_warm_start on a persistent workspace replaces its iterates and turns the warm_start
    setting on (oracle ora_warm_start :1092-1094), keeping scaling and rho."""
    cfg = scenarios.static_config(N=20, K=3, batch=8, identical=False, seed=517)
    pat, v = cfg["pattern"], cfg["values"]
    B = v["q"].shape[0]
    s = impc.default_settings(verbose=0, adaptive_rho_interval=25, warm_start=0)
    rng = np.random.default_rng(11)
    q2 = v["q"] * (1 + 0.05 * rng.standard_normal(v["q"].shape))
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    try:
        b.set_kernel(kernel)
        b.set_settings(s)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        if kernel == impc.KERNEL_STRUCTURED:
            b.set_persistent(True)
        b.solve()
        r1 = b.get()
        xw = r1[0] * 1.01
        yw = r1[1] * 0.99
        b.update_lin_cost(q2)
        b.warm_start(xw, yw)
        b.solve()
        r2 = b.get()
        b.update_lin_cost(v["q"])  # warm_start is on now: the next solve resumes
        b.solve()
        r3 = b.get()
    finally:
        b.close()
    os_ = ora.settings_from(s)
    for i in range(B):
        w = ora.Workspace(pat, v["Px"][i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], os_)
        check(r1[0][i], r1[2][i], w.solve())
        w.update_lin_cost(q2[i])
        w.warm_start(xw[i], yw[i])
        check(r2[0][i], r2[2][i], w.solve())
        w.update_lin_cost(v["q"][i])
        check(r3[0][i], r3[2][i], w.solve())
        w.close()


@pytest.mark.parametrize("N,which", [(20, "P"), (20, "A"), (20, "PA"), (20, "A+q"), (30, "A"), (30, "A+q"),
                                     (40, "P"), (40, "A"), (40, "PA"), (40, "A+q")])
def test_matrix_update_matches_osqp_update_P_A(ctx, N, which):
    """impc_batch_update_matrices on a persistent structured workspace against the oracle's
    osqp_update_P / _A / _P_A (ora_update_P_A: unscale_data, new values, scale_data, refactor, the
    scaled iterates kept): setup + solve -> update q -> solve -> new P and / or A -> solve -> update
    bounds -> solve (the replayed scaling is the new one).  Identical statuses and iteration counts,
    primal within 1e-5 relative at every step.  N = 20 runs the W = 19 instance, N = 30 / 40 the long
    shape's chunked W = 29 / W = 39 instances (resume mode 2, the config-5 closed loop's path)."""
    cfg = scenarios.static_config(N=N, K=4, batch=12, identical=False, seed=518 + N)
    pat, v = cfg["pattern"], cfg["values"]
    B = v["q"].shape[0]
    s = impc.default_settings(verbose=0, adaptive_rho_interval=25)
    rng = np.random.default_rng(12)
    q2 = v["q"] * (1 + 0.05 * rng.standard_normal(v["q"].shape))
    P3 = v["Px"] * (1.0 + 0.5 * rng.uniform(size=v["Px"].shape)) if "P" in which else None
    A3 = v["Ax"] * (1.0 + 0.02 * rng.standard_normal(v["Ax"].shape)) if "A" in which else None
    q5 = v["q"] * (1 + 0.3 * rng.standard_normal(v["q"].shape))
    l4, u4 = v["l"].copy(), v["u"].copy()
    fin = np.isfinite(l4) & np.isfinite(u4) & (u4 - l4 > 1e-3)
    l4[fin] -= 0.05
    u4[fin] += 0.05
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    try:
        b.set_kernel(impc.KERNEL_STRUCTURED)
        b.set_settings(s)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.set_persistent(True)
        with pytest.raises(impc.ImpcError):  # before the first solve there is no workspace to update
            b.update_matrices(P3, A3)
        b.solve()
        r1 = b.get()
        b.update_lin_cost(q2)
        b.solve()
        r2 = b.get()
        b.update_matrices(P3, A3)
        if which == "A+q":  # q after the matrices: OSQP scaled the cost with the q held at the update
            b.update_lin_cost(q5)
        b.solve()
        r3 = b.get()
        b.update_bounds(l4, u4)
        b.solve()
        r4 = b.get()
    finally:
        b.close()
    os_ = ora.settings_from(s)
    for i in range(B):
        w = ora.Workspace(pat, v["Px"][i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], os_)
        check(r1[0][i], r1[2][i], w.solve())
        w.update_lin_cost(q2[i])
        check(r2[0][i], r2[2][i], w.solve())
        w.update_matrices(None if P3 is None else P3[i], None if A3 is None else A3[i])
        if which == "A+q":
            w.update_lin_cost(q5[i])
        check(r3[0][i], r3[2][i], w.solve())
        w.update_bounds(l4[i], u4[i])
        check(r4[0][i], r4[2][i], w.solve())
        w.close()


def test_nonconvex_first_solve_then_convex_matrix_update(ctx):
    """An indefinite P: a QP whose first setup fails to factorise (P + sigma I + A'RA not positive
    definite: osqp_setup returns OSQP_NONCVX_ERROR, no workspace; here status NON_CVX with
    setup_exitflag 5) leaves a defined workspace (the settings' rho, zero iterates), and a convex P
    then given through impc_batch_update_matrices solves exactly as an oracle setup from scratch
    with that P.  A QP that factorises but diverges (status NON_CVX from the residual test) keeps
    its workspace with the iterates cold-started (store_solution), as the oracle's does through
    osqp_update_P.  The other QPs of the batch follow the oracle's setup -> solve -> osqp_update_P
    -> solve."""
    cfg = scenarios.static_config(N=20, K=4, batch=8, identical=False, seed=520)
    pat, v = cfg["pattern"], cfg["values"]
    B = v["q"].shape[0]
    s = impc.default_settings(verbose=0, adaptive_rho_interval=25)
    bad = np.arange(B) % 2 == 0
    Pbad = v["Px"].copy()
    Pbad[bad] = -1e4
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    try:
        b.set_kernel(impc.KERNEL_STRUCTURED)
        b.set_settings(s)
        b.set_values(Pbad, v["q"], v["Ax"], v["l"], v["u"])
        b.set_persistent(True)
        b.solve()
        r1 = b.get()
        rho, xs, zs, ys = b.get_persistent()
        b.update_matrices(v["Px"], None)
        b.solve()
        r2 = b.get()
    finally:
        b.close()
    os_ = ora.settings_from(s)
    kinds = set()
    for i in range(B):
        try:
            w = ora.Workspace(pat, Pbad[i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], os_)
        except RuntimeError:  # OSQP: osqp_setup fails, no workspace
            kinds.add("setup")
            assert r1[2][i]["status_val"] == -7 and r1[2][i]["setup_exitflag"] == 5, r1[2][i]
            assert rho[i] == s.rho and not xs[i].any() and not zs[i].any() and not ys[i].any()
            w = ora.Workspace(pat, v["Px"][i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], os_)
            check(r2[0][i], r2[2][i], w.solve())
            w.close()
            continue
        x1 = w.solve()
        check(r1[0][i], r1[2][i], x1)
        if x1[2]["status_val"] == -7:
            kinds.add("diverged")
            assert not xs[i].any() and not zs[i].any() and not ys[i].any()  # store_solution's cold_start
        w.update_matrices(v["Px"][i], None)
        check(r2[0][i], r2[2][i], w.solve())
        w.close()
    assert kinds == {"setup", "diverged"}  # the scenario reaches both kinds


@KERNELS
def test_failed_rho_update_ends_the_solve_unsolved(ctx, kernel):
    """osqp_solve with an adaptive-rho update whose refactorisation fails (P indefinite, but
    P + sigma I + A'RA positive definite at the first rho) returns exitflag 1 with the status still
    UNSOLVED at the iteration of that update (osqp.c, adapt_rho -> goto exit; oracle ora_solve_ws).
    The seed's third QP is left out: with an indefinite P its iterates grow until the rho update,
    and the iteration at which that happens differs between any two implementations (the oracle
    1,025, the kernels' CPU builds 900 / 925, the generic kernel on MI355X 675; same status)."""
    cfg = scenarios.static_config(N=20, K=4, batch=4, identical=False, seed=520)
    pat, v = cfg["pattern"], cfg["values"]
    keep = [0, 1, 3]
    v = {k: a[keep] for k, a in v.items()}
    B = v["q"].shape[0]
    s = impc.default_settings(verbose=0, adaptive_rho_interval=25)
    P = np.full_like(v["Px"], -1e3)
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    try:
        b.set_kernel(kernel)
        b.set_settings(s)
        b.set_values(P, v["q"], v["Ax"], v["l"], v["u"])
        b.solve()
        _, _, info = b.get()
    finally:
        b.close()
    _, _, io = ora.solve_batch(pat, P, v["q"], v["Ax"], v["l"], v["u"], ora.settings_from(s))
    assert (io["status_val"] == -10).any()  # the scenario does reach a failed rho update
    np.testing.assert_array_equal(info["status_val"], io["status_val"])
    np.testing.assert_array_equal(info["iter"], io["iter"])
    np.testing.assert_array_equal(info["rho_updates"], io["rho_updates"])


def test_solve_without_solution_cold_starts_the_next(ctx):
    """store_solution (auxil.c): a solve that ends without a solution (primal infeasible here)
    cold-starts the workspace's iterates, so the next solve after osqp_update_bounds starts from
    zero -- not from the divergent iterates -- as the oracle's persistent workspace does."""
    cfg = scenarios.static_config(N=20, K=4, batch=4, identical=False, seed=606)
    pat, v = cfg["pattern"], cfg["values"]
    B = v["q"].shape[0]
    s = impc.default_settings(verbose=0, adaptive_rho_interval=25)
    l1 = v["l"].copy()
    l1[0, 8 * 20 + 1] = 4.9  # box row contradicting the pinned x0 -> primal infeasible
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    try:
        b.set_kernel(impc.KERNEL_STRUCTURED)
        b.set_settings(s)
        b.set_values(v["Px"], v["q"], v["Ax"], l1, v["u"])
        b.set_persistent(True)
        b.solve()
        r1 = b.get()
        _, xs, zs, ys = b.get_persistent()
        b.update_bounds(v["l"], v["u"])
        b.solve()
        r2 = b.get()
    finally:
        b.close()
    os_ = ora.settings_from(s)
    assert r1[2][0]["status_val"] == -3
    assert not xs[0].any() and not zs[0].any() and not ys[0].any()
    for i in range(B):
        w = ora.Workspace(pat, v["Px"][i], v["q"][i], v["Ax"][i], l1[i], v["u"][i], os_)
        check(r1[0][i], r1[2][i], w.solve())
        w.update_bounds(v["l"][i], v["u"][i])
        check(r2[0][i], r2[2][i], w.solve())
        w.close()


def test_matrix_update_generic_kernel_is_refused(ctx):
    cfg = scenarios.static_config(N=20, K=2, batch=4, identical=False, seed=519)
    pat, v = cfg["pattern"], cfg["values"]
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], 4)
    try:
        b.set_kernel(impc.KERNEL_GENERIC)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.solve()
        with pytest.raises(impc.ImpcError) as e:
            b.update_matrices(v["Px"], None)
        assert e.value.code == 102  # IMPC_UNSUPPORTED
    finally:
        b.close()
