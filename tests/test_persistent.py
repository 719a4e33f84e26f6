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


@pytest.mark.parametrize("which", ["P", "A", "PA", "A+q"])
def test_matrix_update_matches_osqp_update_P_A(ctx, which):
    """impc_batch_update_matrices on a persistent structured workspace against the oracle's
    osqp_update_P / _A / _P_A (ora_update_P_A: unscale_data, new values, scale_data, refactor, the
    scaled iterates kept): setup + solve -> update q -> solve -> new P and / or A -> solve -> update
    bounds -> solve (the replayed scaling is the new one).  Identical statuses and iteration counts,
    primal within 1e-5 relative at every step."""
    cfg = scenarios.static_config(N=20, K=4, batch=12, identical=False, seed=518)
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
