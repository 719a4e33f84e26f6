"""GPU parity: libimpc_qp.so on MI355X vs the OSQP 0.6.2 oracle on identical (P, q, A, l, u).

Tolerance (BASELINE.json north_star): primal within 1e-5 relative (inf-norm over each QP); status
and iteration count identical; NaN-constant x (2143289344.0) for QPs without a solution.
"""
import numpy as np
import pytest

import impc
from impc import scenarios

from helpers import compare, gpu, oracle

pytestmark = pytest.mark.gpu

S25 = dict(verbose=0, adaptive_rho_interval=25)
KERNELS = pytest.mark.parametrize("kernel", [impc.KERNEL_GENERIC, impc.KERNEL_STRUCTURED], ids=["generic", "structured"])


@KERNELS
def test_config1_first_call(ctx, kernel):
    cfg = scenarios.first_call_config(batch=64, seed=101)
    s = impc.default_settings(**S25)
    compare(gpu(ctx, cfg, s, kernel), oracle(cfg, s))


@KERNELS
def test_config2_static_obstacles(ctx, kernel):
    cfg = scenarios.static_config(batch=96, identical=False, seed=202)
    s = impc.default_settings(**S25)
    compare(gpu(ctx, cfg, s, kernel), oracle(cfg, s))


@KERNELS
def test_config3_intent_hypotheses(ctx, kernel):
    buckets = scenarios.intent_config(instances=24, seed=303)
    s = impc.default_settings(**S25)
    for K, bk in buckets.items():
        compare(gpu(ctx, bk, s, kernel), oracle(bk, s))


@KERNELS
def test_default_auto_interval_matches_pinned(ctx, kernel):
    """adaptive_rho_interval = 0 resolves to check_termination (25) on the device."""
    cfg = scenarios.static_config(batch=32, identical=False, seed=404)
    r0 = gpu(ctx, cfg, impc.default_settings(verbose=0), kernel)
    r25 = gpu(ctx, cfg, impc.default_settings(**S25), kernel)
    assert np.array_equal(r0[0], r25[0]) and np.array_equal(r0[2]["iter"], r25[2]["iter"])


@KERNELS
def test_identical_batch_full_size(ctx, kernel):
    """Config 2 shape at batch 4096: every copy of one QP gives bitwise the same answer, and that
    answer matches the oracle's single solve (size-independent property at full batch)."""
    cfg = scenarios.static_config(batch=4096, identical=True, seed=2000)
    s = impc.default_settings(verbose=0)
    x, y, info = gpu(ctx, cfg, s, kernel)
    assert np.all(x == x[0]) and np.all(info["iter"] == info["iter"][0])
    one = dict(cfg, values={k: v[:1] for k, v in cfg["values"].items()})
    compare((x[:1], y[:1], info[:1]), oracle(one, s))


def test_auto_selects_structured_for_mpc_patterns(ctx):
    for cfg in (scenarios.first_call_config(batch=2), scenarios.static_config(batch=2)):
        pat = cfg["pattern"]
        b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], 2)
        try:
            st = b.stats()
            assert st["structured_ok"] == 1 and st["kernel"] == impc.KERNEL_STRUCTURED
        finally:
            b.close()


@KERNELS
def test_nonbinding_time_limit_changes_nothing(ctx, kernel):
    """time_limit reads the device clock inside the ADMM loop; a limit that never triggers must
    leave every result bitwise unchanged (the reference passes 0.05 s, mpcPlanner.cpp:440-444)."""
    cfg = scenarios.static_config(batch=64, identical=False, seed=515)
    r0 = gpu(ctx, cfg, impc.default_settings(**S25), kernel)
    r1 = gpu(ctx, cfg, impc.default_settings(time_limit=100.0, **S25), kernel)
    assert np.array_equal(r0[0], r1[0]) and np.array_equal(r0[2]["iter"], r1[2]["iter"])
    assert np.array_equal(r0[2]["status_val"], r1[2]["status_val"])


@KERNELS
def test_binding_time_limit_status(ctx, kernel):
    """A limit far below one solve's duration stops every QP with OSQP_TIME_LIMIT_REACHED (-6)
    and a primal iterate (x is reported, not NaN), as osqp_solve does (osqp.c time check)."""
    cfg = scenarios.static_config(batch=32, identical=False, seed=616)
    x, y, info = gpu(ctx, cfg, impc.default_settings(time_limit=1e-7, **S25), kernel)
    assert np.all(info["status_val"] == impc.TIME_LIMIT_REACHED)
    assert np.all(np.isfinite(x)) and not np.any(x == impc.OSQP_NAN)


@KERNELS
@pytest.mark.parametrize("N", [3, 6, 11, 19, 20, 21, 30, 40])
def test_horizons(ctx, kernel, N):
    """Stage counts W = N-1 of both parities and short horizons (the structured kernel's paired
    recursions have single-step heads/tails for odd W)."""
    cfg = scenarios.static_config(N=N, K=3, batch=24, identical=False, seed=900 + N)
    s = impc.default_settings(**S25)
    compare(gpu(ctx, cfg, s, kernel), oracle(cfg, s))


@pytest.mark.parametrize("K", [3, 10, 11, 14])
def test_long_horizon_chunked_recursions(ctx, K):
    """N = 40 (W = 39): the long shape's stage recursions in four chunks on the four wavefronts
    (chunk ends from zero, starts from the chunk operators, chunks re-run), over two, three and four
    general-row slots per lane; rho = 1e-3 forces adaptive-rho refactorisations, which rebuild the
    chunk operators."""
    cfg = scenarios.static_config(N=40, K=K, batch=48, identical=False, seed=4000 + K)
    for rho in (0.1, 1e-3):
        s = impc.default_settings(rho=rho, **S25)
        ref = oracle(cfg, s)
        compare(gpu(ctx, cfg, s, impc.KERNEL_STRUCTURED), ref)
        if rho < 0.1:
            assert ref[2]["rho_updates"].max() >= 1


@pytest.mark.parametrize("rho", [0.1, 1e-3])
def test_live_horizon_N30_intent_buckets(ctx, rho):
    """N = 30, the reference's live planner horizon (planner_param.yaml:25): the long shape's
    compile-time W = 29 instance (chunked recursions of 8 / 8 / 8 / 5 steps).  The K = 8 / 9
    intent buckets of config 3's generator at N = 30, warm-started from the previous plan, in ONE
    grouped launch, against the oracle; rho = 1e-3 forces refactorisations (chunk operators
    rebuilt)."""
    buckets = scenarios.intent_config(N=30, K=8, instances=24, hyps=8, seed=3030 if rho == 0.1 else 3031)
    s = impc.default_settings(rho=rho, **S25)
    bs = []
    try:
        for K, bk in sorted(buckets.items()):
            pat, v = bk["pattern"], bk["values"]
            b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], v["q"].shape[0])
            b.set_settings(s)
            b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
            b.warm_start(bk["x_ws"], None)
            st = b.stats()
            assert st["kernel"] == impc.KERNEL_STRUCTURED and st["var_slots"] == 3, st
            bs.append((b, bk))
        impc.solve_group([b for b, _ in bs])
        upd = 0
        for b, bk in bs:
            ref = oracle(bk, s)
            compare(b.get(), ref)
            upd += int(ref[2]["rho_updates"].max())
        if rho < 0.1:
            assert upd >= 1
    finally:
        for b, _ in bs:
            b.close()


def test_grouped_launch_equals_separate_solves(ctx):
    """impc_batch_solve_group over the K / K+1 buckets of a replan gives bitwise the results of
    separate impc_batch_solve calls (one work queue, per-batch tables)."""
    buckets = scenarios.intent_config(instances=40, seed=808)
    s = impc.default_settings(verbose=0, adaptive_rho_interval=25)

    def make():
        out = []
        for K, bk in sorted(buckets.items()):
            pat, v = bk["pattern"], bk["values"]
            b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], v["q"].shape[0])
            b.set_settings(s)
            b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
            b.warm_start(bk["x_ws"], None)
            out.append(b)
        return out

    sep = make()
    for b in sep:
        b.solve()
    ref = [b.get() for b in sep]
    grp = make()
    impc.solve_group(grp)
    impc.solve_group(grp)  # repeated launch of the same group (cached entries)
    got = [b.get() for b in grp]
    for (x0, y0, i0), (x1, y1, i1) in zip(ref, got):
        assert np.array_equal(x0, x1) and np.array_equal(y0, y1) and np.array_equal(i0["iter"], i1["iter"])
    for b in sep + grp:
        b.close()


def solve_shared(ctx, cfg, settings, kernel):
    pat, v = cfg["pattern"], cfg["values"]
    B = v["q"].shape[0]
    split = impc.shared_split(v["Px"], v["Ax"])
    assert split is not None
    Px0, Ax0, var, Axv = split
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    try:
        b.set_kernel(kernel)
        b.set_settings(settings)
        b.set_values_shared(Px0, Ax0, var, Axv, v["q"], v["l"], v["u"])
        if cfg.get("x_ws") is not None:
            b.warm_start(cfg["x_ws"], None)
        b.solve()
        return b.get(), var.size
    finally:
        b.close()


@KERNELS
def test_shared_structure_values_match_full_values(ctx, kernel):
    """impc_batch_set_values_shared (P and the dynamics / box entries of A once, obstacle-row
    entries per QP) gives bitwise the results of impc_batch_set_values on the same QPs."""
    buckets = scenarios.intent_config(instances=16, seed=606)
    s = impc.default_settings(**S25)
    for K, bk in buckets.items():
        (xs, ys, infs), nvar = solve_shared(ctx, bk, s, kernel)
        assert 0 < nvar < bk["values"]["Ax"].shape[1]
        xf, yf, inff = gpu(ctx, bk, s, kernel)
        np.testing.assert_array_equal(xs, xf)
        np.testing.assert_array_equal(ys, yf)
        np.testing.assert_array_equal(infs["iter"], inff["iter"])


def test_per_qp_latency_recorded_by_structured_kernel(ctx):
    cfg = scenarios.static_config(batch=64, identical=False, seed=808)
    pat, v = cfg["pattern"], cfg["values"]
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], 64)
    try:
        b.set_settings(impc.default_settings(verbose=0))
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.set_profiling(True)
        b.set_kernel(impc.KERNEL_STRUCTURED)
        b.solve()
        lat = b.qp_latency()
        assert np.all(lat > 0) and np.all(lat < 1000)
        b.set_kernel(impc.KERNEL_GENERIC)
        b.solve()
        with pytest.raises(impc.ImpcError):
            b.qp_latency()
    finally:
        b.close()


@KERNELS
@pytest.mark.parametrize("K", [19, 20])
def test_many_obstacles_three_general_row_slots(ctx, kernel, K):
    """Config 4's largest buckets: K = 19, 20 obstacles push the general rows past 512 (the
    structured kernel's three-slot shape, and its larger products region)."""
    cfg = scenarios.static_config(N=20, K=K, batch=16, identical=False, seed=950 + K)
    s = impc.default_settings(**S25)
    compare(gpu(ctx, cfg, s, kernel), oracle(cfg, s))
