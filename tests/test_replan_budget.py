"""The replan's wall-clock budget (makePlanWithPred, mpcPlanner.cpp:609-628): the 0.15 s candidate
issue cut-off, timeLimit = max(solverTimeLimit_ - time, solverTimeLimit_) on every candidate of an
instance that is not on its first plan (solveTraj sets it only when not firstTime_, :442-444), and
the selection over the candidates whose solveTraj succeeded (initSolver and solveProblem NoError,
:475-478, :513-518).  The limit is measured on the device's constant-rate clock, whose rate is read from
the device (hipDeviceAttributeWallClockRate) and checked against HIP events here."""
import time

import numpy as np
import pytest

import impc
from impc import scenarios
from impc.replan import ISSUE_CUTOFF_S, DeviceReplan, candidate_valid


def test_candidate_valid_maps_slots_to_batch_rows():
    # two instances; slot < 4 -> single-intent row 4i+slot, else two-intent row 2i+slot-4; a
    # candidate is valid when solveTraj succeeded: setup ok and solveProblem NoError -- every final
    # status (TIME_LIMIT_REACHED, a diverged NON_CVX) but a failed setup or a failed rho update
    slot = np.array([[0, 1, 2, 3, 4, 5], [4, 0, 5, 1, 2, 3]])
    info_s = np.zeros(8, impc.INFO_DTYPE)
    info_s["status_val"] = [1, 1, 1, impc.NON_CVX, 1, impc.TIME_LIMIT_REACHED, 1, 1]
    info_s["setup_exitflag"][3] = 5                       # initSolver failed (OSQP_NONCVX_ERROR)
    info_p = np.zeros(4, impc.INFO_DTYPE)
    info_p["status_val"] = [1, impc.NON_CVX, -10, 1]    # diverged (valid) / failed rho update (not)
    got = candidate_valid(slot, info_s, info_p)
    np.testing.assert_array_equal(got, [[1, 1, 1, 0, 1, 1], [0, 1, 1, 1, 1, 1]])
    assert got.dtype == np.int8
    assert ISSUE_CUTOFF_S == 0.15


def _scenario(I=16, K=3, N=20, seed=811, first_time=None):
    buckets = scenarios.intent_config(N=N, K=K, instances=I, hyps=6, seed=seed)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    L = inst["pred"].shape[3]
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    ft = np.zeros(I, np.int8) if first_time is None else np.asarray(first_time, np.int8)
    args = (inst["pos"], inst["vel"], inst["xref"], inst["prev"], ft, np.full(I, N, np.int32),
            inst["obp"], inst["pred"], pred_size, inst["prob_all"])
    return p, pd, I, K, L, args


def _describe(lim, free, nm, rows):
    st, it = lim["info_" + nm]["status_val"], lim["info_" + nm]["iter"]
    lat = lim["lat_" + nm]
    return "; ".join(f"{nm}[{r}] status {st[r]} iter {it[r]} (free {free['info_' + nm]['iter'][r]}) "
                     f"latency {lat[r]:.3f} ms" for r in rows[:12])


@pytest.mark.gpu
def test_device_clock_rate_matches_hip_events(ctx):
    hz = ctx.clock_rate()
    assert 1e6 <= hz <= 1e10, hz
    ctx.clock_check(0.001)  # the first launch also loads the module between the events
    for s in (0.02, 0.1):
        ev = ctx.clock_check(s)
        # one launch of one wavefront: launch overhead is microseconds
        assert abs(ev - s) <= 0.02 * s + 2e-4, (s, ev, hz)


@pytest.mark.gpu
def test_budget_nonbinding_limit_is_bit_identical(ctx):
    """A limit no QP comes near (100 s) takes the grouped kernel's time-limited loop (deltas every
    iteration, a team clock reduction per iteration) and must change nothing."""
    p, pd, I, K, L, args = _scenario()
    rp = DeviceReplan(ctx, p, pd, I, K, L, impc.default_settings(verbose=0))
    try:
        free = rp.run(*args)
        lim = rp.run(*args, solver_time_limit=100.0, profile=True)
        assert lim["issued"] and lim["time_limit"] == 100.0
        for nm in ("single", "pair"):
            np.testing.assert_array_equal(lim["info_" + nm]["status_val"], free["info_" + nm]["status_val"])
            np.testing.assert_array_equal(lim["info_" + nm]["iter"], free["info_" + nm]["iter"])
            np.testing.assert_array_equal(lim["x_" + nm], free["x_" + nm])
            assert (lim["lat_" + nm] > 0).all() and (lim["lat_" + nm] < 1e5).all()
        np.testing.assert_array_equal(lim["best_cand"], free["best_cand"])
    finally:
        rp.close()


@pytest.mark.gpu
def test_budget_time_limit_and_cutoff(ctx):
    p, pd, I, K, L, args = _scenario()
    rp = DeviceReplan(ctx, p, pd, I, K, L, impc.default_settings(verbose=0))
    try:
        free = rp.run(*args)
        # solverTimeLimit_ = 0.05 s (mpcPlanner.cpp:167), counted on the device clock from the tick
        # the QP's setup starts.  Strict: a QP that reports OSQP_TIME_LIMIT_REACHED must have run at
        # least that long by the same clock (its recorded latency), and every other QP is bit-identical
        # to the unlimited replan
        lim = rp.run(*args, solver_time_limit=0.05, profile=True)
        assert lim["issued"] and lim["time_limit"] == 0.05
        hit_any = False
        for nm in ("single", "pair"):
            st = lim["info_" + nm]["status_val"]
            hit = st == impc.TIME_LIMIT_REACHED
            hit_any |= bool(hit.any())
            early = np.flatnonzero(hit & (lim["lat_" + nm] < 50.0))
            assert early.size == 0, "time limit fired early: " + _describe(lim, free, nm, early)
            ok = ~hit
            diff = np.flatnonzero(ok & ((lim["x_" + nm] != free["x_" + nm]).any(axis=1) |
                                        (lim["info_" + nm]["iter"] != free["info_" + nm]["iter"])))
            assert diff.size == 0, "QPs inside the limit differ: " + _describe(lim, free, nm, diff)
            assert (lim["info_" + nm]["iter"][hit] <= free["info_" + nm]["iter"][hit]).all()
        if not hit_any:
            np.testing.assert_array_equal(lim["best_cand"], free["best_cand"])
        assert (lim["valid"] == 1).all() and (lim["best_cand"] >= 0).all()
        # a time limit every QP exceeds: OSQP_TIME_LIMIT_REACHED is still a successful solveTraj,
        # so every candidate stays in the selection
        tiny = rp.run(*args, solver_time_limit=1e-9)
        assert tiny["time_limit"] == 1e-9
        for nm in ("single", "pair"):
            st = tiny["info_" + nm]["status_val"]
            # the post-loop check_termination may still call a warm-started QP solved
            assert (st == impc.TIME_LIMIT_REACHED).mean() >= 0.5 and (st != impc.NON_CVX).all()
            assert (tiny["info_" + nm]["iter"] < free["info_" + nm]["iter"]).all()
        assert (tiny["valid"] == 1).all() and (tiny["best_cand"] >= 0).all()
        # past the 0.15 s cut-off no candidate is issued: validTraj = false for every instance
        late = rp.run(*args, t_start=time.perf_counter() - 1.0)
        assert not late["issued"] and late["x_single"] is None and late["info_pair"] is None
        assert (late["valid"] == 0).all() and (late["best_cand"] == -1).all()
    finally:
        rp.close()


@pytest.mark.gpu
def test_per_qp_time_limits_generic_and_structured(ctx):
    """impc_batch_set_time_limits on both kernels: QPs with limit 0 run to completion bit-identically,
    QPs with a limit below their solve time stop with OSQP_TIME_LIMIT_REACHED; clearing restores
    the settings' limit."""
    buckets = scenarios.intent_config(N=20, K=8, instances=4, hyps=8, seed=5)
    bk = buckets[min(buckets)]
    pat, v = bk["pattern"], bk["values"]
    B = v["q"].shape[0]
    for kernel in (impc.KERNEL_STRUCTURED, impc.KERNEL_GENERIC):
        b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B).set_kernel(kernel)
        try:
            b.set_settings(impc.default_settings(verbose=0))
            b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
            b.warm_start(bk["x_ws"], None)
            b.solve()
            x0, _, i0 = b.get()
            tl = np.where(np.arange(B) % 2 == 0, 0.0, 1e-9)
            b.set_time_limits(tl)
            b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
            b.warm_start(bk["x_ws"], None)
            b.solve()
            x1, _, i1 = b.get()
            free = tl == 0
            np.testing.assert_array_equal(x1[free], x0[free])
            np.testing.assert_array_equal(i1["iter"][free], i0["iter"][free])
            assert (i1["status_val"][~free] == impc.TIME_LIMIT_REACHED).mean() >= 0.5
            b.set_time_limits(None)
            b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
            b.warm_start(bk["x_ws"], None)
            b.solve()
            x2, _, i2 = b.get()
            np.testing.assert_array_equal(x2, x0)
            with pytest.raises(impc.ImpcError):
                b.set_time_limits(np.full(B, -1.0))
        finally:
            b.close()
