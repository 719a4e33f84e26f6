"""Config 5's closed receding loop on the device (bench.py RecedingLoop) against the oracle's
persistent workspaces, step by step, at a size the oracle finishes in seconds: per step every QP's
next x0 and linearisation point come from its own last solution (impc_batch_follow_plan_device =
mpcPlanner::getPos / getVel(dt), mpc_node.cpp:216-224, and currentStatesSol_, mpcPlanner.cpp:636-639),
the reference and the predicted obstacles move one step on (impc_copy_rows_device), the device
builder rebuilds the QP (castMPCToQP*), and the workspace takes osqp_update_A / _lin_cost / _bounds
(impc_batch_update_matrices_device, ...) before the solve.  The oracle chain replays the same
updates with the device-built values (bench.cpu_baseline_receding).  Parity is unpinned against the
real libosqp."""
import math

import numpy as np
import pytest

import impc
from impc import scenarios

import bench
from helpers import PRIMAL_RTOL

pytestmark = pytest.mark.gpu


def _loop(ctx, N, K, instances, steps, seed):
    settings = impc.default_settings(verbose=0)
    buckets = scenarios.intent_config(N=N, K=K, instances=instances, hyps=8, seed=seed)
    bks = [bk for _, bk in sorted(buckets.items())]
    batches = [(bk, bench.make_batch(impc, ctx, bk, settings, False, profile=False)[0]) for bk in bks]
    rec = bench.RecedingLoop(impc, ctx, batches, steps)
    return settings, bks, batches, rec


def _check_chain(rec, settings, steps):
    """Every closed-loop step against the oracle re-synchronised to the device's persisted state
    (bench.oracle_chains resync: rho and the scaled iterates after the previous solve loaded with
    ora_set_state): identical status and iterations, x and y within 1e-5 relative (BASELINE.json) --
    each step compared from the same starting point.  Returns the per-step parity records."""
    out = rec.replay(sum(b.B for _, b in rec.batches), persist=True)  # every QP of every bucket
    _, ref, own = bench.oracle_chains(out, settings, threads=4, resync=True)
    recs = []
    for t in range(steps):
        got = [e["got"][t] for e in out["buckets"]]
        p = bench.parity_vs_oracle(got, [r[t] for r in ref])
        recs.append(p)
        assert p["status_equal"] == p["qps"] and p["iter_equal"] == p["qps"], (t + 1, p)
        assert p["max_rel_x"] <= PRIMAL_RTOL and p["max_rel_y"] <= PRIMAL_RTOL, (t + 1, p)
        # the device's state before the step is the oracle's own after the same solve, up to rounding
        for bi, e in enumerate(out["buckets"]):
            worst, worst_rho = bench.state_diff(e["pst"][t], own[bi][t])
            assert worst <= 1e-6 and worst_rho <= 1e-6, (t + 1, bi, worst, worst_rho)
    assert out["per_step"][-1]["step"] == steps  # the loop moved: every step rebuilt the QPs
    return recs


def test_closed_loop_steps_match_the_oracle_chain(ctx):
    steps = 4
    settings, bks, batches, rec = _loop(ctx, 20, 8, 4, steps, 5005)
    try:
        _check_chain(rec, settings, steps)
    finally:
        rec.close()
        for _, b in batches:
            b.close()


@pytest.mark.parametrize("N,K,steps", [(40, 10, 12), (30, 8, 10)])
def test_long_horizon_closed_loop_every_step(ctx, N, K, steps):
    """Config 5's closed loop on the kernel the bench times: N = 40 (the chunked W = 39 instance) with
    K = 10 / 11 obstacle rows, osqp_update_A + _lin_cost + _bounds every step (resume mode 2 with the
    q snapshot), >= 10 steps; N = 30 the live horizon's W = 29 instance."""
    settings, bks, batches, rec = _loop(ctx, N, K, 2, steps, 5000 + N)
    try:
        assert all(b.stats()["var_slots"] == 3 for _, b in batches)  # the long-horizon shape
        _check_chain(rec, settings, steps)
    finally:
        rec.close()
        for _, b in batches:
            b.close()


def test_follow_plan_device_is_getpos_getvel_of_each_solution(ctx):
    """impc_batch_follow_plan_device against mpcPlanner::getPos / getVel (mpcPlanner.cpp:1257-1290)
    restated on the host, at t = ts (state 1) and t = 1.5 ts (interpolated); QPs without a solution
    keep their x0 and linearisation point."""
    settings, bks, batches, rec = _loop(ctx, 20, 8, 2, 1, 5006)
    try:
        rec.start()
        N = 20
        for e in rec.buckets:
            b, nb, ts = e["b"], e["nb"], e["ts"]
            x, _, info = b.get()
            for t in (ts, 1.5 * ts):
                e["pos"].set(e["pos0"])
                e["vel"].set(e["vel0"])
                e["lin"].set(e["lin0"])
                b.follow_plan_device(N, ts, t, e["pos"].ptr, e["vel"].ptr, e["lin"].ptr)
                ctx.synchronize()
                pos, vel, lin = e["pos"].get(), e["vel"].get(), e["lin"].get()
                idx = min(max(int(math.floor(t / ts)), 0), N - 1)
                nxt = min(idx + 1, N - 1)
                dt = t - idx * ts
                for i in range(nb):
                    s, en = x[i, 8 * idx: 8 * idx + 8], x[i, 8 * nxt: 8 * nxt + 8]
                    if int(info["status_val"][i]) in (1, 2, -2, -6):
                        # (the device may fuse the interpolation's multiply-add: ulp-level at t = 1.5 ts)
                        np.testing.assert_allclose(pos[i], s[:3] + (en[:3] - s[:3]) / ts * dt, rtol=1e-14, atol=1e-14)
                        np.testing.assert_allclose(vel[i], s[3:6] + (en[3:6] - s[3:6]) / ts * dt, rtol=1e-14, atol=1e-14)
                        np.testing.assert_array_equal(lin[i].reshape(-1), x[i, : 8 * N])
                    else:
                        np.testing.assert_array_equal(pos[i], e["pos0"][i])
                        np.testing.assert_array_equal(lin[i].reshape(-1), e["lin0"][i].reshape(-1))
    finally:
        rec.close()
        for _, b in batches:
            b.close()
