"""The replan's wall-clock budget (makePlanWithPred, mpcPlanner.cpp:609-628): the 0.15 s candidate
issue cut-off, timeLimit = max(solverTimeLimit_ - time, solverTimeLimit_) on every candidate, and
the selection over the candidates whose solveTraj succeeded (every OSQP status but NON_CVX,
:513-518)."""
import time

import numpy as np
import pytest

import impc
from impc import scenarios
from impc.replan import ISSUE_CUTOFF_S, DeviceReplan, candidate_valid


def test_candidate_valid_maps_slots_to_batch_rows():
    # two instances; slot < 4 -> single-intent row 4i+slot, else two-intent row 2i+slot-4
    slot = np.array([[0, 1, 2, 3, 4, 5], [4, 0, 5, 1, 2, 3]])
    st_single = np.array([1, 1, 1, impc.NON_CVX, 1, impc.TIME_LIMIT_REACHED, 1, 1])
    st_pair = np.array([1, impc.NON_CVX, impc.NON_CVX, 1])
    got = candidate_valid(slot, st_single, st_pair)
    np.testing.assert_array_equal(got, [[1, 1, 1, 0, 1, 0], [0, 1, 1, 1, 1, 1]])
    assert got.dtype == np.int8
    assert ISSUE_CUTOFF_S == 0.15


def _scenario(I=16, K=3, N=20, seed=811):
    buckets = scenarios.intent_config(N=N, K=K, instances=I, hyps=6, seed=seed)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    L = inst["pred"].shape[3]
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    args = (inst["pos"], inst["vel"], inst["xref"], inst["prev"], np.ones(I, np.int8), np.full(I, N, np.int32),
            inst["obp"], inst["pred"], pred_size, inst["prob_all"])
    return p, pd, I, K, L, args


@pytest.mark.gpu
def test_budget_time_limit_and_cutoff(ctx):
    p, pd, I, K, L, args = _scenario()
    rp = DeviceReplan(ctx, p, pd, I, K, L, impc.default_settings(verbose=0))
    try:
        free = rp.run(*args)
        # solverTimeLimit_ = 0.05 s (mpcPlanner.cpp:167), measured on the device clock from each
        # QP's dequeue: a QP that finishes inside it is bit-identical to the unlimited replan; one
        # that reaches it (a slow or shared box) stops early with OSQP_TIME_LIMIT_REACHED
        lim = rp.run(*args, solver_time_limit=0.05)
        assert lim["issued"] and lim["time_limit"] == 0.05
        hit_any = False
        for nm in ("single", "pair"):
            hit = lim["info_" + nm]["status_val"] == impc.TIME_LIMIT_REACHED
            hit_any |= bool(hit.any())
            ok = ~hit
            np.testing.assert_array_equal(lim["x_" + nm][ok], free["x_" + nm][ok])
            np.testing.assert_array_equal(lim["info_" + nm]["iter"][ok], free["info_" + nm]["iter"][ok])
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
