"""makePlanWithPred's two branches in the batched replan, and the planner state carried between
replans on the device (impc_replan_run through impc.replan.DeviceReplan, include/impc_replan.h), against the
restatement oracle/replan_ref.py (mpcPlanner.cpp:571-661).

One mixed batch of instances: on a first plan with and without predictions, with predictions
(the fan-out), without predictions and with / without current dynamic obstacles.  Per replan and
instance: the branch taken; the fan-out's closest obstacle and candidate order; every assembled
QP bit for bit (restatement of solveTraj's assembly with the instance's own warm start and
linearisation point); every solution against the OSQP oracle (identical status and iterations,
1e-5); the selection, recomputed by the restatement on the GPU's solutions, bit for bit; the
committed plan (the chosen solution, bitwise) and firstTime_.  Three chained replans: the second
and third start from the state the device committed (x0 from the plan's next state, predictions
advanced one step), so first-plan instances move on to the fan-out.  Parity of the solutions
unpinned against the real libosqp."""
import numpy as np
import pytest

import impc
from impc import scenarios
from impc.replan import FANOUT, SINGLE_CURRENT, SINGLE_FIRST, DeviceReplan
from oracle import replan_ref as ref

from helpers import compare

I, K, N = 24, 3, 20


def _scenario(seed=4242):
    buckets = scenarios.intent_config(N=N, K=K, instances=I, hyps=6, seed=seed)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    return p, pd, inst, pred_size


def test_branch_table():
    """:606 -- fan-out only with predictions and not firstTime_; a first plan never keeps obstacles."""
    assert ref.branch(0, True) == ref.FANOUT
    assert ref.branch(1, True) == ref.SINGLE_FIRST
    assert ref.branch(1, False, 3) == ref.SINGLE_FIRST
    assert ref.branch(0, False, 0) == ref.SINGLE_FIRST
    assert ref.branch(0, False, 3) == ref.SINGLE_CURRENT
    from impc.replan import branches
    got = branches([0, 1, 1, 0, 0], [1, 1, 0, 0, 0], [0, 0, 3, 0, 3])
    np.testing.assert_array_equal(got, [FANOUT, SINGLE_FIRST, SINGLE_FIRST, SINGLE_FIRST, SINGLE_CURRENT])


def test_oracle_chain_first_plan_then_fanout():
    """CPU: the restatement's state machine -- a first-plan instance solves the obstacle-free QP,
    commits it, and fans out on the next replan (warm-started from that plan)."""
    p, pd, inst, pred_size = _scenario(seed=11)
    s = impc.default_settings(verbose=0)
    i = 0
    st = dict(first_time=1, plan_x=None)
    r1 = ref.make_plan_with_pred(pd, pd, s, st, inst["pos"][i], inst["vel"][i], inst["xref"][i], inst["obp"][i],
                                 inst["pred"][i], pred_size[i], inst["prob_all"][i], True)
    assert r1["branch"] == ref.SINGLE_FIRST and r1["valid"] and st["first_time"] == 0
    np.testing.assert_array_equal(st["plan_x"], r1["x"])
    r2 = ref.make_plan_with_pred(pd, pd, s, st, inst["pos"][i], inst["vel"][i], inst["xref"][i], inst["obp"][i],
                                 inst["pred"][i], pred_size[i], inst["prob_all"][i], True)
    assert r2["branch"] == ref.FANOUT and r2["valid"] and 0 <= r2["best"] < 6


def _row(out, k, r):
    """x, y, info and assembled values of row r of shape k (k obstacle rows per stage)."""
    sh = out["shapes"][k]
    return sh["x"][r], sh["y"][r], sh["info"][r], [v[r] for v in sh["vals"]]


def _solution_check(x, y, info, xo, yo, io, degenerate):
    """A QP's solution against the oracle's.  degenerate: the instance's state is an OSQP_NAN plan
    (2143289344.0 in every entry) that an earlier replan committed -- the reference does commit one
    when every candidate is infeasible or diverged, since solveProblem returns NoError for them
    (mpcPlanner.cpp:513-518, 629-639) -- so the QP is linearised and warm-started at 2e9 and only its
    status is compared (its iterates carry no precision)."""
    if degenerate:
        assert info["status_val"] == io["status_val"], (info, io)
    else:
        compare((x[None], y[None], info[None]), (xo[None], yo[None], io[None]))


def _check_replan(out, before, pos, vel, xref, dyn_cur, pred, pred_size, prob, has_pred, cur_size, cur_count, pd, s,
                  num_pred=None, static=None):
    """One replan against the restatement, instance by instance (num_pred [I]: each instance's
    obstacle count K_i, its first K_i slots; None = every slot).  static = (centroid [I][S][3],
    size [I][S][3], yaw [I][S]): every instance's static obstacles.  With a non-zero yaw the static
    rows go through the device cos / sin (a few ulp, include/impc_mpc.h): the assembled values are
    then compared within 1e-13 and each QP is solved by the oracle on the values the device
    assembled, everything else stays exact."""
    plan_x, first, _, _ = before
    I = len(out["branch"])
    Kall = pred.shape[1]
    kp = np.full(I, Kall) if num_pred is None else np.asarray(num_pred)
    stat = [[]] * I if static is None else [[(static[0][i][j], static[1][i][j], float(static[2][i][j]))
                                              for j in range(len(static[2][i]))] for i in range(I)]
    exact = static is None or not np.any(np.asarray(static[2]))
    for i in range(I):
        assert out["branch"][i] == ref.branch(first[i], bool(has_pred[i]) and kp[i] > 0, cur_count[i]), i
    expect = plan_x.copy()
    expect_first = first.copy()

    def check_qp(pat_vals, rows_vals, msg):
        """the assembled values against the restatement's; returns the values the oracle solves"""
        pat, vals = pat_vals
        for key, got in zip(("Px", "q", "Ax", "l", "u"), rows_vals):
            if exact:
                np.testing.assert_array_equal(got, vals[key], err_msg=f"{msg} {key}")
            else:
                fin = np.isfinite(vals[key])
                np.testing.assert_array_equal(np.isfinite(got), fin, err_msg=f"{msg} {key}")
                np.testing.assert_allclose(got[fin], vals[key][fin], rtol=1e-13, atol=1e-13, err_msg=f"{msg} {key}")
        return vals if exact else dict(zip(("Px", "q", "Ax", "l", "u"), rows_vals))

    for i in out["inst_fanout"]:
        Ki = int(kp[i])
        assert out["num_obs"][i] == Ki, i
        px = plan_x[i]
        fo, qps = ref.fanout_qps(pd, 0, px, pos[i], vel[i], xref[i], dyn_cur[i][:Ki], pred[i][:Ki],
                                 pred_size[i][:Ki], prob[i][:Ki], stat[i])
        assert out["ob_idx"][i] == fo["ob_idx"], i
        np.testing.assert_array_equal(out["cand_type"][i], fo["types"])
        xs, oks = [], []
        for c in range(6):
            k, r = out["cand_rows"][i][c]
            assert k == Ki + (1 if out["cand_slot"][i][c] >= 4 else 0)
            x, y, info, vals = _row(out, k, r)
            sv = check_qp(qps[c][:2], vals, f"instance {i} candidate {c}")
            xo, yo, io = ref.solve(qps[c][0], sv, qps[c][2], s)
            _solution_check(x, y, info, xo, yo, io, np.abs(px).max() >= 1e9)
            xs.append(x)
            oks.append(ref.solve_traj_ok(info))
        best = ref.select(pd, pd, 0, px, xref[i], fo, xs, oks, prob[i][fo["ob_idx"]], stat[i])
        assert out["best_cand"][i] == best, (i, out["best_cand"][i], best)
        if best >= 0:
            expect[i] = xs[best]
            expect_first[i] = 0
    for idx, br in ((out["inst_first"], SINGLE_FIRST), (out["inst_current"], SINGLE_CURRENT)):
        for i in idx:
            cur = br == SINGLE_CURRENT
            ci = int(cur_count[i]) if cur else 0
            pat, vals, ws = ref.single_qp(pd, first[i], plan_x[i], pos[i], vel[i], xref[i],
                                          dyn_cur[i][:ci] if cur else None, cur_size[i][:ci] if cur else None,
                                          stat[i])
            k, r = out["single_rows"][i]
            # the first plans' shape: K + 2 when the replan carries static obstacles (include/impc_replan.h)
            assert k == (Kall + 2 if static is not None and first[i] else ci), (i, k, ci)
            assert out["num_obs"][i] == ci, i
            x, y, info, got_vals = _row(out, k, r)
            sv = check_qp((pat, vals), got_vals, f"instance {i} single ({'current' if cur else 'first'})")
            xo, yo, io = ref.solve(pat, sv, ws, s)
            _solution_check(x, y, info, xo, yo, io, not first[i] and np.abs(plan_x[i]).max() >= 1e9)
            if ref.solve_traj_ok(info):
                expect[i] = x
                expect_first[i] = 0
    return expect, expect_first


@pytest.mark.gpu
def test_mixed_branches_three_chained_replans(ctx):
    p, pd, inst, pred_size = _scenario()
    s = impc.default_settings(verbose=0)
    L = inst["pred"].shape[3]
    idx = np.arange(I)
    first = (idx % 4 == 0).astype(np.int8)                   # first plans (half of them with predictions)
    has_pred = [idx % 3 != 1, idx % 5 != 2, idx % 7 != 3]    # per replan: obPredPos_ non-empty
    cur_count = np.where(idx % 2 == 0, K, 0)                  # current obstacles kept without predictions
    cur_size = np.broadcast_to(inst["size"], (I, K, 3)).copy()
    rp = DeviceReplan(ctx, p, pd, I, K, L, s)
    rp.set_state(inst["prev"], first)
    pos, vel, pred = inst["pos"].copy(), inst["vel"].copy(), inst["pred"].copy()
    seen = set()
    try:
        for step in range(3):
            before = rp.plans()
            dyn_cur = pred[:, :, 0, 0, :]                     # the obstacles' current positions
            out = rp.run(pos, vel, inst["xref"], dyn_cur=dyn_cur, pred_pos=pred, pred_size=pred_size,
                         prob=inst["prob_all"], has_pred=has_pred[step], cur_size=cur_size,
                         cur_count=cur_count)
            seen.update(int(b) for b in out["branch"])
            expect, expect_first = _check_replan(out, before, pos, vel, inst["xref"], dyn_cur, pred, pred_size,
                                                 inst["prob_all"], has_pred[step], cur_size, cur_count, pd, s)
            plan_x, ft, pc, valid = rp.plans()
            np.testing.assert_array_equal(plan_x, expect)       # the committed plans, bitwise
            np.testing.assert_array_equal(ft, expect_first)
            assert (pc[ft == 0] == N).all()
            # next replan: x0 = the plan's next state, predictions one step on
            pos = np.where(valid[:, None] == 1, plan_x[:, 8:11], pos)
            vel = np.where(valid[:, None] == 1, plan_x[:, 11:14], vel)
            pred = np.concatenate([pred[:, :, :, 1:], pred[:, :, :, -1:]], axis=3)
        assert seen == {FANOUT, SINGLE_FIRST, SINGLE_CURRENT}
        # every first-plan instance with a plan fanned out on a later replan with predictions
        assert (rp.plans()[1] == 0).all()
    finally:
        rp.close()


@pytest.mark.gpu
def test_per_instance_obstacle_counts_three_chained_replans(ctx):
    """Every instance with its own obstacle count per replan (K_i = predPos.size(), 0..K: the
    detector keeps the obstacles in range and view, fakeDetector.cpp:493 -> updatePredObstacles
    :343-373) and its own number of current obstacles without predictions (c_i, 0..K): the
    candidates of an instance have K_i and K_i + 1 obstacle rows, all shapes of the replan in one
    grouped launch.  Three chained replans against the restatement, instance by instance."""
    Kmax = 5
    buckets = scenarios.intent_config(N=N, K=Kmax, instances=I, hyps=6, seed=4343)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    s = impc.default_settings(verbose=0)
    L = inst["pred"].shape[3]
    idx = np.arange(I)
    rng = np.random.default_rng(43)
    first = (idx % 6 == 0).astype(np.int8)
    num_pred = [rng.integers(0, Kmax + 1, I) for _ in range(3)]          # K_i per replan, 0 = none
    cur_count = rng.integers(0, Kmax + 1, I).astype(np.int32)
    cur_size = np.broadcast_to(inst["size"], (I, Kmax, 3)).copy()
    rp = DeviceReplan(ctx, p, pd, I, Kmax, L, s)
    rp.set_state(inst["prev"], first)
    pos, vel, pred = inst["pos"].copy(), inst["vel"].copy(), inst["pred"].copy()
    shapes_seen = set()
    try:
        for step in range(3):
            before = rp.plans()
            dyn_cur = pred[:, :, 0, 0, :]
            out = rp.run(pos, vel, inst["xref"], dyn_cur=dyn_cur, pred_pos=pred, pred_size=pred_size,
                         prob=inst["prob_all"], num_pred=num_pred[step], cur_size=cur_size, cur_count=cur_count)
            shapes_seen.update(out["shapes"])
            expect, expect_first = _check_replan(out, before, pos, vel, inst["xref"], dyn_cur, pred, pred_size,
                                                 inst["prob_all"], np.ones(I, bool), cur_size, cur_count, pd, s,
                                                 num_pred=num_pred[step])
            plan_x, ft, pc, valid = rp.plans()
            np.testing.assert_array_equal(plan_x, expect)
            np.testing.assert_array_equal(ft, expect_first)
            pos = np.where(valid[:, None] == 1, plan_x[:, 8:11], pos)
            vel = np.where(valid[:, None] == 1, plan_x[:, 11:14], vel)
            pred = np.concatenate([pred[:, :, :, 1:], pred[:, :, :, -1:]], axis=3)
        assert len(shapes_seen) >= Kmax  # most obstacle counts 0 .. K + 1 took part
    finally:
        rp.close()


def _statics(inst, S, seed, yaw):
    """S static obstacles per instance (staticObstacle: centroid, size, yaw) beside each instance's
    reference path, so that their rows bind: centroids 0.6-1.2 m off the reference at steps spread
    over the horizon, sizes 0.4-1.0 m, yaw 0 or in [-pi, pi)."""
    rng = np.random.default_rng(seed)
    xr = inst["xref"]
    nI = xr.shape[0]
    steps = np.linspace(N // 4, N - 2, S).astype(int)
    cen = xr[:, steps, :3] + rng.uniform(0.6, 1.2, (nI, S, 3)) * rng.choice([-1.0, 1.0], (nI, S, 3)) * [1, 1, 0.2]
    size = rng.uniform(0.4, 1.0, (nI, S, 3))
    yw = rng.uniform(-np.pi, np.pi, (nI, S)) if yaw else np.zeros((nI, S))
    return cen, size, yw


def test_oracle_static_obstacles_enter_every_solve_but_a_first_plan():
    """CPU: the restatement's static obstacles (makePlanWithPred :593-602) -- a first plan's QP has
    no obstacle rows, a later single solve and every candidate carry S static rows per stage (with
    the dynamic ones before them), and the selection scores them."""
    p, pd, inst, pred_size = _scenario(seed=12)
    S = 2
    cen, size, yw = _statics(inst, S, 7, True)
    i = 1
    stat = [(cen[i][j], size[i][j], float(yw[i][j])) for j in range(S)]
    base = ref.single_qp(pd, 1, None, inst["pos"][i], inst["vel"][i], inst["xref"][i])[0]["m"]
    pat0 = ref.single_qp(pd, 1, None, inst["pos"][i], inst["vel"][i], inst["xref"][i], static_obs=stat)[0]
    assert pat0["m"] == base
    px = np.zeros(13 * N - 5)
    px[: 8 * N] = inst["prev"][i].reshape(-1)
    pat1 = ref.single_qp(pd, 0, px, inst["pos"][i], inst["vel"][i], inst["xref"][i], static_obs=stat)[0]
    assert pat1["m"] == base + S * (N - 1)
    s = impc.default_settings(verbose=0)
    x_st = ref.solve(*ref.single_qp(pd, 0, px, inst["pos"][i], inst["vel"][i], inst["xref"][i], static_obs=stat), s)[0]
    x_free = ref.solve(*ref.single_qp(pd, 0, px, inst["pos"][i], inst["vel"][i], inst["xref"][i]), s)[0]
    assert np.abs(x_st - x_free).max() > 1e-2  # the statics placed by _statics bind
    fo, qps = ref.fanout_qps(pd, 0, px, inst["pos"][i], inst["vel"][i], inst["xref"][i], inst["obp"][i],
                             inst["pred"][i], pred_size[i], inst["prob_all"][i], stat)
    for c, (pat, _, _) in enumerate(qps):
        assert pat["m"] == base + (len(fo["cands"][c][0]) + S) * (N - 1)
    st = dict(first_time=0, plan_x=px)
    r = ref.make_plan_with_pred(pd, pd, s, st, inst["pos"][i], inst["vel"][i], inst["xref"][i], inst["obp"][i],
                                inst["pred"][i], pred_size[i], inst["prob_all"][i], True, static_obs=stat)
    assert r["branch"] == ref.FANOUT


@pytest.mark.gpu
@pytest.mark.parametrize("yaw", [False, True], ids=["yaw0", "yaw"])
def test_static_obstacles_three_chained_replans(ctx, yaw):
    """impc_replan_config.num_static: every instance's static obstacles in each solveTraj not on a
    first plan and in getTrajectoryScore (obclustering_->getStaticObstacles(), mpcPlanner.cpp:594,
    615, 620, 652), with the isDyamic index quirk (:1194) reaching the candidates whose dynamic
    obstacles precede them; first plans in their own shape without obstacle rows.  Mixed branches
    and obstacle counts, three chained replans against the restatement, instance by instance."""
    Kmax, S = 4, 3
    buckets = scenarios.intent_config(N=N, K=Kmax, instances=I, hyps=6, seed=4646)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    s = impc.default_settings(verbose=0)
    L = inst["pred"].shape[3]
    idx = np.arange(I)
    rng = np.random.default_rng(46)
    first = (idx % 5 == 0).astype(np.int8)
    num_pred = [rng.integers(0, Kmax + 1, I) for _ in range(3)]
    cur_count = rng.integers(0, Kmax + 1, I).astype(np.int32)
    cur_size = np.broadcast_to(inst["size"], (I, Kmax, 3)).copy()
    static = _statics(inst, S, 47, yaw)
    rp = DeviceReplan(ctx, p, pd, I, Kmax, L, s, num_static=S)
    rp.set_state(inst["prev"], first)
    pos, vel, pred = inst["pos"].copy(), inst["vel"].copy(), inst["pred"].copy()
    seen, shapes_seen = set(), set()
    try:
        for step in range(3):
            before = rp.plans()
            dyn_cur = pred[:, :, 0, 0, :]
            out = rp.run(pos, vel, inst["xref"], dyn_cur=dyn_cur, pred_pos=pred, pred_size=pred_size,
                         prob=inst["prob_all"], num_pred=num_pred[step], cur_size=cur_size, cur_count=cur_count,
                         static=static)
            seen.update(int(b) for b in out["branch"])
            shapes_seen.update(out["shapes"])
            for k, sh in out["shapes"].items():  # S static rows per stage on every shape but the first plans'
                m = sh["y"].shape[1] if hasattr(sh["y"], "shape") else None
                dyn = 0 if k == Kmax + 2 else k
                stat = 0 if k == Kmax + 2 else S
                assert m == impc.mpc_dims(p, stat, dyn)[1], (k, m)
            expect, expect_first = _check_replan(out, before, pos, vel, inst["xref"], dyn_cur, pred, pred_size,
                                                 inst["prob_all"], np.ones(I, bool), cur_size, cur_count, pd, s,
                                                 num_pred=num_pred[step], static=static)
            plan_x, ft, pc, valid = rp.plans()
            np.testing.assert_array_equal(plan_x, expect)
            np.testing.assert_array_equal(ft, expect_first)
            pos = np.where(valid[:, None] == 1, plan_x[:, 8:11], pos)
            vel = np.where(valid[:, None] == 1, plan_x[:, 11:14], vel)
            pred = np.concatenate([pred[:, :, :, 1:], pred[:, :, :, -1:]], axis=3)
        assert seen == {FANOUT, SINGLE_FIRST, SINGLE_CURRENT}
        assert Kmax + 2 in shapes_seen and 0 in shapes_seen
    finally:
        rp.close()
