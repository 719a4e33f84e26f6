"""The batched makePlanWithPred from a compiled C++ program through the C-ABI alone
(tests/native/replan_example.cpp: one impc_replan_run per replan, impc_replan_advance_device for
the next x0), three chained mixed-branch replans checked against the restatement
oracle/replan_ref.py (mpcPlanner.cpp:571-661) exactly as tests/test_replan_branches.py checks the
Python mirror: the branch of every instance, the fan-out's closest obstacle and candidate order,
every assembled QP bit for bit, every solution against the OSQP oracle (identical status and
iterations, 1e-5), the selection bit for bit, the committed plan and firstTime_.  Between replans
the program moves each instance to its plan's next state on the device (getPos / getVel(dt),
mpc_node.cpp:216-224) and the predictions one step on.  Parity of the solutions is unpinned
against the real libosqp."""
import os
import subprocess

import numpy as np
import pytest

import impc
from impc import scenarios
from impc.replan import FANOUT, SINGLE_CURRENT, SINGLE_FIRST, assemble

from test_replan_branches import I, K, N, _check_replan, _scenario, _statics

EXE = os.path.join(os.path.dirname(__file__), "native", "build", "replan_example")


def _read(raw, off, dtype, count):
    a = np.frombuffer(raw, dtype, count=count, offset=off)
    return a, off + a.nbytes


def parse(raw, R, K, S=0):
    n = 13 * N - 5
    outs, off = [], 0
    for _ in range(R):
        o = {}
        o["branch"], off = _read(raw, off, np.int8, I)
        o["best_cand"], off = _read(raw, off, np.int32, I)
        o["ob_idx"], off = _read(raw, off, np.int32, I)
        ct, off = _read(raw, off, np.int32, 6 * I)
        cs, off = _read(raw, off, np.int32, 6 * I)
        o["cand_type"], o["cand_slot"] = ct.reshape(I, 6), cs.reshape(I, 6)
        px, off = _read(raw, off, np.float64, I * n)
        o["plan_x"] = px.reshape(I, n)
        o["first_time"], off = _read(raw, off, np.int8, I)
        o["prev_count"], off = _read(raw, off, np.int32, I)
        o["valid"], off = _read(raw, off, np.int8, I)
        o["num_obs"], off = _read(raw, off, np.int32, I)
        sr, off = _read(raw, off, np.int32, 6 * I)
        o["slot_row"] = sr.reshape(I, 6)
        o["shape"], off = _read(raw, off, np.int32, I)
        shapes = {}
        for k in range(K + 2 + (1 if S else 0)):
            cnt, off = _read(raw, off, np.int64, 1)
            cnt = int(cnt[0])
            if not cnt:
                continue
            sh = {}
            sh["row_inst"], off = _read(raw, off, np.int32, cnt)
            sh["row_code"], off = _read(raw, off, np.int8, cnt)
            dims, off = _read(raw, off, np.int64, 4)
            qn, qm, nnzP, nnzA = (int(d) for d in dims)
            x, off = _read(raw, off, np.float64, cnt * qn)
            y, off = _read(raw, off, np.float64, cnt * qm)
            info, off = _read(raw, off, impc.INFO_DTYPE, cnt)
            sh["x"], sh["y"], sh["info"] = x.reshape(cnt, qn), y.reshape(cnt, qm), info
            vals = []
            for ln in (nnzP, qn, nnzA, qm, qm):
                v, off = _read(raw, off, np.float64, cnt * ln)
                vals.append(v.reshape(cnt, ln))
            sh["vals"] = vals
            shapes[k] = sh
        o["shapes"] = shapes
        o.update(assemble(o, shapes))
        outs.append(o)
    assert off == len(raw), (off, len(raw))
    return outs


def _run(tmp_path, p, s, inst, pred_size, first, has_pred, cur_count, cur_size, num_pred=None, static=None):
    R, K, L = has_pred.shape[0], inst["pred"].shape[1], inst["pred"].shape[3]
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(fin, "wb") as f:
        S = 0 if static is None else static[2].shape[1]
        f.write(np.array([I, K, L, N, R, 0 if num_pred is None else 1, S], np.int32).tobytes())
        f.write(bytes(p))
        f.write(bytes(s))
        for a, dt in ((inst["pos"], np.float64), (inst["vel"], np.float64), (inst["xref"], np.float64),
                      (inst["prev"], np.float64), (first, np.int8), (inst["pred"], np.float64),
                      (pred_size, np.float64), (inst["prob_all"], np.float64), (cur_size, np.float64),
                      (cur_count, np.int32), (has_pred, np.int8)):
            f.write(np.ascontiguousarray(a, dt).tobytes())
        if num_pred is not None:
            f.write(np.ascontiguousarray(num_pred, np.int32).tobytes())
        if S:
            for a in static:
                f.write(np.ascontiguousarray(a, np.float64).tobytes())
    r = subprocess.run([EXE, str(fin), str(fout)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return parse(open(fout, "rb").read(), R, K, S), r.stdout.strip()


def _replay(outs, pd, s, inst, pred_size, first, has_pred, cur_count, cur_size, num_pred=None, static=None):
    """The host replays the chain the program ran: start state, x0 / predictions after each replan."""
    plan_x = np.zeros((I, 13 * N - 5))
    plan_x[:, : 8 * N] = inst["prev"].reshape(I, -1)
    ft = first.copy()
    pos, vel, pred = inst["pos"].copy(), inst["vel"].copy(), inst["pred"].copy()
    seen = set()
    for step, out in enumerate(outs):
        dyn_cur = pred[:, :, 0, 0, :]
        before = (plan_x, ft, None, None)
        expect, expect_first = _check_replan(out, before, pos, vel, inst["xref"], dyn_cur, pred, pred_size,
                                             inst["prob_all"], has_pred[step], cur_size, cur_count, pd, s,
                                             num_pred=None if num_pred is None else num_pred[step], static=static)
        np.testing.assert_array_equal(out["plan_x"], expect)
        np.testing.assert_array_equal(out["first_time"], expect_first)
        np.testing.assert_array_equal(out["prev_count"], np.where(expect_first == 0, N, 0))
        seen.update(int(b) for b in out["branch"])
        plan_x, ft = out["plan_x"].copy(), out["first_time"].copy()
        pos = np.where(out["valid"][:, None] == 1, plan_x[:, 8:11], pos)
        vel = np.where(out["valid"][:, None] == 1, plan_x[:, 11:14], vel)
        pred = np.concatenate([pred[:, :, :, 1:], pred[:, :, :, -1:]], axis=3)
    return seen, ft


@pytest.mark.gpu
def test_cpp_three_chained_replans_match_restatement(tmp_path):
    p, pd, inst, pred_size = _scenario()  # the Python mirror test's scenario (seed 4242)
    s = impc.default_settings(verbose=0)
    idx = np.arange(I)
    first = (idx % 4 == 0).astype(np.int8)
    has_pred = np.array([idx % 3 != 1, idx % 5 != 2, idx % 7 != 3], np.int8)
    cur_count = np.where(idx % 2 == 0, K, 0).astype(np.int32)
    cur_size = np.broadcast_to(inst["size"], (I, K, 3)).copy()
    outs, msg = _run(tmp_path, p, s, inst, pred_size, first, has_pred, cur_count, cur_size)
    seen, ft = _replay(outs, pd, s, inst, pred_size, first, has_pred, cur_count, cur_size)
    assert seen == {FANOUT, SINGLE_FIRST, SINGLE_CURRENT}
    assert (ft == 0).all()
    print(msg)


@pytest.mark.gpu
def test_cpp_per_instance_obstacle_counts(tmp_path):
    """The same program with every instance's obstacle count varying 0..12 per replan (K_i =
    predPos.size(), mpcPlanner.cpp:343-373) and its current obstacles 0..12: shapes of 0..13
    obstacle rows in one grouped launch per replan, checked instance by instance."""
    Kmax = 12
    buckets = scenarios.intent_config(N=N, K=Kmax, instances=I, hyps=6, seed=4545)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    s = impc.default_settings(verbose=0)
    rng = np.random.default_rng(45)
    idx = np.arange(I)
    first = (idx % 5 == 0).astype(np.int8)
    has_pred = np.ones((3, I), np.int8)
    num_pred = rng.integers(0, Kmax + 1, (3, I)).astype(np.int32)
    cur_count = rng.integers(0, Kmax + 1, I).astype(np.int32)
    cur_size = np.broadcast_to(inst["size"], (I, Kmax, 3)).copy()
    outs, msg = _run(tmp_path, p, s, inst, pred_size, first, has_pred, cur_count, cur_size, num_pred)
    seen, _ = _replay(outs, pd, s, inst, pred_size, first, has_pred, cur_count, cur_size, num_pred)
    assert seen == {FANOUT, SINGLE_FIRST, SINGLE_CURRENT}
    assert len(set().union(*[o["shapes"] for o in outs])) >= 10
    print(msg)


@pytest.mark.gpu
def test_cpp_static_obstacles(tmp_path):
    """The same program with every instance's static obstacles (impc_replan_config.num_static = 3,
    random yaw; obclustering_->getStaticObstacles(), mpcPlanner.cpp:594) and obstacle counts 0..6:
    the statics enter every QP but the first plans' (shape K + 2) and the selection, checked
    instance by instance against the restatement."""
    Kmax, S = 6, 3
    buckets = scenarios.intent_config(N=N, K=Kmax, instances=I, hyps=6, seed=4747)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    s = impc.default_settings(verbose=0)
    rng = np.random.default_rng(48)
    idx = np.arange(I)
    first = (idx % 4 == 1).astype(np.int8)
    has_pred = np.ones((3, I), np.int8)
    num_pred = rng.integers(0, Kmax + 1, (3, I)).astype(np.int32)
    cur_count = rng.integers(0, Kmax + 1, I).astype(np.int32)
    cur_size = np.broadcast_to(inst["size"], (I, Kmax, 3)).copy()
    static = _statics(inst, S, 49, True)
    outs, msg = _run(tmp_path, p, s, inst, pred_size, first, has_pred, cur_count, cur_size, num_pred, static)
    seen, _ = _replay(outs, pd, s, inst, pred_size, first, has_pred, cur_count, cur_size, num_pred, static)
    assert seen == {FANOUT, SINGLE_FIRST, SINGLE_CURRENT}
    assert Kmax + 2 in outs[0]["shapes"]
    print(msg)
