"""A whole makePlanWithPred replan on the device (impc_replan_run through impc.replan.DeviceReplan):
intent fan-out -> on-device QP assembly of both candidate shapes -> one grouped solve -> candidate
selection, against the host-array entry points of the same library stages on the same scenario
(impc.intent_fanout, the host C++ builder impc.mpc_values, separate solves, impc.select_best).
Every stage must agree bit for bit: the closest obstacle and candidate order, the assembled QP
values, the solutions and the selected candidate.

Every instance here is on the fan-out branch (not firstTime_, predictions present) with a full
previous plan (currentStatesSol_.size() = N, the only size a planner past its first plan holds),
so findClosestObstacle takes its direction-weighted score (mpcPlanner.cpp:687-707).  The branch
selection itself is tests/test_replan_branches.py."""
import numpy as np
import pytest

import impc
from impc import scenarios
from impc.replan import DeviceReplan, candidate_valid

pytestmark = pytest.mark.gpu


def test_device_replan_matches_host_path(ctx):
    I, K, N = 40, 5, 20
    buckets = scenarios.intent_config(N=N, K=K, instances=I, hyps=6, seed=707)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    L = inst["pred"].shape[3]
    s = impc.default_settings(verbose=0)
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    zeros = np.zeros(I, np.int8)
    rp = DeviceReplan(ctx, p, pd, I, K, L, s)
    try:
        out = rp.run(inst["pos"], inst["vel"], inst["xref"], inst["prev"], zeros, None, inst["obp"], inst["pred"],
                     pred_size, inst["prob_all"])
    finally:
        rp.close()
    assert (out["branch"] == 0).all()
    fo = impc.intent_fanout(ctx, inst["pos"], zeros, inst["prev"], np.full(I, N, np.int32), inst["obp"],
                            inst["pred"], pred_size, inst["prob_all"])
    np.testing.assert_array_equal(out["ob_idx"], fo["ob_idx"])
    np.testing.assert_array_equal(out["cand_type"], fo["cand_type"])
    np.testing.assert_array_equal(out["cand_slot"], fo["cand_slot"])
    n = 13 * N - 5
    ws = np.zeros((I, n))
    ws[:, : 8 * N] = inst["prev"].reshape(I, -1)
    batches = {}
    try:
        for nm, rep, kk, dp, dsz in (("single", 4, K, "single_pos", "single_size"), ("pair", 2, K + 1, "pair_pos",
                                                                                     "pair_size")):
            rows = np.repeat(np.arange(I), rep)
            host = impc.mpc_values(p, inst["pos"][rows], inst["vel"][rows], inst["xref"][rows], inst["prev"][rows],
                                   dyn_pos=fo[dp].reshape(rep * I, kk, L, 3), dyn_size=fo[dsz].reshape(rep * I, kk, L, 3))
            for got, key in zip(out["vals_" + nm], ("Px", "q", "Ax", "l", "u")):
                np.testing.assert_array_equal(got, host[key], err_msg=f"{nm} {key}")
            pat = impc.mpc_pattern(p, 0, kk)
            b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], rep * I)
            b.set_settings(s)
            b.set_values(host["Px"], host["q"], host["Ax"], host["l"], host["u"])
            b.warm_start(ws[rows], None)
            b.solve()
            x, _, info = b.get()
            np.testing.assert_array_equal(out["x_" + nm], x)
            np.testing.assert_array_equal(out["info_" + nm]["iter"], info["iter"])
            batches[nm] = (b, info)
        # the host entry point of the selection over the same solutions
        xs = {nm: batches[nm][0].device_results()[0] for nm in batches}
        slot = fo["cand_slot"]
        ptrs = np.zeros((I, 6), np.uint64)
        dyn_count = np.zeros((I, 6), np.int32)
        dyn_pos = np.zeros((I, 6, K + 1, L, 3))
        dyn_size = np.zeros((I, 6, K + 1, L, 3))
        for i in range(I):
            for c in range(6):
                sl = int(slot[i, c])
                if sl < 4:
                    ptrs[i, c] = xs["single"] + 8 * n * (4 * i + sl)
                    dyn_count[i, c] = K
                    dyn_pos[i, c, :K], dyn_size[i, c, :K] = fo["single_pos"][i, sl], fo["single_size"][i, sl]
                else:
                    ptrs[i, c] = xs["pair"] + 8 * n * (2 * i + sl - 4)
                    dyn_count[i, c] = K + 1
                    dyn_pos[i, c], dyn_size[i, c] = fo["pair_pos"][i, sl - 4], fo["pair_size"][i, sl - 4]
        valid = candidate_valid(slot, batches["single"][1], batches["pair"][1])
        params = dict(horizon=N, num_candidates=6, max_dynamic=K + 1, pred_len=L, num_static=0, prev_len=N,
                      dynamic_safety_dist=pd["dynamic_safety_dist"], static_safety_dist=pd["static_safety_dist"])
        ref = impc.select_best(ctx, params, ptrs.reshape(-1), valid, zeros, inst["prev"], np.full(I, N, np.int32),
                               inst["xref"], np.zeros((I, 0, 3)), np.zeros((I, 0, 3)), dyn_count, dyn_pos, dyn_size,
                               fo["closest_prob"])
    finally:
        for b, _ in batches.values():
            b.close()
    np.testing.assert_array_equal(out["best_cand"], ref["best_cand"])
    assert (out["valid"] == (ref["best_cand"] >= 0)).all()


def test_device_replan_from_paths(ctx):
    """The replan's reference from the instances' input paths on the device (getReferenceTraj /
    getXRef, impc.ReferencePaths) over two replans: the references equal the restatement's
    (oracle/reftraj_ref.py, stateful lastRefStartIdx_) and the assembled gradients q equal the host
    builder's with those references."""
    from oracle.reftraj_ref import ReferencePath
    I, K, N = 24, 3, 20
    buckets = scenarios.intent_config(N=N, K=K, instances=I, hyps=6, seed=708)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    L = inst["pred"].shape[3]
    rng = np.random.default_rng(5)
    paths = []
    for i in range(I):
        d = inst["xref"][i, 1, :3] - inst["xref"][i, 0, :3]
        start = inst["pos"][i] - 5 * d
        paths.append(start + d * np.arange(3 * N + int(rng.integers(0, 20)))[:, None])
    refs = [ReferencePath(pth, pd["ts"], N) for pth in paths]
    dev = impc.ReferencePaths(ctx, paths, pd["ts"], N)
    rp = DeviceReplan(ctx, p, pd, I, K, L, impc.default_settings(verbose=0))
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    try:
        pos = inst["pos"].copy()
        for step in range(2):
            out = rp.run(pos, inst["vel"], dev, inst["prev"], np.zeros(I, np.int8), None, inst["obp"], inst["pred"],
                         pred_size, inst["prob_all"])
            exp = np.array([r.xref(pos[i]) for i, r in enumerate(refs)])
            assert np.array_equal(out["xref"], exp), step
            rows = np.repeat(np.arange(I), 4)
            host = impc.mpc_values(p, pos[rows], inst["vel"][rows], exp[rows], inst["prev"][rows],
                                   dyn_pos=np.zeros((4 * I, K, L, 3)), dyn_size=np.ones((4 * I, K, L, 3)))
            np.testing.assert_array_equal(out["vals_single"][1], host["q"])
            pos = pos + 0.5 * inst["vel"]
    finally:
        rp.close()
        dev.close()
