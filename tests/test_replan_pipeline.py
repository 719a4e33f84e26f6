"""A whole makePlanWithPred replan on the device (impc.replan.DeviceReplan): intent fan-out ->
on-device QP assembly of both candidate shapes -> one grouped solve -> candidate selection,
against the host-built path of the same scenario (scenarios.intent_config, hypotheses 0-5 =
getIntentComb's candidates, the distance-based closest obstacle).  Every stage must agree bit for
bit: the candidate order, the assembled QP values, the solutions and the selected candidate.

Every instance here is on the fan-out branch (not firstTime_, predictions present); its previous
plan holds a single state (prev_count = 1), so findClosestObstacle takes its distance fallback
(mpcPlanner.cpp:676-685) -- the scenario's closest obstacle -- while the QPs are linearised at and
warm-started from the scenario's whole previous plan.  The branch selection itself is
tests/test_replan_branches.py."""
import numpy as np
import pytest

import impc
from impc import scenarios
from impc.replan import DeviceReplan

from helpers import gpu

pytestmark = pytest.mark.gpu


def test_device_replan_matches_host_path(ctx):
    I, K, N = 40, 5, 20
    buckets = scenarios.intent_config(N=N, K=K, instances=I, hyps=6, seed=707)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    L = inst["pred"].shape[3]
    s = impc.default_settings(verbose=0)
    rp = DeviceReplan(ctx, p, pd, I, K, L, s)
    try:
        pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
        out = rp.run(inst["pos"], inst["vel"], inst["xref"], inst["prev"], np.zeros(I, np.int8),
                     np.ones(I, np.int32), inst["obp"], inst["pred"], pred_size, inst["prob_all"])
    finally:
        rp.close()
    assert (out["branch"] == 0).all()
    assert np.array_equal(out["ob_idx"], inst["closest"])
    for nm, kk in (("single", K), ("pair", K + 1)):
        bk = buckets[kk]
        v = bk["values"]
        for got, key in zip(out["vals_" + nm], ("Px", "q", "Ax", "l", "u")):
            np.testing.assert_array_equal(got, v[key], err_msg=f"{nm} {key}")
        x, y, info = gpu(ctx, bk, s)
        np.testing.assert_array_equal(out["x_" + nm], x)
        np.testing.assert_array_equal(out["info_" + nm]["iter"], info["iter"])
    # the host path's selection over the same solutions
    batches = {}
    for kk, bk in buckets.items():
        pat, v = bk["pattern"], bk["values"]
        b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], v["q"].shape[0])
        b.set_settings(s)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.warm_start(bk["x_ws"], None)
        b.solve()
        b.get()
        batches[kk] = b
    try:
        d = scenarios.selection_arrays(buckets, {kk: b.device_results()[0] for kk, b in batches.items()})
        params = dict(horizon=N, num_candidates=6, max_dynamic=d["kmax"], pred_len=d["L"], num_static=0, prev_len=N,
                      dynamic_safety_dist=pd["dynamic_safety_dist"], static_safety_dist=pd["static_safety_dist"])
        ref = impc.select_best(ctx, params, d["x_ptrs"], np.ones((I, 6), np.int8), np.zeros(I, np.int8), d["prev"],
                               np.ones(I, np.int32), d["xref"], np.zeros((I, 0, 3)), np.zeros((I, 0, 3)),
                               d["dyn_count"], d["dyn_pos"], d["dyn_size"], d["prob"])
    finally:
        for b in batches.values():
            b.close()
    np.testing.assert_array_equal(out["best_cand"], ref["best_cand"])


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
            out = rp.run(pos, inst["vel"], dev, inst["prev"], np.zeros(I, np.int8), np.ones(I, np.int32),
                         inst["obp"], inst["pred"], pred_size, inst["prob_all"])
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


def test_cpp_replan_example_matches_python_replan(ctx, tmp_path):
    """tests/native/replan_example.cpp -- the batched makePlanWithPred a C++ planner would write
    over the C-ABI alone (fan-out, per-candidate copies, assembly, grouped solve, selection) --
    gives bit for bit the selection and solutions of impc.replan.DeviceReplan on one scenario."""
    import ctypes as C
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "native", "build", "replan_example")
    I, K, N = 32, 4, 20
    buckets = scenarios.intent_config(N=N, K=K, instances=I, hyps=6, seed=709)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    L = inst["pred"].shape[3]
    s = impc.default_settings(verbose=0)
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    first = np.zeros(I, np.int8)
    pcount = np.ones(I, np.int32)
    rp = DeviceReplan(ctx, p, pd, I, K, L, s)
    try:
        out = rp.run(inst["pos"], inst["vel"], inst["xref"], inst["prev"], first, pcount, inst["obp"], inst["pred"],
                     pred_size, inst["prob_all"])
    finally:
        rp.close()
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(fin, "wb") as f:
        f.write(np.array([I, K, L, N, inst["prev"].shape[1]], np.int32).tobytes())
        f.write(bytes(p))
        f.write(bytes(s))
        f.write(np.array([pd["dynamic_safety_dist"], pd["static_safety_dist"]]).tobytes())
        for a, dt in ((inst["pos"], np.float64), (inst["vel"], np.float64), (inst["xref"], np.float64),
                      (inst["prev"], np.float64), (first, np.int8), (pcount, np.int32), (inst["obp"], np.float64),
                      (inst["pred"], np.float64), (pred_size, np.float64), (inst["prob_all"], np.float64)):
            f.write(np.ascontiguousarray(a, dt).tobytes())
    r = subprocess.run([exe, str(fin), str(fout)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(fout, "rb").read()
    best = np.frombuffer(raw[: 4 * I], np.int32)
    np.testing.assert_array_equal(best, out["best_cand"])
    off = 4 * I
    for nm, cnt, kk in (("single", 4, K), ("pair", 2, K + 1)):
        n = buckets[kk]["pattern"]["n"]
        x = np.frombuffer(raw[off: off + 8 * cnt * I * n], np.float64).reshape(cnt * I, n)
        off += 8 * cnt * I * n
        it = np.frombuffer(raw[off: off + 8 * cnt * I], np.int64)
        off += 8 * cnt * I
        np.testing.assert_array_equal(x, out["x_" + nm])
        np.testing.assert_array_equal(it, out["info_" + nm]["iter"])
    assert off == len(raw)
