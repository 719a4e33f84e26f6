"""A whole makePlanWithPred replan on the device (impc.replan.DeviceReplan): intent fan-out ->
on-device QP assembly of both candidate shapes -> one grouped solve -> candidate selection,
against the host-built path of the same scenario (scenarios.intent_config, hypotheses 0-5 =
getIntentComb's candidates, first-call closest obstacle).  Every stage must agree bit for bit:
the candidate order, the assembled QP values, the solutions and the selected candidate."""
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
        out = rp.run(inst["pos"], inst["vel"], inst["xref"], inst["prev"], np.ones(I, np.int8),
                     np.full(I, N, np.int32), inst["obp"], inst["pred"], pred_size, inst["prob_all"])
    finally:
        rp.close()
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
        ref = impc.select_best(ctx, params, d["x_ptrs"], np.ones((I, 6), np.int8), np.ones(I, np.int8), d["prev"],
                               np.full(I, N, np.int32), d["xref"], np.zeros((I, 0, 3)), np.zeros((I, 0, 3)),
                               d["dyn_count"], d["dyn_pos"], d["dyn_size"], d["prob"])
    finally:
        for b in batches.values():
            b.close()
    np.testing.assert_array_equal(out["best_cand"], ref["best_cand"])
