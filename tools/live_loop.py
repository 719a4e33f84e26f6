#!/usr/bin/env python3
"""The live replan loop's rate on one GPU: I planning instances flying the reference's benchmark
path (ref_trajectory_dynus_benchmark.txt) at the live horizon N = 30 with K dynamic obstacles each,
R chained replans as mpcNavigation::mpcCB runs them -- per replan getXRef on the device
(impc_reference_traj_device), ONE impc_replan_run (makePlanWithPred for every instance) and the
vehicle following its plan for 0.1 s (impc_replan_advance_device).  Every replan's predictions are
resident on the device before the timed loop (the predictor's output, scenarios.live_loop); each
replan is timed from its first call to the end of its device work.  Prints one JSON line.
The same loop at small I is checked replan by replan against the restatements in
tests/test_live_loop.py."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python")]
import impc  # noqa: E402
from impc import scenarios  # noqa: E402
from impc.replan import DeviceReplan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--instances", type=int, default=8192)
    ap.add_argument("--obstacles", type=int, default=4)
    ap.add_argument("--replans", type=int, default=30)
    ap.add_argument("--horizon", type=int, default=30)
    a = ap.parse_args()
    I, K, R, N = a.instances, a.obstacles, a.replans, a.horizon
    t0 = time.time()
    sc = scenarios.live_loop(I, K, R, N=N, seed=4100)
    gen_s = time.time() - t0
    p, pd, L = sc["params"], sc["pd"], sc["L"]
    ctx = impc.Context(0)
    rp = DeviceReplan(ctx, p, pd, I, K, L, impc.default_settings(verbose=0))
    paths = impc.ReferencePaths(ctx, list(sc["paths"]), pd["ts"], N)
    D = impc.DeviceArray
    pos_d, vel_d, xref_d = D(ctx, sc["pos0"]), D(ctx, sc["vel0"]), D(ctx, (I, N, 8))
    psize_d, prob_d = D(ctx, sc["pred_size"]), D(ctx, np.ascontiguousarray(sc["prob"]))
    pred_d, cur_d = D(ctx, np.ascontiguousarray(sc["pred_pos"])), D(ctx, np.ascontiguousarray(sc["dyn_cur"]))
    step_pred, step_cur = pred_d.nbytes // R, cur_d.nbytes // R
    walls, stats = [], []
    for r in range(R):
        ctx.synchronize()
        t = time.perf_counter()
        paths.xref_device(pos_d.ptr, xref_d.ptr)
        rp.run_device(pos_d.ptr, vel_d.ptr, xref_d.ptr, cur_d.ptr + r * step_cur, pred_d.ptr + r * step_pred,
                      psize_d.ptr, prob_d.ptr)
        rp.advance_device(pd["ts"], pos_d.ptr, vel_d.ptr)
        ctx.synchronize()
        walls.append(time.perf_counter() - t)
        st = rp.stats()
        stats.append((st["fanout"], st["single_first"], st["single_current"]))
    last = rp.results(values=False)
    its = np.concatenate([last["info_" + nm]["iter"] for nm in ("single", "pair") if last["info_" + nm] is not None])
    sts = np.concatenate([last["info_" + nm]["status_val"] for nm in ("single", "pair")
                          if last["info_" + nm] is not None])
    valid = rp.plans()[3]
    w = np.array(walls)
    fan = w[1:]  # replans 1..R-1: every instance on the fan-out branch (6 candidates)
    print(json.dumps({
        "workload": f"live loop: {I} instances on ref_trajectory_dynus_benchmark.txt, N={N}, K={K} dynamic "
                    f"obstacles, {R} chained replans (getXRef + makePlanWithPred + follow plan 0.1 s per replan)",
        "instances": I, "replans": R, "first_replan_s": float(w[0]), "fanout_replan_s": fan.tolist(),
        "fanout_replan_s_median": float(np.median(fan)), "replans_per_s": float(I / np.median(fan)),
        "qp_solves_per_s": float(6 * I / np.median(fan)), "branches": stats[-1],
        "last_replan": {"mean_iter": float(its.mean()), "p50_iter": float(np.median(its)), "max_iter": int(its.max()),
                        "status_counts": {str(int(k)): int(v) for k, v in zip(*np.unique(sts, return_counts=True))},
                        "valid_plans": int(valid.sum())},
        "ref_start_idx_mean": float(paths.last_idx().mean()), "gen_s": gen_s,
        "build_id": impc.lib.impc_build_id().decode()}))
    for d in (pos_d, vel_d, xref_d, psize_d, prob_d, pred_d, cur_d):
        d.free()
    paths.close()
    rp.close()
    ctx.close()


if __name__ == "__main__":
    main()
