#!/usr/bin/env python3
"""Whole-replan throughput on one GPU: makePlanWithPred for I planning instances with every stage
on the device (impc.replan.DeviceReplan: fan-out -> build -> grouped solve -> select), the
config 3 workload (K = 8 dynamic obstacles, 6 candidates per instance, N = 20).  Prints one
JSON line with the stage times of the last of `--reps` runs."""
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
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    I, K, N = a.instances, 8, 20
    buckets = scenarios.intent_config(N=N, K=K, instances=I, hyps=6, seed=3000)
    inst = next(iter(buckets.values()))["instances"]
    p, pd = impc.mpc_params(horizon=N)
    L = inst["pred"].shape[3]
    ctx = impc.Context(0)
    rp = DeviceReplan(ctx, p, pd, I, K, L, impc.default_settings(verbose=0))
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    t = {}
    for _ in range(a.reps):
        t0 = time.perf_counter()
        # a replan after the first: the previous plan drives findClosestObstacle and the scores
        out = rp.run(inst["pos"], inst["vel"], inst["xref"], inst["prev"], np.zeros(I, np.int8),
                     np.full(I, N, np.int32), inst["obp"], inst["pred"], pred_size, inst["prob_all"], timings=t)
        t["total_s"] = time.perf_counter() - t0
    qps = 6 * I
    print(json.dumps({"instances": I, "candidate_qps": qps, "device_stages_s": t["fanout_build_solve_s"],
                      "replans_per_s_device": I / t["fanout_build_solve_s"],
                      "qp_solves_per_s_incl_fanout_build": qps / t["fanout_build_solve_s"],
                      "upload_s": t["upload_s"], "select_device_s": t["select_s"], "total_s": t["total_s"],
                      "mean_iter": float(np.concatenate([out["info_single"]["iter"], out["info_pair"]["iter"]]).mean()),
                      "picked_histogram": np.bincount(out["best_cand"][out["best_cand"] >= 0], minlength=6).tolist()}))
    rp.close()
    ctx.close()


if __name__ == "__main__":
    main()
