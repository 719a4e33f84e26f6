#!/usr/bin/env python3
"""Iteration counts of the batched solve against the reference-path spacing.

The synthetic reference of SURVEY.md 8d advances 0.5-2.5 m per 0.1 s step (5-25 m/s, the live
benchmark path's raw 2.5 m point spacing), mostly beyond vmax = 5 m/s, so the QPs track a
reference they cannot reach.  This sweep fixes the spacing per run and reports the mean / p50
ADMM iterations (identical to the oracle's, tests/test_gpu_parity.py) for the first-call shape
(config 1: K = 0, cold) and the intent shape (config 3: K = 8 dynamic obstacles, warm-started).
Runs on the GPU through the C-ABI (one batch per point)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python")]
import impc  # noqa: E402
from impc import scenarios  # noqa: E402


def solve(ctx, cfg, s):
    pat, v = cfg["pattern"], cfg["values"]
    B = v["q"].shape[0]
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    b.set_settings(s)
    b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
    if cfg.get("x_ws") is not None:
        b.warm_start(cfg["x_ws"], None)
    b.solve()
    info = b.get()[2]
    b.close()
    return info


def main():
    ctx = impc.Context(0)
    s = impc.default_settings(verbose=0)
    for step in (0.1, 0.2, 0.3, 0.5, 1.0, 1.5, 2.0, 2.5, (0.5, 2.5)):
        rng = step if isinstance(step, tuple) else (step, step)
        i1 = solve(ctx, scenarios.first_call_config(batch=512, seed=11, step_range=rng), s)
        b3 = scenarios.intent_config(N=20, K=8, instances=256, hyps=8, seed=12, step_range=rng)
        i3 = np.concatenate([solve(ctx, bk, s) for bk in b3.values()])
        print(json.dumps({"step_m_per_0.1s": rng, "speed_m_s": [10 * rng[0], 10 * rng[1]],
                          "config1_K0_cold": {"mean_iter": float(i1["iter"].mean()),
                                              "p50_iter": float(np.median(i1["iter"]))},
                          "config3_K8_warm": {"mean_iter": float(i3["iter"].mean()),
                                              "p50_iter": float(np.median(i3["iter"])),
                                              "solved": float(np.mean(i3["status_val"] == 1))}}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
