#!/usr/bin/env python3
"""Throughput of the min-snap path QPs (polyTrajSolver, impc/minsnap.py) on one GPU: `--paths`
random paths of `--waypoints` points, live poly_traj parameters (degree 7, snap, C3), OSQP
defaults; the x/y/z QPs of all paths are one generic-kernel batch.  Times the setUpProblem solve
and an updateProblem solve (new start velocities, bounds only, workspace kept) with the values
resident on the device (kernel events), beside the OSQP restatement on one host core for a
sample.  One JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python"), os.path.join(ROOT, "tests")]
import impc  # noqa: E402
from impc import minsnap  # noqa: E402
from oracle import osqp_oracle as ora  # noqa: E402
from test_minsnap import paths  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--paths", type=int, default=16384)
    ap.add_argument("--waypoints", type=int, default=6)
    ap.add_argument("--cpu-sample", type=int, default=192)
    a = ap.parse_args()
    nb, W = a.paths, a.waypoints
    ctx = impc.Context(0)
    p = minsnap.params()
    s = impc.default_settings(verbose=0)
    path = paths(nb, W, seed=77)
    iv2 = np.random.default_rng(78).normal(scale=0.5, size=(nb, 3))
    ms = minsnap.MinsnapBatch(ctx, p, nb, W, s)
    ms.batch.set_profiling(True)
    ms.update_path(path)
    ms.solve()
    t1 = ms.batch.timings()
    _, _, info2 = ms.solve(init_vel=iv2)
    t2 = ms.batch.timings()
    ms.close()
    B = 3 * nb
    # CPU: the same QPs, setup + solve per QP on one core (the reference's per-axis solver)
    v = minsnap.values(p, path[: (a.cpu_sample + 2) // 3])
    pat = minsnap.pattern(p, W)
    k = min(a.cpu_sample, v["q"].shape[0])
    t = time.perf_counter()
    ora.solve_batch(pat, v["Px"][:k], v["q"][:k], v["Ax"][:k], v["l"][:k], v["u"][:k], ora.settings_from(s))
    cpu = k / (time.perf_counter() - t)
    ms1 = t1[0] + t1[1]
    print(json.dumps({
        "paths": nb, "waypoints": W, "qps": B, "n": pat["n"], "m": pat["m"],
        "setup_solve_ms": ms1, "qp_solves_per_s_setup": B / (ms1 * 1e-3),
        "update_solve_ms": t2[1], "qp_solves_per_s_update": B / (t2[1] * 1e-3),
        "mean_iter_update": float(np.mean(info2["iter"])),
        "cpu_port_qp_per_s_1core": cpu, "cpu_sample": k, "kernel": "generic"}))
    ctx.close()


if __name__ == "__main__":
    main()
