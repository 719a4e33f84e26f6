#!/usr/bin/env python3
"""Throughput of the device obstacle predictor (impc_predict_traj + impc_intent_prob) on one GPU:
`--count` tracked obstacles in the test world of tests/test_predict.py (0.1 m voxels, walls and a
pillar), predictor_param.yaml parameters, 24-entry histories.  One JSON line."""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python"), os.path.join(ROOT, "tests")]
import impc  # noqa: E402
from test_predict import TP, track, world  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--count", type=int, default=4096)
    a = ap.parse_args()
    ctx = impc.Context(0)
    m, occ = world()
    tp = impc.TrajParams(num_pred=TP["num_pred"], dt=TP["dt"], stop_velocity=TP["stop_vel"],
                         front_angle_deg=TP["front_angle_deg"], min_turning_time=TP["min_turning_time"],
                         max_turning_time=TP["max_turning_time"], z_score=TP["z_score"])
    om = impc.OccMap()
    om.origin[:] = m["origin"]
    om.resolution = m["res"]
    om.dims[:] = m["dims"]
    rng = np.random.default_rng(5)
    n = a.count
    pos = np.stack([rng.uniform(-6, 4, n), rng.uniform(-6, 6, n), np.full(n, 1.0)], axis=1)
    hd = rng.uniform(-math.pi, math.pi, n)
    sp = rng.uniform(0.3, 2.0, n)
    vel = np.stack([sp * np.cos(hd), sp * np.sin(hd), np.zeros(n)], axis=1)
    size = np.tile([0.5, 0.5, 1.0], (n, 1))
    impc.predict_traj(ctx, tp, om, occ.reshape(-1), pos[:64], vel[:64], size[:64])  # warm-up
    t = time.perf_counter()
    pp, ps = impc.predict_traj(ctx, tp, om, occ.reshape(-1), pos, vel, size)
    t_traj = time.perf_counter() - t
    H = 24
    ph, vh = np.zeros((n, H, 3)), np.zeros((n, H, 3))
    for o in range(min(n, 256)):
        p_, v_ = track(hd[o], sp[o], H)
        ph[o], vh[o] = p_, v_
    ph[256:], vh[256:] = ph[:1], vh[:1]
    ip = impc.intent_params()
    impc.intent_prob(ctx, ip, ph[:64], vh[:64], np.full(64, H, np.int32))
    t = time.perf_counter()
    impc.intent_prob(ctx, ip, ph, vh, np.full(n, H, np.int32))
    t_prob = time.perf_counter() - t
    print(json.dumps({"obstacles": n, "predict_traj_s_incl_transfers": t_traj, "obstacles_per_s_traj": n / t_traj,
                      "intent_prob_s_incl_transfers": t_prob, "num_pred": TP["num_pred"], "history": H}))
    ctx.close()


if __name__ == "__main__":
    main()
