#!/usr/bin/env python3
"""What one QP's setup costs against its ADMM iterations on the structured kernel: the per-QP
device latency (impc_batch_get_qp_latency: dequeue -> results written) of a full batch of
mpcPlanner QPs solved with max_iter = 1, 26, 51, 101, 201, fitted as latency = S + t * iterations
(S: load + Ruiz scaling + rho + factorisation + output, t: one ADMM iteration with its share of the
termination checks).  Then the persistent workspace's resumes: osqp_update_lin_cost (scaling
replayed, refactorisation) and osqp_update_A (data scaled afresh, refactorisation), each with
max_iter = 1.  Usage: python tools/setup_cost.py [N [K [instances [scaling]]]] (scaling: OSQP's
Ruiz pass count, default 10; 0 isolates the passes' cost); prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python")]
import impc  # noqa: E402
from impc import scenarios  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    inst = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    scl = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    bk = scenarios.intent_config(N=N, K=K, instances=inst, seed=3000)[K]
    pat, v = bk["pattern"], bk["values"]
    B = v["q"].shape[0]
    ctx = impc.Context(0)
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    b.set_profiling(True)
    pts = []
    for mi in (1, 26, 51, 101, 201):
        b.set_settings(impc.default_settings(verbose=0, max_iter=mi, scaling=scl))
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.warm_start(bk["x_ws"], None)
        lat = []
        for _ in range(2):
            b.solve()
            _, _, info = b.get()
            lat.append(b.qp_latency().mean())
        pts.append((float(info["iter"].mean()), min(lat), b.timings()[1]))
    it = np.array([p[0] for p in pts])
    la = np.array([p[1] for p in pts])
    t, S = np.polyfit(it, la, 1)
    # persistent resumes
    b.set_settings(impc.default_settings(verbose=0, max_iter=1, scaling=scl))
    b.set_persistent(True)
    b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
    b.warm_start(bk["x_ws"], None)
    b.solve()
    b.get()
    full = b.qp_latency().mean()
    b.update_lin_cost(v["q"] * 1.001)
    b.solve()
    b.get()
    res1 = b.qp_latency().mean()
    b.update_matrices(None, v["Ax"])
    b.solve()
    b.get()
    res2 = b.qp_latency().mean()
    print(json.dumps({
        "workload": f"intent_config N={N} K={K}, {B} QPs, warm-started, scaling={scl}, per-QP device latency (ms)",
        "points": [{"mean_iter": p[0], "mean_latency_ms": p[1], "launch_ms": p[2]} for p in pts],
        "fit": {"setup_ms": S, "per_iter_us": 1e3 * t},
        "persistent_max_iter_1": {"first_solve_ms": full, "resume_update_lin_cost_ms": res1,
                                  "resume_update_A_ms": res2},
        "build_id": impc.lib.impc_build_id().decode(),
    }))
    b.close()
    ctx.close()


if __name__ == "__main__":
    main()
