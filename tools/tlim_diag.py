"""Diagnosis of round 2's replan time-limit failure: runs the round-2 budget
scenario (16 instances x 6 candidates, K = 3/4, first_time = 1, solver_time_limit = 0.05 s) with
the library of the tree given as argv[1] (this tree, or the round-2 tree built into _r02tree/) and
prints, per limited QP, status / iterations / the unlimited run's iterations, and the host wall
time of the limited replan.  Usage: python tools/tlim_diag.py <tree-root> [label]"""
import json
import os
import sys
import time

import numpy as np

root = os.path.abspath(sys.argv[1])
label = sys.argv[2] if len(sys.argv) > 2 else root
sys.path.insert(0, os.path.join(root, "intent-mpc_amd", "python"))
import impc  # noqa: E402
from impc import scenarios  # noqa: E402
from impc.replan import DeviceReplan  # noqa: E402

I, K, N = 16, 3, 20
buckets = scenarios.intent_config(N=N, K=K, instances=I, hyps=6, seed=811)
inst = next(iter(buckets.values()))["instances"]
p, pd = impc.mpc_params(horizon=N)
L = inst["pred"].shape[3]
pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
args = (inst["pos"], inst["vel"], inst["xref"], inst["prev"], np.ones(I, np.int8), np.full(I, N, np.int32),
        inst["obp"], inst["pred"], pred_size, inst["prob_all"])
ctx = impc.Context(0)
out = dict(tree=label)
if hasattr(ctx, "clock_rate"):
    out["clock_hz"] = ctx.clock_rate()
    out["clock_check_0.02s"] = ctx.clock_check(0.02)
    out["clock_check_0.1s"] = ctx.clock_check(0.1)
rp = DeviceReplan(ctx, p, pd, I, K, L, impc.default_settings(verbose=0))
free = rp.run(*args)
for rep in range(3):
    prof = "profile" in DeviceReplan.run.__code__.co_varnames  # this tree: per-QP device latency
    t = time.perf_counter()
    lim = rp.run(*args, solver_time_limit=0.05, **(dict(profile=True) if prof else {}))
    host = time.perf_counter() - t
    r = dict(rep=rep, host_replan_s=round(host, 4), time_limit=lim["time_limit"])
    if prof:
        lat = np.concatenate([lim["lat_single"], lim["lat_pair"]])
        r["device_qp_latency_ms"] = dict(p50=round(float(np.median(lat)), 3), max=round(float(lat.max()), 3))
    for nm in ("single", "pair"):
        st, it = lim["info_" + nm]["status_val"], lim["info_" + nm]["iter"]
        fit = free["info_" + nm]["iter"]
        diff = ~np.all(lim["x_" + nm] == free["x_" + nm], axis=1)
        hit = st == impc.TIME_LIMIT_REACHED
        r[nm] = dict(qps=int(st.size), differ=int(diff.sum()), time_limit_status=int(hit.sum()),
                     iters_limited=it[hit][:12].tolist(), iters_free_of_those=fit[hit][:12].tolist(),
                     differ_without_limit_status=int((diff & ~hit).sum()))
    print(json.dumps(r), flush=True)
rp.close()
ctx.close()
print(json.dumps(out), flush=True)
