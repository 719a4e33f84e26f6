#!/usr/bin/env python3
"""Per-config throughput on one MI355X for BASELINE.json's configs (bench.py measures configs[2]).

  config 1  one N=20, K=0 QP, cold (latency of a single solve through the batch API)
  config 2  4096 identical N=20 QPs with 10 static-obstacle rows
  config 4  this GPU's share of 262,144 mixed-K QPs (K ~ U{0..20}): rank 0 of the 8-way Sigma m
            shard plan (bench.py --workload config4 runs the whole job), one grouped launch
  config 5  this GPU's share of 65,536 N=40, K=10 QPs: 8,192, warm-started (previous-plan rollout),
            cold (full setup per step) and as a receding window on persistent workspaces (each
            step: osqp_update_lin_cost with the shifted xRef + osqp_update_bounds with the next x0,
            then the solve resumes from the kept scaling, rho and iterates)

Prints one JSON line per config (QP-solves/s over `--steps` timed steps after one warm-up, kernel
chosen, mean iterations).  Synthetic data (impc.scenarios), inputs resident on the device.
"""
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


QUEUE = "longest"  # work-queue order of the launches (impc_batch_set_queue_order), --queue


def run(ctx, name, cfgs, steps, settings):
    batches = []
    for cfg in cfgs:
        pat, v = cfg["pattern"], cfg["values"]
        B = v["q"].shape[0]
        b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
        b.set_settings(settings)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        if cfg.get("x_ws") is not None:
            b.warm_start(cfg["x_ws"], None)
        if QUEUE == "longest":
            b.set_queue_order(impc.QUEUE_LONGEST_FIRST, scenarios.queue_weight(cfg["params"], cfg["N"]))
        batches.append(b)
    total = sum(b.B for b in batches)

    shapes = {b.stats()["kernel"] for b in batches}
    grouped = len(batches) > 1 and shapes == {impc.KERNEL_STRUCTURED} and len({b.n > 256 for b in batches}) == 1

    def step():
        if grouped:  # one persistent launch over all pattern buckets
            impc.solve_group(batches)
            return
        for b in batches:
            b.setup()
            b.solve()

    step()
    ctx.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.synchronize()
    el = time.perf_counter() - t
    iters = np.concatenate([b.get()[2]["iter"] for b in batches])
    kernels = sorted({"structured" if b.stats()["kernel"] == impc.KERNEL_STRUCTURED else "generic" for b in batches})
    for b in batches:
        b.close()
    return {"config": name, "qps": total, "steps": steps, "ms_per_step": 1000 * el / steps,
            "qp_solves_per_s": total * steps / el, "mean_iter": float(iters.mean()), "kernels": kernels,
            "launch": "grouped" if grouped else "per batch", "queue": QUEUE}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--queue", choices=("longest", "fifo"), default="longest")
    args = ap.parse_args()
    global QUEUE
    QUEUE = args.queue
    ctx = impc.Context(0)
    s = impc.default_settings(verbose=0)
    print(json.dumps(run(ctx, "1: single N=20 K=0 QP (cold)", [scenarios.first_call_config(batch=1, seed=1)],
                         max(args.steps, 20), s)), flush=True)
    print(json.dumps(run(ctx, "2: 4096 identical N=20 K=10 static", [scenarios.static_config(batch=4096, seed=2000)],
                         args.steps, s)), flush=True)
    from impc import distributed as D
    Kinst, w = scenarios.config4_plan(total_qps=262144)
    bounds = D.shard_plan(w, 8)
    cfg4 = scenarios.config4_rank(int(bounds[0]), int(bounds[1]), Kinst)
    print(json.dumps(run(ctx, "4: rank 0 of 262144 mixed K in 0..20, 8-way Sigma m shard", cfg4, args.steps, s)),
          flush=True)
    b5 = scenarios.intent_config(N=40, K=10, instances=1024, hyps=8, seed=5000)
    print(json.dumps(run(ctx, "5: 8192 of 65536 N=40 K=10(+1) warm-started, full setup per step (this GPU's share)",
                         list(b5.values()), args.steps, s)), flush=True)
    print(json.dumps(receding(ctx, list(b5.values()), args.steps, s)), flush=True)
    ctx.close()


def receding(ctx, bks, steps, settings):
    """Config 5 as a receding window: persistent workspaces, each step updates q (shifted xRef)
    and l, u (next x0) and resumes the solve (scaling, rho and iterates kept; impc_qp.h
    impc_batch_set_persistent).  Timed: the host -> device updates plus the grouped launch."""
    ups = []
    for sh in range(1, steps + 2):
        ups.append([scenarios.receding_update(bk, shift=sh) for bk in bks])
    batches = []
    for bk in bks:
        pat, v = bk["pattern"], bk["values"]
        B = v["q"].shape[0]
        b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
        b.set_settings(settings)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.warm_start(bk["x_ws"], None)
        b.set_persistent(True)
        if QUEUE == "longest":
            b.set_queue_order(impc.QUEUE_LONGEST_FIRST, scenarios.queue_weight(bk["params"], bk["N"]))
        batches.append(b)
    total = sum(b.B for b in batches)
    impc.solve_group(batches)  # setup + first solve (t = 0)
    ctx.synchronize()
    it0 = np.concatenate([b.get()[2]["iter"] for b in batches])

    def step(u):
        for b, v in zip(batches, u):
            b.update_lin_cost(v["q"])
            b.update_bounds(v["l"], v["u"])
        impc.solve_group(batches)

    step(ups[0])  # warm-up replan
    ctx.synchronize()
    t = time.perf_counter()
    for k in range(steps):
        step(ups[k + 1])
    ctx.synchronize()
    el = time.perf_counter() - t
    iters = np.concatenate([b.get()[2]["iter"] for b in batches])
    for b in batches:
        b.close()
    return {"config": "5: 8192 of 65536 N=40 K=10(+1) receding window, persistent workspaces (update q, l, u; "
                      "scaling replayed from the kept factors, rho and iterates kept)", "qps": total, "steps": steps, "ms_per_step": 1000 * el / steps,
            "qp_solves_per_s": total * steps / el, "mean_iter": float(iters.mean()),
            "mean_iter_first_solve": float(it0.mean()), "kernels": ["structured"], "launch": "grouped", "queue": QUEUE}


if __name__ == "__main__":
    main()
