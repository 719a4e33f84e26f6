#!/usr/bin/env python3
"""Per-config throughput on one MI355X for BASELINE.json's configs (bench.py measures configs[2]).

  config 1  one N=20, K=0 QP, cold (latency of a single solve through the batch API)
  config 2  4096 identical N=20 QPs with 10 static-obstacle rows
  config 4  this GPU's share of 262,144 mixed-K QPs (K ~ U{0..20}): 32,768 QPs, one batch per K
  config 5  this GPU's share of 65,536 N=40, K=10 QPs: 8,192, warm-started (previous-plan rollout)

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
            "launch": "grouped" if grouped else "per batch"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    ctx = impc.Context(0)
    s = impc.default_settings(verbose=0)
    print(json.dumps(run(ctx, "1: single N=20 K=0 QP (cold)", [scenarios.first_call_config(batch=1, seed=1)],
                         max(args.steps, 20), s)), flush=True)
    print(json.dumps(run(ctx, "2: 4096 identical N=20 K=10 static", [scenarios.static_config(batch=4096, seed=2000)],
                         args.steps, s)), flush=True)
    rng = np.random.default_rng(4000)
    ks = rng.integers(0, 21, 32768)
    cfg4 = []
    for K in range(21):
        cnt = int((ks == K).sum())
        if cnt == 0:
            continue
        if K == 0:
            cfg4.append(scenarios.first_call_config(batch=cnt, seed=4100))
        else:
            b = scenarios.intent_config(N=20, K=K, instances=cnt // 6 + 1, hyps=8, seed=4200 + K)
            bk = b[K]
            take = min(cnt, bk["values"]["q"].shape[0])
            cfg4.append(dict(pattern=bk["pattern"], values={k: v[:take] for k, v in bk["values"].items()},
                             x_ws=bk["x_ws"][:take]))
    print(json.dumps(run(ctx, "4: 32768 of 262144 mixed K in 0..20 (this GPU's share)", cfg4, args.steps, s)),
          flush=True)
    b5 = scenarios.intent_config(N=40, K=10, instances=1024, hyps=8, seed=5000)
    print(json.dumps(run(ctx, "5: 8192 of 65536 N=40 K=10(+1) warm-started (this GPU's share)", list(b5.values()),
                         args.steps, s)), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
