#!/usr/bin/env python3
"""Small-batch latency on one MI355X (the drop-in / single-planner regime): wall time per solve
step for one cold N=20 QP (config 1) and for the candidate QPs of I planning instances x 6 intent
hypotheses (K = 8 / 9 obstacles, warm-started), through tools/bench_configs.run.  Run once per
library variant (IMPC_LIB_VARIANT) to compare kernel shapes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python"), os.path.join(ROOT, "tools")]
import impc  # noqa: E402
from impc import scenarios  # noqa: E402
from bench_configs import run  # noqa: E402


def main():
    ctx = impc.Context(0)
    s = impc.default_settings(verbose=0)
    var = os.environ.get("IMPC_LIB_VARIANT", "base")
    r = run(ctx, "1: single N=20 K=0 QP (cold)", [scenarios.first_call_config(batch=1, seed=1)], 30, s)
    print(json.dumps(dict(variant=var, **r)), flush=True)
    for inst in (1, 8, 64, 512):
        b = scenarios.intent_config(N=20, K=8, instances=inst, hyps=6, seed=900 + inst)
        r = run(ctx, f"replan: {inst} instance(s) x 6 candidates, K=8/9", list(b.values()), 20 if inst < 64 else 5, s)
        print(json.dumps(dict(variant=var, **r)), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
