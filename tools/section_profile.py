#!/usr/bin/env python3
"""Per-section cycle breakdown of the structured kernel (profiling build, `make prof`).

usage: IMPC_SECTION_PROF=1 python tools/section_profile.py [instances [N [K [max_iter]]]]
Runs the bench workload (intent_config, N=20, K=8/9; or horizon N with K/K+1 obstacles) once and prints, per section, the time (100 MHz
s_memrealtime ticks -> ns) seen by lane 0 of each team, summed over QPs, normalised per QP and per
ADMM iteration.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python")]
os.environ.setdefault("IMPC_SECTION_PROF", "1")
import impc  # noqa: E402
from impc import scenarios  # noqa: E402

NAMES = ["setup", "factor", "warm", "rhs", "S1", "fwd", "S3", "bwd", "S5", "update", "products", "checks", "output",
         "f-assembly", "f-dense"]


def main():
    inst = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    kw = dict(N=N, K=int(sys.argv[3])) if len(sys.argv) > 3 else (dict(N=N) if N != 20 else {})
    mi = int(sys.argv[4]) if len(sys.argv) > 4 else 4000  # max_iter = 1: the setup's sections alone
    assert "prof" in os.path.basename(impc.LIB_PATH)
    impc.lib.impc_debug_sections.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    buckets = scenarios.intent_config(instances=inst, seed=3000, **kw)
    ctx = impc.Context(0)
    s = impc.default_settings(verbose=0, max_iter=mi)
    for K, bk in sorted(buckets.items()):
        pat, v = bk["pattern"], bk["values"]
        B = v["q"].shape[0]
        b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
        b.set_settings(s)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.warm_start(bk["x_ws"], None)
        b.set_profiling(True)
        b.solve()
        _, _, info = b.get()
        sec = (C.c_ulonglong * 16)()
        impc.lib.impc_debug_sections(b.h, sec)
        sec = np.array(sec[:], dtype=np.float64)
        iters = sec[15]
        tot = sec[:15].sum()
        tot_ns, per_ns = 10.0 * tot, 10.0 * sec
        print(f"K={K} B={B} kernel {b.timings()[1]:.1f} ms, mean iter {iters / B:.1f}, "
              f"us/QP {tot_ns / B / 1e3:.1f}, ns/iter {tot_ns / iters:.0f}")
        for i, nm in enumerate(NAMES):
            print(f"  {nm:9s} {100 * sec[i] / tot:5.1f}%  per-iter {per_ns[i] / iters:8.0f} ns  per-QP {per_ns[i] / B / 1e3:8.2f} us")
        b.close()
    ctx.close()


if __name__ == "__main__":
    main()
