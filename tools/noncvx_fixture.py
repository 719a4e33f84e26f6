#!/usr/bin/env python3
"""The NON_CVX candidates traced at scale (tools/trace_noncvx.py on MI355X) against the oracle and
the CPU emulation of the structured kernel, and the committed fixture tests/golden/noncvx_live.npz
(the first --keep QPs: inputs, warm start, the device's status / iterations, the oracle's).
Usage: python tools/noncvx_fixture.py [gpurun_out/r06/noncvx.npz] [--keep 8]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python"), os.path.join(ROOT, "tests")]
import impc  # noqa: E402
from oracle import osqp_oracle as ora  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump", nargs="?", default=os.path.join(ROOT, "gpurun_out", "r06", "noncvx.npz"))
    ap.add_argument("--keep", type=int, default=8)
    ap.add_argument("--codes", default="0,4", help="candidate slots kept in the fixture (0-3 one intent, 4-5 two)")
    ap.add_argument("--groups", type=int, default=3, help="distinct (replan, instance) groups kept")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "noncvx_live.npz"))
    a = ap.parse_args()
    d = np.load(a.dump)
    N = int(d["N"])
    p, _ = impc.mpc_params(horizon=N)
    s = impc.default_settings(verbose=0)
    so = ora.settings_from(s)
    rows, keep = [], {}
    codes = {int(c) for c in a.codes.split(",")}
    groups = []
    seen = {}
    for j in range(d["inst"].shape[0]):
        K = int(d["K"][j])
        idx = seen.get(K, 0)
        seen[K] = idx + 1
        pat = impc.mpc_pattern(p, 0, K)
        v = {key: d[f"{key}_K{K}"][idx] for key in ("Px", "q", "Ax", "l", "u")}
        xo, yo, io = ora.solve_batch(pat, v["Px"][None], v["q"][None], v["Ax"][None], v["l"][None], v["u"][None], so,
                                     x_ws=d["x_ws"][j][None])
        r = dict(replan=int(d["replan"][j]), inst=int(d["inst"][j]), code=int(d["code"][j]), K=K,
                 device=dict(status=int(d["status"][j]), iter=int(d["iter"][j]), setup=int(d["setup_exitflag"][j]),
                             pri_res=float(d["pri_res"][j]), dua_res=float(d["dua_res"][j])),
                 oracle=dict(status=int(io["status_val"][0]), iter=int(io["iter"][0]), setup=int(io["setup_exitflag"][0]),
                             pri_res=float(io["pri_res"][0]), dua_res=float(io["dua_res"][0]),
                             rho_updates=int(io["rho_updates"][0])))
        rows.append(r)
        grp = (r["replan"], r["inst"])
        if grp not in groups and len(groups) < a.groups:
            groups.append(grp)
        if len(keep.get("inst", [])) < a.keep and grp in groups and r["code"] in codes:
            for key, val in (("K", K), ("replan", r["replan"]), ("inst", r["inst"]), ("code", r["code"]),
                             ("status", r["device"]["status"]), ("iter", r["device"]["iter"]),
                             ("oracle_status", r["oracle"]["status"]), ("oracle_iter", r["oracle"]["iter"])):
                keep.setdefault(key, []).append(val)
            for key in ("Px", "q", "Ax", "l", "u"):
                keep.setdefault(f"{key}_{len(keep['inst']) - 1}", v[key])
            keep.setdefault(f"x_ws_{len(keep['inst']) - 1}", d["x_ws"][j])
    agree = sum(r["device"]["status"] == r["oracle"]["status"] and r["device"]["iter"] == r["oracle"]["iter"] for r in rows)
    print(json.dumps({"qps": len(rows), "status_and_iter_equal_oracle": agree, "rows": rows}, indent=1))
    if keep:
        np.savez_compressed(a.out, N=N, **{k: np.asarray(v) for k, v in keep.items()})
        print("wrote", a.out)


if __name__ == "__main__":
    main()
