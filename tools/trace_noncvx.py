#!/usr/bin/env python3
"""Trace the NON_CVX candidates of the live loop at scale: the loop of
tools/live_loop.py (I vehicles on the reference's benchmark path, N = 30, K obstacles), and after
every replan each QP that ended with status NON_CVX -- its assembled values (device builder), its
warm start (the instance's plan before the replan; zeros on a first plan) and the device's info
record -- saved to an .npz (tools/noncvx_fixture.py turns it into tests/golden fixtures, the oracle
and the CPU emulation of the kernel then solve the same QPs).  Prints one JSON line."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python")]
import impc  # noqa: E402
from impc import scenarios  # noqa: E402
from impc.replan import DeviceReplan, ROW_FIRST  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--instances", type=int, default=8192)
    ap.add_argument("--obstacles", type=int, default=4)
    ap.add_argument("--replans", type=int, default=30)
    ap.add_argument("--horizon", type=int, default=30)
    ap.add_argument("--max-dump", type=int, default=64)
    ap.add_argument("--out", default=os.path.join("gpurun_out", "r06", "noncvx.npz"))
    ap.add_argument("--watch", default="", help="instances (comma-separated) whose every replan is logged: "
                    "branch, chosen candidate, each candidate's status / iterations / max |x|, max |plan| after")
    a = ap.parse_args()
    I, K, R, N = a.instances, a.obstacles, a.replans, a.horizon
    sc = scenarios.live_loop(I, K, R, N=N, seed=4100)
    p, pd, L = sc["params"], sc["pd"], sc["L"]
    ctx = impc.Context(0)
    rp = DeviceReplan(ctx, p, pd, I, K, L, impc.default_settings(verbose=0))
    paths = impc.ReferencePaths(ctx, list(sc["paths"]), pd["ts"], N)
    D = impc.DeviceArray
    pos_d, vel_d, xref_d = D(ctx, sc["pos0"]), D(ctx, sc["vel0"]), D(ctx, (I, N, 8))
    psize_d, prob_d = D(ctx, sc["pred_size"]), D(ctx, np.ascontiguousarray(sc["prob"]))
    pred_d, cur_d = D(ctx, np.ascontiguousarray(sc["pred_pos"])), D(ctx, np.ascontiguousarray(sc["dyn_cur"]))
    step_pred, step_cur = pred_d.nbytes // R, cur_d.nbytes // R
    dump = {k: [] for k in ("replan", "inst", "code", "K", "Px", "q", "Ax", "l", "u", "x_ws", "status", "iter",
                            "setup_exitflag", "pri_res", "dua_res", "rho_updates")}
    per_replan = []
    watch = [int(v) for v in a.watch.split(",") if v]
    log = []
    for r in range(R):
        plan_x, first, _, _ = rp.plans()  # the warm starts of this replan
        paths.xref_device(pos_d.ptr, xref_d.ptr)
        rp.run_device(pos_d.ptr, vel_d.ptr, xref_d.ptr, cur_d.ptr + r * step_cur, pred_d.ptr + r * step_pred,
                      psize_d.ptr, prob_d.ptr)
        ctx.synchronize()
        out = rp.results(values=True)
        n_bad = 0
        for k, sh in out["shapes"].items():
            bad = np.flatnonzero(sh["info"]["status_val"] == impc.NON_CVX)
            n_bad += bad.size
            for row in bad:
                if len(dump["inst"]) >= a.max_dump:
                    break
                i, code = int(sh["row_inst"][row]), int(sh["row_code"][row])
                ws = np.zeros_like(plan_x[i]) if (code == ROW_FIRST and first[i]) else plan_x[i]
                dump["replan"].append(r)
                dump["inst"].append(i)
                dump["code"].append(code)
                dump["K"].append(k)
                for j, key in enumerate(("Px", "q", "Ax", "l", "u")):
                    dump[key].append(sh["vals"][j][row])
                dump["x_ws"].append(ws)
                inf = sh["info"][row]
                for key, f in (("status", "status_val"), ("iter", "iter"), ("setup_exitflag", "setup_exitflag"),
                               ("pri_res", "pri_res"), ("dua_res", "dua_res"), ("rho_updates", "rho_updates")):
                    dump[key].append(inf[f])
        per_replan.append(int(n_bad))
        if watch:
            plan_after, _, _, valid = rp.plans()
            for i in watch:
                cands = []
                for k, sh in out["shapes"].items():
                    for row in np.flatnonzero(sh["row_inst"] == i):
                        inf = sh["info"][row]
                        cands.append(dict(k=int(k), code=int(sh["row_code"][row]), status=int(inf["status_val"]),
                                          iter=int(inf["iter"]), max_abs_x=float(np.abs(sh["x"][row]).max())))
                log.append(dict(replan=r, inst=i, branch=int(out["branch"][i]), best=int(out["best_cand"][i]),
                                valid=int(valid[i]), max_abs_plan=float(np.abs(plan_after[i]).max()),
                                cands=sorted(cands, key=lambda c: c["code"])))
        rp.advance_device(pd["ts"], pos_d.ptr, vel_d.ptr)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    arrays = {}
    for k, v in dump.items():
        if not v:
            continue
        if k in ("Px", "q", "Ax", "l", "u"):  # rows of different shapes: one array per obstacle count
            for kk in sorted(set(dump["K"])):
                arrays[f"{k}_K{kk}"] = np.array([x for x, s in zip(v, dump["K"]) if s == kk])
        else:
            arrays[k] = np.array(v)
    np.savez(a.out, N=N, **arrays)
    if watch:
        with open(os.path.splitext(a.out)[0] + "_watch.json", "w") as f:
            json.dump(log, f, indent=0)
    print(json.dumps({"instances": I, "replans": R, "noncvx_per_replan": per_replan, "dumped": len(dump["inst"]),
                      "out": a.out, "build_id": impc.lib.impc_build_id().decode()}), flush=True)
    for d in (pos_d, vel_d, xref_d, psize_d, prob_d, pred_d, cur_d):
        d.free()
    paths.close()
    rp.close()
    ctx.close()


if __name__ == "__main__":
    main()
