"""Diagnostic (tools only): the live loop of tests/test_live_loop.py, replan by replan, reporting the
first assembled-QP mismatch against the restatement with its replan, instance, candidate and rows."""
import os
import sys

R0 = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R0, 'tests'), os.path.join(R0, 'intent-mpc_amd/python'), R0]
import numpy as np  # noqa: E402
import impc  # noqa: E402
from impc import scenarios  # noqa: E402
from impc.replan import DeviceReplan  # noqa: E402
from oracle import replan_ref as ref  # noqa: E402
from oracle.reftraj_ref import ReferencePath  # noqa: E402

I, K, R, N = 6, 3, 30, 30
sc = scenarios.live_loop(I, K, R, N=N, seed=4100)
p, pd, L = sc["params"], sc["pd"], sc["L"]
s = impc.default_settings(verbose=0)
ctx = impc.Context(0)
rp = DeviceReplan(ctx, p, pd, I, K, L, s)
paths = impc.ReferencePaths(ctx, list(sc["paths"]), pd["ts"], N)
refs = [ReferencePath(pth, pd["ts"], N) for pth in sc["paths"]]
D = impc.DeviceArray
pos_d, vel_d, xref_d = D(ctx, sc["pos0"]), D(ctx, sc["vel0"]), D(ctx, (I, N, 8))
psize_d, prob_d = D(ctx, sc["pred_size"]), D(ctx, np.ascontiguousarray(sc["prob"]))
done = False
for r in range(R):
    pred_d, cur_d = D(ctx, np.ascontiguousarray(sc["pred_pos"][r])), D(ctx, sc["dyn_cur"][r])
    before = rp.plans()
    pos, vel = pos_d.get(), vel_d.get()
    paths.xref_device(pos_d.ptr, xref_d.ptr)
    rp.run_device(pos_d.ptr, vel_d.ptr, xref_d.ptr, cur_d.ptr, pred_d.ptr, psize_d.ptr, prob_d.ptr)
    ctx.synchronize()
    out = rp.results()
    xref = xref_d.get()
    exp_x = np.array([refs[i].xref(pos[i]) for i in range(I)])
    print("replan", r, "branches", out["branch"].tolist(), "xref ok", np.array_equal(xref, exp_x),
          "valid", out["valid"].tolist(), "best", out["best_cand"].tolist(), flush=True)
    for j, i in enumerate(out["inst_fanout"]):
        px = before[0][i]
        fo, qps = ref.fanout_qps(pd, 0, px, pos[i], vel[i], xref[i], sc["dyn_cur"][r][i], sc["pred_pos"][r][i],
                                 sc["pred_size"][i], sc["prob"][i])
        if out["ob_idx"][i] != fo["ob_idx"]:
            print("  ob_idx differs", i, out["ob_idx"][i], fo["ob_idx"])
        for c in range(6):
            slot = out["cand_slot"][i][c]
            nm, row = ("single", 4 * j + slot) if slot < 4 else ("pair", 2 * j + slot - 4)
            for kk, key in enumerate(("Px", "q", "Ax", "l", "u")):
                got, want = out["vals_" + nm][kk][row], qps[c][1][key]
                bad = np.flatnonzero((got != want) & ~(np.isnan(got) & np.isnan(want)))
                if bad.size:
                    print(f"  r{r} inst {i} cand {c} slot {slot} {key}: {bad.size} differ, idx {bad[:6].tolist()} "
                          f"got {got[bad[:3]].tolist()} want {want[bad[:3]].tolist()}")
                    print("    lin state 0..2 of plan:", px[:3].tolist(), px[8:11].tolist(), "pos", pos[i].tolist())
                    done = True
    if done:
        break
    rp.advance_device(pd["ts"], pos_d.ptr, vel_d.ptr)
    pred_d.free()
    cur_d.free()
