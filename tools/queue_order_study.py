"""Which a-priori QP features rank config 3's ADMM iteration counts, and what a work-queue order
built on them does to a persistent launch's makespan (the study behind IMPC_QUEUE_LONGEST_FIRST).

Solves a sample of config-3 QPs with the oracle (CPU), computes per QP the warm start's
constraint violation ||A x_ws - proj_[l,u](A x_ws)||_inf, ||q||_inf and the reference's mean
step, prints their Spearman correlation with the iteration count, then list-schedules the sample
on `slots` workgroups (time = iterations) in FIFO order, in descending key order for the
candidate keys, and in the (unknowable) true longest-first order.

    python tools/queue_order_study.py [instances] [seed]
"""
import heapq
import os
import sys

import numpy as np
import scipy.sparse as sp
from scipy.stats import spearmanr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intent-mpc_amd", "python"))
sys.path.insert(0, ROOT)
import impc  # noqa: E402
from impc import scenarios  # noqa: E402
from oracle import osqp_oracle as ora  # noqa: E402


def makespan(order, it, slots):
    h = [0.0] * slots
    for j in order:
        heapq.heappush(h, heapq.heappop(h) + it[j])
    return max(h)


def main():
    I = int(sys.argv[1]) if len(sys.argv) > 1 else 768
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
    bks = scenarios.intent_config(N=20, K=8, instances=I, hyps=8, seed=seed)
    s = ora.settings_from(impc.default_settings(verbose=0))
    it, viol, qmax, step = [], [], [], []
    for K, bk in sorted(bks.items()):
        v, pat = bk["values"], bk["pattern"]
        _, _, info = ora.solve_batch(pat, v["Px"], v["q"], v["Ax"], v["l"], v["u"], s, x_ws=bk["x_ws"], threads=8)
        it.append(info["iter"])
        for i in range(v["q"].shape[0]):
            A = sp.csc_matrix((v["Ax"][i], pat["Ai"], pat["Ap"]), shape=(pat["m"], pat["n"]))
            ax = A @ bk["x_ws"][i]
            viol.append(max(0.0, float(np.max(np.maximum(v["l"][i] - ax, ax - v["u"][i])))))
            qmax.append(float(np.abs(v["q"][i]).max()))
            xr = bk["instances"]["xref"][bk["inst"][i]]
            step.append(float(np.linalg.norm(np.diff(xr[:, :3], axis=0), axis=1).mean()))
    it = np.concatenate(it).astype(float)
    viol, qmax, step = map(np.array, (viol, qmax, step))
    for nm, f in (("warm-start violation", viol), ("||q||_inf", qmax), ("reference step", step)):
        print(f"spearman(iter, {nm}) = {spearmanr(it, f).correlation:.3f}")
    tail = it >= 4000
    print(f"QPs at the 4000-iteration cap: {int(tail.sum())}; of them with violation > 0.3: "
          f"{float((viol[tail] > 0.3).mean()) if tail.any() else float('nan'):.2f}; all QPs with violation > 0.3: "
          f"{float((viol > 0.3).mean()):.3f}")
    pd = scenarios.mpc_params(horizon=20)[1]
    qw = scenarios.queue_weight(pd, 20)
    n = it.size
    for slots, sub in ((512, np.arange(n)), (64, np.arange(min(n, 1024)))):
        i2 = it[sub]
        row = dict(fifo=makespan(sub, it, slots))
        for nm, key in (("violation", viol), ("q", qmax), ("violation + q_weight*q", viol + qw * qmax)):
            row[nm] = makespan(sub[np.argsort(-key[sub], kind="stable")], it, slots)
        row["true LPT"] = makespan(sub[np.argsort(-i2, kind="stable")], it, slots)
        row["lower bound"] = float(i2.sum() / slots)
        print(f"{sub.size} QPs on {slots} slots (makespan in iterations):",
              ", ".join(f"{k} {v:.0f}" for k, v in row.items()))


if __name__ == "__main__":
    main()
