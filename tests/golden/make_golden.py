"""Generates the committed golden vectors under tests/golden/ (run: python tests/golden/make_golden.py).

The reference has no tests for this path and its vendored libosqp.so is prebuilt machine code that
may not be executed here, so the expected outputs come from the oracle (oracle/osqp_oracle.c, the
C restatement of OSQP 0.6.2) -- "parity unpinned" against the real binary.  Inputs come
from the product builder on seeded scenarios (SURVEY.md 8c fixture plan G1-G6).  Each .npz holds
the CSC pattern, per-QP values, warm start, pinned settings and the oracle's x, y, info.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python")]

import impc  # noqa: E402
from impc import scenarios  # noqa: E402
from oracle import osqp_oracle as ora  # noqa: E402

SETTINGS = dict(verbose=0, adaptive_rho_interval=25)


def fixtures():
    b3 = scenarios.intent_config(instances=1, seed=3303)
    g6 = scenarios.static_config(batch=3, identical=False, seed=606)
    l = g6["values"]["l"].copy()
    l[0, 8 * 20 + 1] = 4.9  # box row contradicting the pinned x0 -> primal infeasible
    g6 = dict(g6, values=dict(g6["values"], l=l))
    return {
        "G1_first_call": (scenarios.first_call_config(batch=1, seed=1001), {}),
        "G2_static_K10": (scenarios.static_config(batch=2, identical=False, seed=2002), {}),
        "G3_intent_K8": (b3[8], {}),
        "G3_intent_K9": (b3[9], {}),
        "G4_N40_K10": (scenarios.static_config(N=40, K=10, batch=1, identical=False, seed=4004), {}),
        "G6_infeasible": (g6, {}),
        "G7_max_iter": (scenarios.static_config(batch=1, identical=False, seed=707), {"max_iter": 60}),
    }


def main():
    for name, (cfg, extra) in fixtures().items():
        s = impc.default_settings(**dict(SETTINGS, **extra))
        v, pat = cfg["values"], cfg["pattern"]
        x, y, info = ora.solve_batch(pat, v["Px"], v["q"], v["Ax"], v["l"], v["u"], ora.settings_from(s),
                                     x_ws=cfg.get("x_ws"), threads=1)
        arrays = dict(n=pat["n"], m=pat["m"], Pp=pat["Pp"], Pi=pat["Pi"], Ap=pat["Ap"], Ai=pat["Ai"],
                      Px=v["Px"], q=v["q"], Ax=v["Ax"], l=v["l"], u=v["u"],
                      x_ws=cfg["x_ws"] if cfg.get("x_ws") is not None else np.zeros((0,)),
                      settings=np.array([getattr(s, f) for f, _ in impc.Settings._fields_], dtype=np.float64),
                      x=x, y=y, iter=info["iter"], status_val=info["status_val"], obj_val=info["obj_val"],
                      rho_updates=info["rho_updates"])
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **arrays)
        print(name, "B=%d" % v["q"].shape[0], "iters", info["iter"], "status", info["status_val"],
              "%.0f KB" % (os.path.getsize(path) / 1024))


if __name__ == "__main__":
    main()
