"""Committed golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces them bit-for-bit (regression pin of the restatement) and the generic
device algorithm (host build) to PRIMAL_RTOL.  GPU: both device kernels reproduce them
(identical status and iteration count, primal/dual within PRIMAL_RTOL/DUAL_RTOL).
"""
import ctypes as C
import glob
import os

import numpy as np
import pytest

import impc
from oracle import osqp_oracle as ora

from helpers import compare, gpu, harness

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(HERE, "G*.npz")))  # the G1-G7 vectors (tail_seed3000.npz: test_tail_seed3000.py)
NAMES = [os.path.basename(f)[:-4] for f in FILES]


def load(name):
    z = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    pat = dict(n=int(z["n"]), m=int(z["m"]), Pp=z["Pp"], Pi=z["Pi"], Ap=z["Ap"], Ai=z["Ai"])
    vals = {k: z[k] for k in ("Px", "q", "Ax", "l", "u")}
    s = impc.Settings()
    for (f, t), v in zip(impc.Settings._fields_, z["settings"]):
        setattr(s, f, float(v) if t is C.c_double else int(v))
    info = np.zeros(z["iter"].shape[0], dtype=impc.INFO_DTYPE)
    info["iter"], info["status_val"], info["obj_val"] = z["iter"], z["status_val"], z["obj_val"]
    info["rho_updates"] = z["rho_updates"]
    cfg = dict(pattern=pat, values=vals, x_ws=z["x_ws"] if z["x_ws"].size else None)
    return cfg, s, (z["x"], z["y"], info)


def test_fixtures_present():
    assert {"G1_first_call", "G2_static_K10", "G3_intent_K8", "G3_intent_K9", "G4_N40_K10", "G6_infeasible",
            "G7_max_iter"} <= set(NAMES)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden_bitwise(name):
    cfg, s, (x, y, info) = load(name)
    v = cfg["values"]
    xo, yo, io = ora.solve_batch(cfg["pattern"], v["Px"], v["q"], v["Ax"], v["l"], v["u"], ora.settings_from(s),
                                 x_ws=cfg["x_ws"], threads=1)
    np.testing.assert_array_equal(xo, x)
    np.testing.assert_array_equal(yo, y)
    np.testing.assert_array_equal(io["iter"], info["iter"])
    np.testing.assert_array_equal(io["status_val"], info["status_val"])


@pytest.mark.parametrize("name", NAMES)
def test_generic_core_reproduces_golden(name):
    cfg, s, ref = load(name)
    compare(harness(cfg, s), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [impc.KERNEL_GENERIC, impc.KERNEL_STRUCTURED], ids=["generic", "structured"])
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reproduces_golden(ctx, name, kernel):
    cfg, s, ref = load(name)
    compare(gpu(ctx, cfg, s, kernel), ref)
