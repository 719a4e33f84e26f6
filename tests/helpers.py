"""Shared test helpers: oracle / GPU / CPU-harness runners and the parity comparison."""
import ctypes as C
import os

import numpy as np

import impc
from oracle import osqp_oracle as ora

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS_PATH = os.path.join(ROOT, "tests", "native", "build", "libimpc_core_cpu.so")
EMU_PATH = os.path.join(ROOT, "tests", "native", "build", "libwave_emu.so")
EMU64_PATH = os.path.join(ROOT, "tests", "native", "build", "libwave_emu64.so")  # one QP per wavefront

# BASELINE.json north_star: primal within 1e-5 relative of the reference solver.
PRIMAL_RTOL = 1e-5
# Duals: same iteration sequence on both sides, so the same relative bound is used for y.
DUAL_RTOL = 1e-5
HAS_SOLUTION = (1, 2, -2, -6)  # solved, solved inaccurate, max iter, time limit


def oracle(cfg, settings):
    v = cfg["values"]
    return ora.solve_batch(cfg["pattern"], v["Px"], v["q"], v["Ax"], v["l"], v["u"], ora.settings_from(settings),
                           x_ws=cfg.get("x_ws"), threads=min(8, os.cpu_count() or 1))


def gpu(ctx, cfg, settings, kernel=impc.KERNEL_AUTO):
    pat, v = cfg["pattern"], cfg["values"]
    B = v["q"].shape[0]
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    try:
        if kernel == impc.KERNEL_STRUCTURED and not b.stats()["structured_ok"]:
            import pytest
            pytest.skip("pattern outside the structured kernel's limits (n <= 256, general rows <= 512)")
        b.set_kernel(kernel)
        if kernel != impc.KERNEL_AUTO:
            assert b.stats()["kernel"] == kernel
        b.set_settings(settings)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        if cfg.get("x_ws") is not None:
            b.warm_start(cfg["x_ws"], None)
        b.solve()
        return b.get()
    finally:
        b.close()


_H = None


def harness(cfg, settings):
    """Test-only CPU build of admm_core.hpp (same algorithm as the GPU kernels)."""
    global _H
    if _H is None:
        _H = C.CDLL(HARNESS_PATH)
        _H.harness_solve_batch.restype = C.c_int
    pat, v = cfg["pattern"], cfg["values"]
    B = v["q"].shape[0]
    n, m = pat["n"], pat["m"]
    keep = [np.ascontiguousarray(v[k], float) for k in ("Px", "q", "Ax", "l", "u")]
    pats = [np.ascontiguousarray(pat[k], np.int64) for k in ("Pp", "Pi", "Ap", "Ai")]
    xw = None if cfg.get("x_ws") is None else np.ascontiguousarray(cfg["x_ws"], float)
    yw = None if xw is None else np.zeros((B, m))
    xo, yo = np.empty((B, n)), np.empty((B, m))
    info = np.empty(B, dtype=impc.INFO_DTYPE)
    nnzL = C.c_int64()
    p = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)  # noqa: E731
    rc = _H.harness_solve_batch(C.c_int64(n), C.c_int64(m), *[p(a) for a in pats], C.c_int64(B),
                                *[p(a) for a in keep], C.byref(settings), p(xw), p(yw), p(xo), p(yo),
                                info.ctypes.data_as(C.c_void_p), C.byref(nnzL))
    assert rc == 0
    return xo, yo, info


_E = {}


def emulate(cfg, settings, path=EMU_PATH):
    """Test-only CPU emulation of the structured wave kernel (mpc_wave.hpp, 256 lanes as threads;
    path=EMU64_PATH: the 64-lane team shape)."""
    if path not in _E:
        _E[path] = C.CDLL(path)
        _E[path].emu_wave_solve_batch.restype = C.c_int
    E = _E[path]
    pat, v = cfg["pattern"], cfg["values"]
    B = v["q"].shape[0]
    n, m = pat["n"], pat["m"]
    keep = [np.ascontiguousarray(v[k], float) for k in ("Px", "q", "Ax", "l", "u")]
    pats = [np.ascontiguousarray(pat[k], np.int64) for k in ("Pp", "Pi", "Ap", "Ai")]
    xw = None if cfg.get("x_ws") is None else np.ascontiguousarray(cfg["x_ws"], float)
    yw = None if xw is None else np.zeros((B, m))
    xo, yo = np.empty((B, n)), np.empty((B, m))
    info = np.empty(B, dtype=impc.INFO_DTYPE)
    p = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)  # noqa: E731
    rc = E.emu_wave_solve_batch(C.c_int64(n), C.c_int64(m), *[p(a) for a in pats], C.c_int64(B),
                                 *[p(a) for a in keep], C.byref(settings), p(xw), p(yw), p(xo), p(yo),
                                 info.ctypes.data_as(C.c_void_p))
    assert rc == 0, rc
    return xo, yo, info


def take(cfg, k):
    """First k QPs of a config."""
    out = dict(cfg, values={kk: vv[:k] for kk, vv in cfg["values"].items()})
    if cfg.get("x_ws") is not None:
        out["x_ws"] = cfg["x_ws"][:k]
    return out


def compare(res, ref, rtol=PRIMAL_RTOL, exact_iters=True):
    """Parity of a batch against the oracle: identical status (and iteration count), primal
    within rtol relative (inf-norm over the QP) where a solution exists, NaN-constant otherwise."""
    x, y, info = res
    xo, yo, io = ref
    assert np.array_equal(info["status_val"], io["status_val"]), (info["status_val"], io["status_val"])
    if exact_iters:
        assert np.array_equal(info["iter"], io["iter"]), (info["iter"], io["iter"])
    has = np.isin(io["status_val"], HAS_SOLUTION)
    worst = 0.0
    if has.any():
        scale = np.maximum(np.abs(xo[has]).max(axis=1), 1e-12)
        rel = np.abs(x[has] - xo[has]).max(axis=1) / scale
        worst = float(rel.max())
        assert worst <= rtol, worst
        yscale = np.maximum(np.abs(yo[has]).max(axis=1), 1e-12)
        yrel = np.abs(y[has] - yo[has]).max(axis=1) / yscale
        assert yrel.max() <= DUAL_RTOL, yrel.max()
        objrel = np.abs(info["obj_val"][has] - io["obj_val"][has]) / np.maximum(np.abs(io["obj_val"][has]), 1e-12)
        assert objrel.max() <= rtol, objrel.max()
    if (~has).any():
        assert np.all(x[~has] == impc.OSQP_NAN) and np.all(xo[~has] == impc.OSQP_NAN)
    return worst
