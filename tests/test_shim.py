"""include/OsqpEigen/OsqpEigen.h -- the OsqpEigen-compatible C++ front end -- driven with the
mpcPlanner::solveTraj call sequence (reference mpcPlanner.cpp:436-527) by tests/native/shim_test.cpp
(compiled against a test-only Eigen stand-in, since Eigen is not in this image)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "build", "shim_test")


def run(mode):
    p = subprocess.run([EXE, mode], capture_output=True, text=True, timeout=120)
    return p.returncode, p.stdout + p.stderr


def test_shim_conversion_and_no_device_behaviour():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible: the no-device path is not reachable")
    rc, out = run("cpu")
    assert rc == 0, out
    assert "no HIP device" in out  # fails loudly: no CPU fallback


@pytest.mark.gpu
def test_shim_solves_on_gpu():
    rc, out = run("gpu")
    assert rc == 0, out


def _replay(tmp_path, cfg, updates=None, matrices=None):
    """Run the QPs of cfg through the shim's solveTraj call sequence (shim_test replay) and read
    back status / iterations / objective / x / y per solve step."""
    pat, v = cfg["pattern"], cfg["values"]
    n, m = int(pat["n"]), int(pat["m"])
    B = v["q"].shape[0]
    xw = cfg.get("x_ws")
    flags = (1 if xw is not None else 0) | (2 if updates is not None else 0) | (4 if matrices is not None else 0)
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(fin, "wb") as f:
        np.array([n, m, len(pat["Pi"]), len(pat["Ai"]), B, flags], np.int64).tofile(f)
        for k in ("Pp", "Pi", "Ap", "Ai"):
            np.ascontiguousarray(pat[k], np.int64).tofile(f)
        for i in range(B):
            for k in ("Px", "q", "Ax", "l", "u"):
                np.ascontiguousarray(v[k][i], float).tofile(f)
            if xw is not None:
                np.ascontiguousarray(xw[i], float).tofile(f)
            if updates is not None:
                for a in updates:
                    np.ascontiguousarray(a[i], float).tofile(f)
            if matrices is not None:
                for a in matrices:
                    np.ascontiguousarray(a[i], float).tofile(f)
    p = subprocess.run([EXE, "replay", str(fin), str(fout)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    steps = (5 if matrices is not None else 3) if updates is not None else 1
    raw = np.fromfile(fout, float).reshape(B, steps, 3 + n + m)
    return [(raw[:, s, 3:3 + n], raw[:, s, 3 + n:], raw[:, s, 0].astype(int), raw[:, s, 1].astype(int),
             raw[:, s, 2]) for s in range(steps)]


def _check(step, ref, rtol=1e-5):
    """BASELINE.json's parity bar against the oracle: identical status and iteration count, primal,
    duals and objective within 1e-5 relative where a solution exists."""
    x, y, st, it, obj = step
    xo, yo, so, io_, oo = ref
    assert np.array_equal(st, so), (st, so)
    assert np.array_equal(it, io_), (it, io_)
    has = np.isin(so, (1, 2, -2, -6))
    assert has.any()
    rel = lambda a, b: np.abs(a - b).max(axis=1) / np.maximum(np.abs(b).max(axis=1), 1e-12)  # noqa: E731
    assert rel(x[has], xo[has]).max() <= rtol
    assert rel(y[has], yo[has]).max() <= rtol
    assert (np.abs(obj[has] - oo[has]) / np.maximum(np.abs(oo[has]), 1e-12)).max() <= rtol


@pytest.mark.gpu
def test_shim_solvetraj_sequence_vs_oracle(tmp_path):
    """Row a8: config-1 (first call, cold) and config-3 (intent hypotheses, warm start from the
    previous plan, y = 0) QPs through OsqpEigen::Solver as solveTraj drives it
    (mpcPlanner.cpp:436-527), checked against the oracle's osqp_setup + osqp_warm_start +
    osqp_solve -- the shim's Eigen -> upper-triangle CSC conversion (explicit zeros kept) and
    its setWarmStart included."""
    import impc
    from impc import scenarios
    from oracle import osqp_oracle as ora
    os_ = ora.settings_from(impc.default_settings(verbose=0, warm_start=1))
    cfgs = [scenarios.first_call_config(batch=6, seed=811)]
    cfgs += list(scenarios.intent_config(instances=2, hyps=8, seed=812).values())
    for cfg in cfgs:
        (res,) = _replay(tmp_path, cfg)
        v = cfg["values"]
        B = v["q"].shape[0]
        xw = cfg.get("x_ws")
        yw = None if xw is None else np.zeros((B, int(cfg["pattern"]["m"])))
        xo, yo, io = ora.solve_batch(cfg["pattern"], v["Px"], v["q"], v["Ax"], v["l"], v["u"], os_, x_ws=xw,
                                     y_ws=yw, threads=4)
        _check(res, (xo, yo, io["status_val"], io["iter"], io["obj_val"]))


@pytest.mark.gpu
def test_shim_update_sequence_vs_persistent_oracle(tmp_path):
    """Row a8, persistent use: solve -> updateGradient -> solve -> updateBounds -> solve through the
    shim (Solver.hpp updateGradient / updateBounds -> osqp_update_lin_cost / osqp_update_bounds)
    against the oracle's persistent workspace over the same sequence."""
    import impc
    from impc import scenarios
    from oracle import osqp_oracle as ora
    os_ = ora.settings_from(impc.default_settings(verbose=0, warm_start=1))
    bk = scenarios.intent_config(instances=1, hyps=8, seed=813)[8]
    v = bk["values"]
    B, m = v["q"].shape[0], int(bk["pattern"]["m"])
    rng = np.random.default_rng(814)
    q2 = v["q"] * (1 + 0.05 * rng.standard_normal(v["q"].shape))
    l3, u3 = v["l"].copy(), v["u"].copy()
    fin = np.isfinite(l3) & np.isfinite(u3) & (u3 - l3 > 0.1)
    l3[fin] += 0.01
    u3[fin] -= 0.01
    steps = _replay(tmp_path, bk, updates=(q2, l3, u3))
    for i in range(B):
        w = ora.Workspace(bk["pattern"], v["Px"][i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], os_)
        w.warm_start(bk["x_ws"][i], np.zeros(m))
        refs = [w.solve()]
        w.update_lin_cost(q2[i])
        refs.append(w.solve())
        w.update_bounds(l3[i], u3[i])
        refs.append(w.solve())
        w.close()
        for s, (xo, yo, io) in enumerate(refs):
            got = tuple(a[i:i + 1] for a in steps[s])
            _check(got, (xo[None], yo[None], np.array([io["status_val"]]), np.array([io["iter"]]),
                         np.array([io["obj_val"]])))


@pytest.mark.gpu
def test_shim_matrix_updates_vs_osqp_update_P_A(tmp_path):
    """updateHessianMatrix / updateLinearConstraintsMatrix on an unchanged pattern through the shim
    (Solver.tpp:15-212 -> osqp_update_P / osqp_update_A) against the oracle's persistent workspace:
    solve -> updateGradient -> solve -> updateBounds -> solve -> new P -> solve -> new A -> solve,
    identical statuses and iterations, x / y / objective within 1e-5."""
    import impc
    from impc import scenarios
    from oracle import osqp_oracle as ora
    os_ = ora.settings_from(impc.default_settings(verbose=0, warm_start=1))
    bk = scenarios.intent_config(instances=1, hyps=8, seed=815)[8]
    v = bk["values"]
    B, m = v["q"].shape[0], int(bk["pattern"]["m"])
    rng = np.random.default_rng(816)
    q2 = v["q"] * (1 + 0.05 * rng.standard_normal(v["q"].shape))
    l3, u3 = v["l"].copy(), v["u"].copy()
    fin = np.isfinite(l3) & np.isfinite(u3) & (u3 - l3 > 0.1)
    l3[fin] += 0.01
    u3[fin] -= 0.01
    P4 = v["Px"] * (1.0 + 0.5 * rng.uniform(size=v["Px"].shape))
    A4 = v["Ax"] * (1.0 + 0.02 * rng.standard_normal(v["Ax"].shape))
    steps = _replay(tmp_path, bk, updates=(q2, l3, u3), matrices=(P4, A4))
    for i in range(B):
        w = ora.Workspace(bk["pattern"], v["Px"][i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], os_)
        w.warm_start(bk["x_ws"][i], np.zeros(m))
        refs = [w.solve()]
        w.update_lin_cost(q2[i])
        refs.append(w.solve())
        w.update_bounds(l3[i], u3[i])
        refs.append(w.solve())
        w.update_matrices(P4[i], None)
        refs.append(w.solve())
        w.update_matrices(None, A4[i])
        refs.append(w.solve())
        w.close()
        for s, (xo, yo, io) in enumerate(refs):
            got = tuple(a[i:i + 1] for a in steps[s])
            _check(got, (xo[None], yo[None], np.array([io["status_val"]]), np.array([io["iter"]]),
                         np.array([io["obj_val"]])))


def _bench_file(tmp_path, cfg):
    pat, v = cfg["pattern"], cfg["values"]
    n, m = int(pat["n"]), int(pat["m"])
    B = v["q"].shape[0]
    xw = cfg.get("x_ws")
    fin = tmp_path / "bench_in.bin"
    with open(fin, "wb") as f:
        np.array([n, m, len(pat["Pi"]), len(pat["Ai"]), B, 1 if xw is not None else 0], np.int64).tofile(f)
        for k in ("Pp", "Pi", "Ap", "Ai"):
            np.ascontiguousarray(pat[k], np.int64).tofile(f)
        for i in range(B):
            for k in ("Px", "q", "Ax", "l", "u"):
                np.ascontiguousarray(v[k][i], float).tofile(f)
            if xw is not None:
                np.ascontiguousarray(xw[i], float).tofile(f)
    return fin


@pytest.mark.gpu
def test_shim_per_call_cost(tmp_path):
    """The drop-in path's cost per solveTraj call (Solver -> initSolver -> setWarmStart -> solveProblem
    -> getSolution -> clearSolver) on a known pattern: with the workspace pool the host wall time
    stays within 0.25 ms of the device time of the same QP (measured ~0.1 ms, profiles/r04)."""
    import json
    from impc import scenarios
    cfg = next(iter(scenarios.intent_config(N=20, K=8, instances=4, hyps=8, seed=31).values()))
    fin = _bench_file(tmp_path, cfg)
    p = subprocess.run([EXE, "bench", str(fin), "200"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    print(r)
    assert r["pool"] and r["calls"] == 200
    assert r["host_wall_ms"]["p50"] <= r["device_event_ms"]["p50"] + 0.25, r


@pytest.mark.gpu
def test_workspace_pool_reuses_and_resets(ctx):
    """impc_batch_acquire / impc_batch_release: a released batch of the same pattern comes back
    (same handle, default settings, no warm start, all QPs active), another pattern does not."""
    import ctypes as C
    import impc
    from impc import scenarios
    cfg = scenarios.first_call_config(batch=2, seed=5)
    pat, v = cfg["pattern"], cfg["values"]
    arrs = [np.ascontiguousarray(pat[k], np.int64) for k in ("Pp", "Pi", "Ap", "Ai")]
    ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64))  # noqa: E731
    h1, h2, h3 = C.c_void_p(), C.c_void_p(), C.c_void_p()
    assert impc.lib.impc_batch_acquire(ctx.h, pat["n"], pat["m"], *[ip(a) for a in arrs], 2, C.byref(h1)) == 0
    b = impc.Batch.__new__(impc.Batch)
    b.ctx, b.h, b.n, b.m, b.B = ctx, h1, int(pat["n"]), int(pat["m"]), 2
    b.nnzP, b.nnzA = int(arrs[0][-1]), int(arrs[2][-1])
    s = impc.default_settings(verbose=0, max_iter=7)
    b.set_settings(s)
    b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
    b.set_active(1)
    b.solve()
    _, _, info = b.get()
    assert info["iter"][0] <= 7
    assert impc.lib.impc_batch_release(h1) == 0
    assert impc.lib.impc_batch_acquire(ctx.h, pat["n"], pat["m"], *[ip(a) for a in arrs], 2, C.byref(h2)) == 0
    assert h2.value == h1.value
    b.h = h2
    b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
    b.solve()  # default settings again (max_iter 4000), both QPs active
    _, _, info2 = b.get()
    assert (info2["iter"] > 7).all() and (info2["status_val"] == 1).all()
    assert impc.lib.impc_batch_acquire(ctx.h, pat["n"], pat["m"], *[ip(a) for a in arrs], 1, C.byref(h3)) == 0
    assert h3.value != h2.value  # other capacity: a new batch
    b.h = None  # released below: the pool owns it (Batch.__del__ must not destroy it)
    for h in (h2, h3):
        assert impc.lib.impc_batch_release(h) == 0


@pytest.mark.gpu
def test_staged_values_results_subsets_and_update_order(ctx):
    """The small-batch staging: values and warm start staged and uploaded in one DMA
    by the solve, results back in one DMA; a partial impc_batch_get (x only, info only, y only)
    returns what the full one does, and values staged after a solve replace the solved ones."""
    import ctypes as C
    import impc
    from impc import scenarios
    cfg = scenarios.intent_config(N=20, K=8, instances=1, hyps=4, seed=77)[8]
    pat, v = cfg["pattern"], cfg["values"]
    B, n, m = v["q"].shape[0], int(pat["n"]), int(pat["m"])
    b = impc.Batch(ctx, n, m, pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    try:
        b.set_settings(impc.default_settings(verbose=0))
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.warm_start(cfg["x_ws"])
        b.solve()
        x, y, info = b.get()
        xs, ys = np.empty((B, n)), np.empty((B, m))
        inf_s = np.empty(B, dtype=impc.INFO_DTYPE)
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        assert impc.lib.impc_batch_get(b.h, dp(xs), None, None) == 0
        assert impc.lib.impc_batch_get(b.h, None, dp(ys), None) == 0
        assert impc.lib.impc_batch_get(b.h, None, None, inf_s.ctypes.data_as(C.c_void_p)) == 0
        assert np.array_equal(xs, x) and np.array_equal(ys, y)
        assert np.array_equal(inf_s["iter"], info["iter"]) and np.array_equal(inf_s["status_val"], info["status_val"])
        # re-staged values (another cost) after a solve: the next solve sees them, not the old ones
        q2 = np.ascontiguousarray(v["q"] * 0.5)
        b.set_values(v["Px"], q2, v["Ax"], v["l"], v["u"])
        b.warm_start(cfg["x_ws"])
        b.solve()
        x2, _, info2 = b.get()
        ref = oracle_solve(dict(cfg, values=dict(v, q=q2)))
        assert np.array_equal(info2["iter"], ref[2]["iter"])
        assert np.max(np.abs(x2 - ref[0])) <= 1e-5 * max(1.0, np.max(np.abs(ref[0])))
    finally:
        b.close()


def oracle_solve(cfg):
    from helpers import oracle
    import impc
    return oracle(cfg, impc.default_settings(verbose=0))


@pytest.mark.gpu
def test_workspace_pool_is_bounded_and_rejects_double_release(ctx):
    """Releasing more than the pool's 64 batches (distinct capacities, so no reuse) destroys the
    oldest: the pool stays at 64 batches and its device bytes stay those of 64 batches; releasing
    a pooled batch again is refused (the eviction used to drop a second batch unfreed)."""
    import ctypes as C
    import impc
    from impc import scenarios
    cfg = scenarios.first_call_config(batch=1, seed=5)
    pat = cfg["pattern"]
    arrs = [np.ascontiguousarray(pat[k], np.int64) for k in ("Pp", "Pi", "Ap", "Ai")]
    ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64))  # noqa: E731
    nb, nbytes = C.c_int64(), C.c_int64()
    handles = []
    for cap in range(1, 73):
        h = C.c_void_p()
        assert impc.lib.impc_batch_acquire(ctx.h, pat["n"], pat["m"], *[ip(a) for a in arrs], cap, C.byref(h)) == 0
        handles.append(h)
    assert impc.lib.impc_ctx_pool_stats(ctx.h, C.byref(nb), C.byref(nbytes)) == 0
    base = nb.value  # batches other tests left pooled (acquires of a pooled capacity took them out)
    per = []
    for k, h in enumerate(handles):
        assert impc.lib.impc_batch_release(h) == 0
        assert impc.lib.impc_ctx_pool_stats(ctx.h, C.byref(nb), C.byref(nbytes)) == 0
        assert nb.value == min(base + k + 1, 64), (k, nb.value)
        per.append(nbytes.value)
    # the last 64 released batches remain, and they alone hold the pool's device memory
    assert impc.lib.impc_batch_release(handles[-1]) == 101  # IMPC_INVALID_ARGUMENT
    assert impc.lib.impc_ctx_pool_stats(ctx.h, C.byref(nb), C.byref(nbytes)) == 0
    assert nb.value == 64 and nbytes.value == per[-1]
    # past 64, each release adds one batch of capacity c and evicts the one of capacity c - 64:
    # the pool's bytes move by the difference of the two, never by a whole extra batch
    steps = np.diff(per[-8:])
    assert (steps == steps[0]).all(), steps


@pytest.mark.gpu
def test_set_active_generic_kernel_leaves_inactive_rows(ctx):
    """impc_batch_set_active on the generic kernel: rows >= count keep the results they held (the
    kernel, the warm-start and update kernels and the result copy take the active rows only)."""
    import impc
    from impc import scenarios
    bk = scenarios.intent_config(N=20, K=3, instances=2, hyps=4, seed=21)[3]
    pat, v = bk["pattern"], bk["values"]
    B = v["q"].shape[0]
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B).set_kernel(
        impc.KERNEL_GENERIC)
    try:
        s = impc.default_settings(verbose=0)
        b.set_settings(s)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.warm_start(bk["x_ws"], None)
        b.solve()
        x0, y0, i0 = b.get()
        b.set_active(B // 2)
        b.set_values(v["Px"], 0.5 * v["q"], v["Ax"], v["l"], v["u"])
        b.warm_start(bk["x_ws"], None)
        b.solve()
        x1, y1, i1 = b.get()
        np.testing.assert_array_equal(x1[B // 2:], x0[B // 2:])
        np.testing.assert_array_equal(y1[B // 2:], y0[B // 2:])
        np.testing.assert_array_equal(i1["iter"][B // 2:], i0["iter"][B // 2:])
        assert (x1[: B // 2] != x0[: B // 2]).any()
        b.update_lin_cost(v["q"])  # the persistent update of the active rows only
        b.solve()
        x2, _, _ = b.get()
        np.testing.assert_array_equal(x2[B // 2:], x0[B // 2:])
    finally:
        b.close()
