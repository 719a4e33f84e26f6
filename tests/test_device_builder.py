"""On-device MPC -> QP assembly (impc_mpc_build_values_device) against the oracle
restatement of mpcPlanner's assembly (oracle/mpc_qp_ref.py, mpcPlanner.cpp:891-1197) directly, QP by
QP, and against the host builder (impc_mpc_build_values) for the whole batch.

Dynamic obstacles (yaw 0) and everything outside the obstacle rows are bit-identical; static
obstacles with a yaw go through the device cos/sin and may differ by a few ulp.
"""
import math

import numpy as np
import pytest

import impc
from impc import scenarios
from oracle import mpc_qp_ref

pytestmark = pytest.mark.gpu


def inputs(seed, nb, N, S, K, L, lin=True):
    rng = np.random.default_rng(seed)
    pos = np.stack([np.zeros(nb), rng.uniform(-1, 1, nb), rng.uniform(1.5, 2.5, nb)], axis=1)
    vel = np.stack([rng.uniform(0, 5, nb), rng.uniform(-1, 1, nb), np.zeros(nb)], axis=1)
    xref = np.zeros((nb, N, 8))
    xref[:, :, 0] = pos[:, None, 0] + np.arange(N)[None] * rng.uniform(0.5, 2.5, (nb, 1))
    xref[:, :, 1:3] = pos[:, None, 1:3]
    ls = None
    if lin:
        ls = np.zeros((nb, N, 8))
        ls[:, :, :3] = pos[:, None] + 0.1 * np.arange(N)[None, :, None] * vel[:, None]
    sc = np.stack([pos[:, None, 0] + rng.uniform(2, 20, (nb, S)), rng.uniform(-5, 5, (nb, S)),
                   rng.uniform(0.5, 4.5, (nb, S))], axis=2)
    ss = np.where(rng.uniform(size=(nb, S, 1)) < 0.5, [0.4, 0.4, 4.0], [0.4, 4.0, 0.4])
    sy = rng.uniform(-math.pi, math.pi, (nb, S))
    p0 = np.stack([pos[:, None, 0] + rng.uniform(3, 15, (nb, K)), rng.uniform(-4, 4, (nb, K)),
                   rng.uniform(0.5, 3, (nb, K))], axis=2)
    dp = p0[:, :, None, :] + 0.1 * np.arange(L)[None, None, :, None] * rng.normal(0, 1, (nb, K, 1, 3))
    ds = np.full((nb, K, L, 3), 0.8)
    return pos, vel, xref, ls, sc, ss, sy, dp, ds


def oracle_qp(pd, arrays, i, S, K):
    """QP i of the batch as oracle/mpc_qp_ref.build_qp assembles it."""
    pos, vel, xref, ls, sc, ss, sy, dp, ds = arrays
    static = [(sc[i, j], ss[i, j], sy[i, j]) for j in range(S)] if S else []
    dpos = [list(dp[i, k]) for k in range(K)] if K else []
    dsz = [list(ds[i, k]) for k in range(K)] if K else []
    r = mpc_qp_ref.build_qp(pd, pos[i], vel[i], xref[i], None if ls is None else ls[i], static, dpos, dsz)
    return dict(Px=r["P"][2], q=r["q"], Ax=r["A"][2], l=r["l"], u=r["u"])


def device_build(ctx, p, S, K, L, nb, arrays):
    pos, vel, xref, ls, sc, ss, sy, dp, ds = arrays
    n, m, nnzP, nnzA = impc.mpc_dims(p, S, K)
    dev_in = [impc.DeviceArray(ctx, a) if a is not None and a.size else None
              for a in (pos, vel, xref, ls, sc, ss, sy, dp, ds)]
    outs = [impc.DeviceArray(ctx, (nb, k)) for k in (nnzP, n, nnzA, m, m)]
    bld = impc.MpcBuilder(ctx, p, S, K, L)
    bld.build(nb, *[d.ptr if d is not None else None for d in dev_in], *[o.ptr for o in outs])
    host = [o.get() for o in outs]
    bld.close()
    for d in dev_in:
        if d is not None:
            d.free()
    return host, outs


@pytest.mark.parametrize("S,K,lin", [(0, 8, True), (0, 3, False), (0, 0, False)])
def test_dynamic_obstacles_bit_identical(ctx, S, K, lin):
    N, L, nb = 20, 31, 37
    p, pd = impc.mpc_params(horizon=N)
    arrays = inputs(10 + K, nb, N, S, K, L, lin)
    dev, outs = device_build(ctx, p, S, K, L, nb, arrays)
    for o in outs:
        o.free()
    for i in (0, 1, nb // 2, nb - 1):  # the oracle, QP by QP: bit for bit
        ref = oracle_qp(pd, arrays, i, S, K)
        for name, a in zip(("Px", "q", "Ax", "l", "u"), dev):
            assert np.array_equal(a[i], ref[name]), (i, name)
    pos, vel, xref, ls, sc, ss, sy, dp, ds = arrays
    ref = impc.mpc_values(p, pos, vel, xref, ls, dyn_pos=dp if K else None, dyn_size=ds if K else None)
    for name, a in zip(("Px", "q", "Ax", "l", "u"), dev):
        assert np.array_equal(a, ref[name]), name


def test_static_obstacles_with_yaw_within_ulps(ctx):
    N, S, K, L, nb = 20, 4, 2, 31, 23
    p, pd = impc.mpc_params(horizon=N)
    arrays = inputs(77, nb, N, S, K, L, True)
    dev, outs = device_build(ctx, p, S, K, L, nb, arrays)
    for o in outs:
        o.free()
    for i in (0, nb - 1):  # the oracle, QP by QP: device cos/sin within an ulp-level tolerance
        ref = oracle_qp(pd, arrays, i, S, K)
        for name, a in zip(("Px", "q", "Ax", "l", "u"), dev):
            r = ref[name]
            fin = np.isfinite(r)
            assert np.array_equal(np.isfinite(a[i]), fin) and np.array_equal(a[i][~fin], r[~fin]), (i, name)
            np.testing.assert_allclose(a[i][fin], r[fin], rtol=1e-13, atol=1e-13, err_msg=name)
    pos, vel, xref, ls, sc, ss, sy, dp, ds = arrays
    ref = impc.mpc_values(p, pos, vel, xref, ls, st_centroid=sc, st_size=ss, st_yaw=sy, dyn_pos=dp, dyn_size=ds)
    for name, a in zip(("Px", "q", "Ax", "l", "u"), dev):
        r = ref[name]
        fin = np.isfinite(r)
        assert np.array_equal(np.isfinite(a), fin), name
        assert np.array_equal(a[~fin], r[~fin]), name
        np.testing.assert_allclose(a[fin], r[fin], rtol=1e-13, atol=1e-13, err_msg=name)


def test_device_built_qps_solve_like_host_built(ctx):
    """MPC inputs -> device assembly -> batched solve, against the host-assembled solve."""
    cfg = scenarios.intent_config(instances=16, seed=515)
    s = impc.default_settings(verbose=0, adaptive_rho_interval=25)
    K = 8
    bk = cfg[K]
    inst = bk["instances"]
    rows = bk["inst"]
    nb = rows.size
    p, _ = impc.mpc_params(horizon=20)
    pos = inst["prev"][rows, 0, :3]
    vel = inst["prev"][rows, 0, 3:6]
    arrays = (pos, vel, inst["xref"][rows], inst["prev"][rows], None, None, None, bk["dyn_pos"], bk["dyn_size"])
    dev, outs = device_build(ctx, p, 0, K, bk["dyn_pos"].shape[2], nb, arrays)
    ref = impc.mpc_values(p, pos, vel, inst["xref"][rows], inst["prev"][rows], dyn_pos=bk["dyn_pos"],
                          dyn_size=bk["dyn_size"])
    pat = bk["pattern"]
    results = []
    for use_device in (False, True):
        b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], nb)
        b.set_settings(s)
        if use_device:
            b.set_values_device(*[o.ptr for o in outs])
        else:
            b.set_values(ref["Px"], ref["q"], ref["Ax"], ref["l"], ref["u"])
        b.warm_start(bk["x_ws"], None)
        b.solve()
        results.append(b.get())
        b.close()
    for o in outs:
        o.free()
    assert np.array_equal(results[0][0], results[1][0])
    assert np.array_equal(results[0][2]["iter"], results[1][2]["iter"])
