"""The product MPC -> QP builder (impc_mpc_build_pattern / impc_mpc_build_values, mpc_qp.cpp)
against the pure-Python restatement of mpcPlanner's assembly (oracle/mpc_qp_ref.py,
mpcPlanner.cpp:891-1197): bit-exact P, q, A, l, u, including the reference's quirks (float-rounded
matrix entries, skipped zero Hessian entries, R indexed by the global index, isDyamic
static-index overwrite, prediction clamping to the last point)."""
import math

import numpy as np
import pytest

import impc
from oracle import mpc_qp_ref


def ref_qp(pd, pos, vel, xref, lin, cen, size, yaw, dpos, dsize):
    static = [] if cen is None else [(cen[i], size[i], yaw[i]) for i in range(cen.shape[0])]
    dp = [] if dpos is None else [list(dpos[i]) for i in range(dpos.shape[0])]
    ds = [] if dsize is None else [list(dsize[i]) for i in range(dsize.shape[0])]
    return mpc_qp_ref.build_qp(pd, pos, vel, xref, lin, static, dp, ds)


def case(seed, N=20, S=0, K=0, L=31, lin=True, H=0, **kw):
    rng = np.random.default_rng(seed)
    extra = dict(kw)
    if H:
        extra.update(num_half_space=H, half_max=tuple(rng.uniform(-1, 1, 3)), half_min=tuple(rng.uniform(-1, 1, 3)))
    p, pd = impc.mpc_params(horizon=N, **extra)
    pos = np.array([0.0, rng.uniform(-1, 1), rng.uniform(1.5, 2.5)])
    vel = np.array([rng.uniform(0, 5), rng.uniform(-1, 1), 0.0])
    xref = np.zeros((N, 8))
    xref[:, 0] = pos[0] + np.arange(N) * rng.uniform(0.5, 2.5)
    xref[:, 1:3] = pos[1:3]
    linst = None
    if lin:
        linst = np.zeros((N, 8))
        linst[:, :3] = pos + np.arange(N)[:, None] * 0.1 * vel + rng.normal(0, 0.05, (N, 3))
    cen = size = yaw = None
    if S:
        cen = np.stack([pos[0] + rng.uniform(2, 20, S), rng.uniform(-5, 5, S), rng.uniform(0.5, 4.5, S)], axis=1)
        size = np.where(rng.uniform(size=(S, 1)) < 0.5, [0.4, 0.4, 4.0], [0.4, 4.0, 0.4])
        yaw = rng.uniform(-math.pi, math.pi, S)
    dpos = dsize = None
    if K:
        p0 = np.stack([pos[0] + rng.uniform(3, 15, K), rng.uniform(-4, 4, K), rng.uniform(0.5, 3, K)], axis=1)
        v0 = rng.normal(0, 1, (K, 3))
        t = np.arange(L) * 0.1
        dpos = p0[:, None, :] + t[None, :, None] * v0[:, None, :]
        dsize = np.broadcast_to(np.array([0.8, 0.8, 0.8]) + rng.uniform(0, 0.2, (K, 1, 1)), (K, L, 3)).copy()
    return p, pd, pos, vel, xref, linst, cen, size, yaw, dpos, dsize


def product(p, pos, vel, xref, lin, cen, size, yaw, dpos, dsize):
    S = 0 if cen is None else cen.shape[0]
    K = 0 if dpos is None else dpos.shape[0]
    pat = impc.mpc_pattern(p, S, K)
    b = lambda a: None if a is None else a[None]  # noqa: E731
    vals = impc.mpc_values(p, pos[None], vel[None], xref[None], b(lin), st_centroid=b(cen), st_size=b(size),
                           st_yaw=b(yaw), dyn_pos=b(dpos), dyn_size=b(dsize))
    return pat, {k: v[0] for k, v in vals.items()}


CASES = {
    "first_call_K0": dict(seed=1, lin=False),
    "static_K10": dict(seed=2, S=10),
    "dynamic_K8": dict(seed=3, K=8),
    "dynamic_short_prediction": dict(seed=4, K=3, L=7),          # clamp to .back() (:1165-1184)
    "mixed_static_dynamic_quirk": dict(seed=5, S=2, K=4),        # isDyamic static-index (:1194)
    "horizon_not_multiple_of_5": dict(seed=6, N=18, K=2),       # R index misalignment (:945)
    "horizon_40": dict(seed=7, N=40, K=10),
    "half_spaces": dict(seed=8, H=2, K=1),
    "velocity_weight_nonzero": dict(seed=9, K=1, velocity_weight=3.0),
    "default_ranges": dict(seed=10, S=1, y_range_min=-1e10, y_range_max=1e10),
}


@pytest.mark.parametrize("name", list(CASES))
def test_builder_bit_exact(name):
    p, pd, *inp = case(**CASES[name])
    pat, vals = product(p, *inp)
    ref = ref_qp(pd, *inp)
    assert (pat["n"], pat["m"]) == (ref["n"], ref["m"])
    for k, (rp, ri, rx) in (("P", ref["P"]), ("A", ref["A"])):
        np.testing.assert_array_equal(pat[k + "p"], rp)
        np.testing.assert_array_equal(pat[k + "i"], ri)
        np.testing.assert_array_equal(vals[k + "x"], rx)
    for k in ("q", "l", "u"):
        np.testing.assert_array_equal(np.minimum(np.maximum(vals[k], -1e300), 1e300),
                                      np.minimum(np.maximum(ref[k], -1e300), 1e300))
        np.testing.assert_array_equal(np.isinf(vals[k]), np.isinf(ref[k]))


def test_dimensions_formula():
    """n = 13N - 5, m = 21N - 5 + (H + K) W, nnzA = 38N - 22 + 4 K W (H = 0)."""
    for N, K in ((20, 0), (20, 8), (20, 10), (40, 10), (30, 3)):
        p, _ = impc.mpc_params(horizon=N)
        n, m, nnzP, nnzA = impc.mpc_dims(p, 0, K)
        W = N - 1
        assert n == 13 * N - 5 and m == 21 * N - 5 + K * W and nnzA == 38 * N - 22 + 4 * K * W
        assert nnzP == 10 * N - 5  # zero velocity weight entries skipped (:940-948)


def test_batched_builder_matches_per_instance():
    """A batch of instances equals the per-instance builds (no cross-talk in the batched loop)."""
    rows = [case(seed=20 + i, K=3) for i in range(4)]
    p = rows[0][0]
    stack = lambda j: np.stack([r[j] for r in rows])  # noqa: E731
    vals = impc.mpc_values(p, stack(2), stack(3), stack(4), stack(5), dyn_pos=stack(9), dyn_size=stack(10))
    for i, r in enumerate(rows):
        _, one = product(p, *r[2:])
        for k in one:
            np.testing.assert_array_equal(vals[k][i], one[k])


def test_yawed_static_rows_bit_exact_many_draws():
    """Obstacle-row bounds l = 1 - f(c) + grad f(c) . c of yawed static obstacles over many draws:
    the reference's pow(v, 2) is one correctly rounded multiply in its GCC build (pow(x, 2.0) is
    folded to x * x), which libm's pow misses by an ulp now and then -- the oracle squares as the
    reference binary does (oracle/mpc_qp_ref.py _sq)."""
    for seed in range(40, 80):
        p, pd, *inp = case(seed=seed, S=4, K=2)
        pat, vals = product(p, *inp)
        ref = ref_qp(pd, *inp)
        for name, r in (("l", ref["l"]), ("Ax", ref["A"][2]), ("q", ref["q"])):
            assert np.array_equal(vals[name], r), (seed, name)
