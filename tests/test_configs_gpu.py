"""BASELINE.json configs[3] and configs[4] shapes through their production launch paths, every QP
checked against the oracle (identical status and iteration count, primal / dual / objective within
1e-5 relative -- helpers.compare, the north_star bar).

  config 4: mixed obstacle counts K = 0..20 (+ the K+1 two-intent variants, i.e. every bucket of
            bench.py --workload config4) in ONE grouped persistent launch (impc_batch_solve_group)
  config 5: N = 40, K = 10 (+1) on the long-horizon team shape (three variables per lane), as a
            receding window on a persistent workspace: setup + solve -> update_lin_cost (shifted
            xRef) -> solve -> update_bounds (next x0) -> solve, against the oracle's persistent
            OSQP workspace driven through the same osqp_update_* calls
"""
import numpy as np
import pytest

import impc
from helpers import compare, oracle
from impc import scenarios
from oracle import osqp_oracle as ora

pytestmark = pytest.mark.gpu


def _batch(ctx, bk, s, shared=False):
    pat, v = bk["pattern"], bk["values"]
    B = v["q"].shape[0]
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    b.set_settings(s)
    split = impc.shared_split(v["Px"], v["Ax"]) if shared else None
    if split is None:
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
    else:
        b.set_values_shared(split[0], split[1], split[2], split[3], v["q"], v["l"], v["u"])
    if bk.get("x_ws") is not None:
        b.warm_start(bk["x_ws"], np.zeros((B, pat["m"])))
    return b


@pytest.mark.parametrize("shared", [False, True], ids=["full-values", "shared-values"])
def test_config4_all_buckets_one_grouped_launch(ctx, shared):
    K = np.arange(21)                                    # one instance per obstacle count 0..20
    bks = scenarios.config4_rank(0, K.size, K, seed=4400)
    ks = sorted({bk["K"] for bk in bks})
    assert ks == list(range(22))                         # 0..20 plus the K+1 = 21 two-intent bucket
    s = impc.default_settings(verbose=0)
    batches = [_batch(ctx, bk, s, shared) for bk in bks]
    try:
        assert all(b.stats()["kernel"] == impc.KERNEL_STRUCTURED for b in batches)
        impc.solve_group(batches)
        res = [b.get() for b in batches]
    finally:
        for b in batches:
            b.close()
    worst = 0.0
    for bk, r in zip(bks, res):
        worst = max(worst, compare(r, oracle(bk, s)))
    assert worst <= 1e-5


def test_config5_receding_window_persistent(ctx):
    cfg = scenarios.intent_config(N=40, K=10, instances=3, hyps=8, seed=5100)
    s = impc.default_settings(verbose=0)
    os_ = ora.settings_from(s)
    for kk, bk in sorted(cfg.items()):
        pat, v = bk["pattern"], bk["values"]
        B = v["q"].shape[0]
        v2 = scenarios.receding_update(bk, shift=1)
        v3 = scenarios.receding_update(bk, shift=2)
        # legal osqp_update_* steps: P and A unchanged (same linearisation points)
        assert np.array_equal(v2["Px"], v["Px"]) and np.array_equal(v2["Ax"], v["Ax"])
        assert np.array_equal(v3["Px"], v["Px"]) and np.array_equal(v3["Ax"], v["Ax"])
        b = _batch(ctx, bk, s)
        try:
            assert b.stats()["kernel"] == impc.KERNEL_STRUCTURED and pat["n"] == 515
            b.set_persistent(True)
            b.solve()
            r1 = b.get()
            b.update_lin_cost(v2["q"])       # replan t+1: shifted reference
            b.solve()
            r2 = b.get()
            b.update_bounds(v3["l"], v3["u"])  # replan t+2: the next initial state
            b.solve()
            r3 = b.get()
        finally:
            b.close()
        for i in range(B):
            w = ora.Workspace(pat, v["Px"][i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], os_)
            w.warm_start(bk["x_ws"][i], np.zeros(pat["m"]))
            refs = [w.solve()]
            w.update_lin_cost(v2["q"][i])
            refs.append(w.solve())
            w.update_bounds(v3["l"][i], v3["u"][i])
            refs.append(w.solve())
            w.close()
            for r, ref in zip((r1, r2, r3), refs):
                one = (r[0][i:i + 1], r[1][i:i + 1], r[2][i:i + 1])
                compare(one, (ref[0][None], ref[1][None], np.array([ref[2]], dtype=ref[2].dtype)))


def test_config5_device_updates_equal_host_updates(ctx):
    """bench.py --workload config5's step: the receding values built on the device and applied by
    impc_batch_update_*_device give bit for bit the solves of the host-array updates."""
    cfg = scenarios.intent_config(N=40, K=10, instances=2, hyps=8, seed=5200)
    s = impc.default_settings(verbose=0)
    for kk, bk in sorted(cfg.items()):
        v = bk["values"]
        v2 = scenarios.receding_update(bk, shift=1)
        res = []
        for dev in (False, True):
            b = _batch(ctx, bk, s)
            keep = []
            try:
                b.set_persistent(True)
                b.solve()
                if dev:
                    keep = [impc.DeviceArray(ctx, np.ascontiguousarray(v2[k])) for k in ("q", "l", "u")]
                    b.update_lin_cost_device(keep[0].ptr)
                    b.update_bounds_device(keep[1].ptr, keep[2].ptr)
                else:
                    b.update_lin_cost(v2["q"])
                    b.update_bounds(v2["l"], v2["u"])
                b.solve()
                res.append(b.get())
            finally:
                b.close()
                for d in keep:
                    d.free()
        np.testing.assert_array_equal(res[0][0], res[1][0])
        np.testing.assert_array_equal(res[0][2]["iter"], res[1][2]["iter"])
        assert np.array_equal(v2["Px"], v["Px"])


def test_groups_on_two_caller_streams(ctx):
    """Two grouped launches on two caller streams, the second replacing the context's group-entry
    table while the first may still run (impc_qp.h: caller streams are ordered against every
    rewrite): both give the bitwise results of the same groups solved one after the other."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so.7")  # the HIP runtime libimpc_qp.so is linked against (already loaded)
    s = impc.default_settings(verbose=0)
    g1 = list(scenarios.intent_config(N=20, K=3, instances=40, hyps=8, seed=901).values())
    g2 = list(scenarios.intent_config(N=20, K=6, instances=40, hyps=8, seed=902).values())
    ref = []
    for g in (g1, g2):
        bs = [_batch(ctx, bk, s) for bk in g]
        impc.solve_group(bs)
        ref.append([b.get() for b in bs])
        for b in bs:
            b.close()
    b1 = [_batch(ctx, bk, s) for bk in g1]
    b2 = [_batch(ctx, bk, s) for bk in g2]
    st1, st2 = C.c_void_p(), C.c_void_p()
    assert hip.hipStreamCreate(C.byref(st1)) == 0 and hip.hipStreamCreate(C.byref(st2)) == 0
    try:
        for _ in range(3):
            impc.solve_group(b1, stream=st1.value)
            impc.solve_group(b2, stream=st2.value)
        out = [[b.get() for b in b1], [b.get() for b in b2]]
    finally:
        for b in b1 + b2:
            b.close()
        hip.hipStreamDestroy(st1)
        hip.hipStreamDestroy(st2)
    for got, exp in zip(out, ref):
        for (x, y, i), (xr, yr, ir) in zip(got, exp):
            assert np.array_equal(x, xr) and np.array_equal(y, yr)
            assert np.array_equal(i["iter"], ir["iter"]) and np.array_equal(i["status_val"], ir["status_val"])


def test_comm_single_rank_gather_and_timer(ctx):
    """impc_comm (RCCL) on one rank: the packed, padded cost-record gather returns this rank's
    impc_info records bit for bit, and the step timer brackets a launch."""
    from impc import distributed as D
    s = impc.default_settings(verbose=0)
    g = list(scenarios.intent_config(N=20, K=2, instances=8, hyps=8, seed=903).values())
    bs = [_batch(ctx, bk, s) for bk in g]
    comm = D.make_comm(None, ctx)
    total = sum(b.B for b in bs)
    recv = impc.DeviceArray(ctx, (total + 5,), impc.INFO_DTYPE)
    try:
        ctx.timer_mark()
        impc.solve_group(bs)
        ctx.timer_mark()
        comm.gather_info(bs, total + 5, recv.ptr)
        ms = ctx.timer_read()
        got = recv.get()
        mine = np.concatenate([b.get()[2] for b in bs])
        assert ms.size == 1 and ms[0] > 0
        assert got[:total].tobytes() == mine.tobytes()
        assert not got[total:].tobytes().strip(b"\0")           # zero padding
        assert comm.max(3.5) == 3.5
    finally:
        recv.free()
        comm.close()
        for b in bs:
            b.close()
