"""The NON_CVX candidates of the live loop at scale, pinned.

tools/trace_noncvx.py ran the loop of tools/live_loop.py (8,192 vehicles on the reference's
benchmark path, N = 30, K = 4, 30 chained replans) on MI355X and dumped every QP that ended NON_CVX
(42: all six candidates of one vehicle in each of replans 19, 22, 23, 24, 27, 28, 29); the oracle
and the device agreed on every one (status and iteration count, tools/noncvx_fixture.py).
tests/golden/noncvx_live.npz keeps six of them -- a single-intent (K = 4) and a two-intent (K = 5)
candidate of three vehicles -- with the warm start each was solved from.

The cause: each of those vehicles had committed a plan whose states are ~1e18-1e19 (a
diverged candidate's iterate, valid for the reference because solveTraj reports success whenever
osqp_solve returns, mpcPlanner.cpp:513-518); the next replan warm-starts from it and linearises its
obstacle rows around it (castMPCToQPConstraintMatrix :1042-1051), the ADMM residuals reach 1e30 by
the first check (iteration 25) and OSQP 0.6.2 reports NON_CVX -- the solver does what the
reference's does, the scenario is what degenerates.
"""
import os

import numpy as np
import pytest

import impc

from helpers import ROOT, compare, emulate, gpu, oracle

FIX = os.path.join(ROOT, "tests", "golden", "noncvx_live.npz")


def _configs():
    d = np.load(FIX)
    N = int(d["N"])
    p, _ = impc.mpc_params(horizon=N)
    out = {}
    for j in range(d["K"].shape[0]):
        K = int(d["K"][j])
        c = out.setdefault(K, dict(pattern=impc.mpc_pattern(p, 0, K), values={k: [] for k in ("Px", "q", "Ax", "l", "u")},
                                   x_ws=[], rec=[]))
        for k in c["values"]:
            c["values"][k].append(d[f"{k}_{j}"])
        c["x_ws"].append(d[f"x_ws_{j}"])
        c["rec"].append(dict(status=int(d["status"][j]), iter=int(d["iter"][j]), oracle_status=int(d["oracle_status"][j]),
                             oracle_iter=int(d["oracle_iter"][j])))
    for c in out.values():
        c["values"] = {k: np.array(v) for k, v in c["values"].items()}
        c["x_ws"] = np.array(c["x_ws"])
    return out


SETTINGS = dict(verbose=0)


def test_fixture_is_the_degenerate_warm_start_case():
    """Every kept QP starts from a plan of magnitude > 1e17 and ended NON_CVX at iteration 25 on
    the device and in the oracle."""
    for K, c in _configs().items():
        assert np.abs(c["x_ws"]).max(axis=1).min() > 1e17
        for r in c["rec"]:
            assert r["status"] == r["oracle_status"] == impc.NON_CVX
            assert r["iter"] == r["oracle_iter"] == 25


@pytest.mark.parametrize("K", [4, 5])
def test_oracle_reproduces_the_trace(K):
    c = _configs()[K]
    s = impc.default_settings(**SETTINGS)
    _, _, info = oracle(c, s)
    assert info["status_val"].tolist() == [r["oracle_status"] for r in c["rec"]]
    assert info["iter"].tolist() == [r["oracle_iter"] for r in c["rec"]]
    assert (info["setup_exitflag"] == 0).all()  # the factorisation succeeded: the residual test decided


@pytest.mark.parametrize("K", [4, 5])
def test_structured_emulation_matches_oracle(K):
    c = _configs()[K]
    s = impc.default_settings(**SETTINGS)
    compare(emulate(c, s), oracle(c, s))


@pytest.mark.gpu
@pytest.mark.parametrize("K", [4, 5])
def test_device_matches_oracle_and_trace(K):
    c = _configs()[K]
    s = impc.default_settings(**SETTINGS)
    ctx = impc.Context(0)
    try:
        res = gpu(ctx, c, s)
    finally:
        ctx.close()
    compare(res, oracle(c, s))
    assert res[2]["status_val"].tolist() == [r["status"] for r in c["rec"]]
    assert res[2]["iter"].tolist() == [r["iter"] for r in c["rec"]]
