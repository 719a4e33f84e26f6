"""The bench workload's tail (bench.py default: BASELINE.json configs[2], 65,536 QPs, seed 3000):
every QP the oracle does not end SOLVED or runs to the 4000-iteration cap -- solved inaccurate,
max-iter, primal infeasible (inaccurate or not) -- checked on the GPU exactly as bench.py launches
the workload (shared-structure values, warm start, one grouped longest-first launch over both
pattern buckets), against the oracle solving the same QPs.  The tail set itself comes from the
committed fixture tests/golden/tail_seed3000.npz (tests/golden/make_tail_seed3000.py: the oracle
over all 65,536 QPs); parity unpinned against the real libosqp."""
import os

import numpy as np
import pytest

import impc
from impc import scenarios

from helpers import compare, oracle

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tail_seed3000.npz")


def subset(bk, idx):
    out = dict(bk, values={k: v[idx] for k, v in bk["values"].items()})
    out["x_ws"] = bk["x_ws"][idx]
    return out


@pytest.fixture(scope="module")
def workload():
    return scenarios.intent_config(N=20, K=8, instances=8192, hyps=8, seed=3000)


def test_fixture_matches_oracle(workload):
    """CPU: the first tail QPs of each bucket re-solved by the oracle give the fixture's status and
    iteration count (the fixture is the oracle's, not a hand-edited list)."""
    fx = np.load(FIX)
    s = impc.default_settings(verbose=0)
    for K, bk in sorted(workload.items()):
        idx = fx[f"K{K}_index"][:6]
        _, _, io = oracle(subset(bk, idx), s)
        assert np.array_equal(io["status_val"], fx[f"K{K}_status"][:6])
        assert np.array_equal(io["iter"], fx[f"K{K}_iter"][:6])


@pytest.mark.gpu
def test_tail_qps_on_gpu(ctx, workload):
    fx = np.load(FIX)
    s = impc.default_settings(verbose=0)
    bks = [bk for _, bk in sorted(workload.items())]
    qw = scenarios.queue_weight(bks[0]["params"], bks[0]["N"])
    batches = []
    try:
        for bk in bks:
            pat, v = bk["pattern"], bk["values"]
            b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], v["q"].shape[0])
            batches.append(b)
            b.set_settings(s)
            Px0, Ax0, var, Axv = impc.shared_split(v["Px"], v["Ax"])
            b.set_values_shared(Px0, Ax0, var, Axv, v["q"], v["l"], v["u"])
            b.warm_start(bk["x_ws"], None)
            b.set_queue_order(impc.QUEUE_LONGEST_FIRST, qw)
        impc.solve_group(batches)
        for bk, b in zip(bks, batches):
            K = bk["K"]
            x, y, info = b.get()
            assert info.size == int(fx[f"K{K}_count"])
            st, it = info["status_val"], info["iter"]
            # the GPU's tail is the oracle's tail, with the same statuses and iteration counts
            tail = np.nonzero((st != 1) | (it == 4000))[0]
            assert np.array_equal(tail, fx[f"K{K}_index"]), (K, len(tail), len(fx[f"K{K}_index"]))
            assert np.array_equal(st[tail], fx[f"K{K}_status"])
            assert np.array_equal(it[tail], fx[f"K{K}_iter"])
            ref = oracle(subset(bk, tail), s)
            compare((x[tail], y[tail], info[tail]), ref)
    finally:
        for b in batches:
            b.close()
