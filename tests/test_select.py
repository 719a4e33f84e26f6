"""Candidate scoring and selection (include/impc_select.h) against the restatement of
mpcPlanner's getTrajectoryScore / evaluateTraj (oracle/select_ref.py, mpcPlanner.cpp:771-887).

Parity unpinned against the reference binary (no tests or fixtures for this path exist in the
reference); the CPU tests pin the restatement to the reference's written semantics on
hand-checkable cases, the GPU test compares the device kernels with it on solved QPs.
"""
import math

import numpy as np
import pytest

import impc
from impc import scenarios
from oracle import select_ref as ref

SAFE = dict(dynamic_safety_dist=1.5, static_safety_dist=0.8)


def line(N, y=0.0, step=1.0):
    return [[k * step, y, 2.0, 0, 0, 0, 0, 0] for k in range(N)]


def test_consistency_score_first_time_and_floor():
    st = line(20)
    assert ref.consistency_score(st, line(20), first_time=True) == 0.0
    assert ref.consistency_score(st, [], first_time=False) == 0.0
    assert ref.consistency_score(st, line(20), first_time=False) == 0.1  # identical -> floor 0.1
    # 10 steps only (:781): a deviation at step 12 does not count
    prev = line(20)
    prev[12] = [99.0] * 8
    assert ref.consistency_score(st, prev, first_time=False) == 0.1


def test_detour_score_mean_distance():
    st = line(10, y=0.0)
    assert math.isclose(ref.detour_score(st, line(10, y=2.0)), 2.0)


def test_safety_dynamic_uses_full_size_static_half():
    st = line(1)
    # one obstacle 3 m away: weight = 1 - tanh(atanh(.5) / (safety + maxSize) * d)
    d = 3.0
    dyn = ref.safety_score(st, [], [[[d, 0.0, 2.0]]], [[[0.8, 0.8, 0.8]]], 1.5, 0.8)
    sta = ref.safety_score(st, [([d, 0.0, 2.0], [0.8, 0.8, 0.8])], [], [], 1.5, 0.8)
    assert math.isclose(dyn, d, rel_tol=1e-15) and math.isclose(sta, d, rel_tol=1e-15)  # single obstacle: d itself
    two = ref.safety_score(st, [([1.0, 0.0, 0.0], [0.8, 0.8, 0.8])], [[[d, 0.0, 2.0]]], [[[0.8, 0.8, 0.8]]], 1.5, 0.8)
    c = math.atanh(0.5)
    wd = 1 - math.tanh(c / (1.5 + math.sqrt(0.64 + 0.64)) * d)        # full size (dynamic)
    ws = 1 - math.tanh(c / (0.8 + math.sqrt(0.16 + 0.16)) * 1.0)      # half size (static)
    assert math.isclose(two, (d * wd + 1.0 * ws) / (wd + ws), rel_tol=1e-15)


def test_safety_nan_when_every_weight_underflows():
    st = line(1)
    assert math.isnan(ref.safety_score(st, [], [[[1e6, 0.0, 0.0]]], [[[0.8, 0.8, 0.8]]], 1.5, 0.8))


def test_evaluate_weights_by_candidate_position_and_first_max():
    prob = [0.1, 0.2, 0.3, 0.4]  # FORWARD, LEFT, RIGHT, STOP
    scores = [(1.0, 1.0, 1.0)] * 6
    best, w = ref.evaluate(scores, list(range(6)), prob)
    # equal scores: weighted = weight(i) * 3 with weight = (STOP, LEFT, RIGHT, FORWARD, max(L,F), max(R,F))
    assert np.allclose(w, 3 * np.array([0.4, 0.2, 0.3, 0.1, 0.2, 0.3]))
    assert best == 0
    # ties keep the first maximum (Eigen maxCoeff)
    best, _ = ref.evaluate([(1.0, 1.0, 1.0)] * 2, [4, 5], [0.5, 0.5, 0.5, 0.0])
    assert best == 0


def selection_inputs(buckets, x_by_bucket, ptr_by_bucket, C=6):
    """impc.scenarios.selection_arrays plus the candidates' state trajectories on the host."""
    d = scenarios.selection_arrays(buckets, ptr_by_bucket, C)
    N = d["N"]
    states = [[None] * C for _ in range(d["I"])]
    for K, (inst, hyp, rows) in d["rows"].items():
        for i, h, r in zip(inst, hyp, rows):
            states[i][h] = x_by_bucket[K][r, :8 * N].reshape(N, 8)
    d["states"] = states
    return d


def test_selection_arrays_layout():
    """Every instance gets its 6 candidates, each pointing at its own bucket row."""
    buckets = scenarios.intent_config(instances=5, seed=99)
    ptrs = {K: 1 << 40 for K in buckets}
    d = scenarios.selection_arrays(buckets, ptrs)
    assert d["x_ptrs"].shape == (5 * 6,) and np.all(d["x_ptrs"] >= (1 << 40))
    assert set(np.unique(d["dyn_count"])) <= set(buckets)
    for K, bk in buckets.items():
        i, h, r = d["rows"][K]
        n = bk["pattern"]["n"]
        assert np.all(d["x_ptrs"][i * 6 + h] == (1 << 40) + r * n * 8)
        assert np.array_equal(d["dyn_pos"][i, h, :K], bk["dyn_pos"][r])


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["all_valid", "some_invalid_first_time_static"])
def test_device_selection_matches_restatement(ctx, variant):
    buckets = scenarios.intent_config(instances=24, seed=4242)
    s = impc.default_settings(verbose=0, adaptive_rho_interval=25)
    batches, xs, ptrs = [], {}, {}
    for K, bk in buckets.items():
        pat, v = bk["pattern"], bk["values"]
        B = v["q"].shape[0]
        b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
        b.set_settings(s)
        b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.warm_start(bk["x_ws"], None)
        b.solve()
        xs[K] = b.get()[0]
        ptrs[K] = b.device_results()[0]
        batches.append(b)
    d = selection_inputs(buckets, xs, ptrs)
    I, C, N = d["I"], d["C"], d["N"]
    rng = np.random.default_rng(7)
    valid = np.ones((I, C), np.int8)
    first = np.zeros(I, np.int8)
    S = 0
    st_c = np.zeros((I, 0, 3))
    st_s = np.zeros((I, 0, 3))
    if variant != "all_valid":
        valid = (rng.uniform(size=(I, C)) > 0.3).astype(np.int8)
        valid[0] = 0  # an instance without any successful candidate
        first[1] = 1
        S = 2
        st_c = np.stack([d["prev"][:, 5, 0:1] + rng.uniform(2, 10, (I, S)), rng.uniform(-4, 4, (I, S)),
                         rng.uniform(1, 3, (I, S))], axis=2)
        st_s = np.broadcast_to([0.4, 4.0, 0.4], (I, S, 3)).copy()
    params = dict(horizon=N, num_candidates=C, max_dynamic=d["kmax"], pred_len=d["L"], num_static=S, prev_len=N, **SAFE)
    out = impc.select_best(ctx, params, d["x_ptrs"], valid, first, d["prev"], np.full(I, N, np.int32), d["xref"],
                           st_c, st_s, d["dyn_count"], d["dyn_pos"], d["dyn_size"], d["prob"])
    for b in batches:
        b.close()
    for i in range(I):
        cand_pos = [d["dyn_pos"][i, c, :d["dyn_count"][i, c]] for c in range(C)]
        cand_size = [d["dyn_size"][i, c, :d["dyn_count"][i, c]] for c in range(C)]
        static = [(st_c[i, j], st_s[i, j]) for j in range(S)]
        best, pos, raw, weighted = ref.select_instance(d["states"][i], valid[i], d["prev"][i], bool(first[i]),
                                                       d["xref"][i], static, cand_pos, cand_size, d["prob"][i],
                                                       SAFE["dynamic_safety_dist"], SAFE["static_safety_dist"])
        assert out["best_cand"][i] == best and out["best_pos"][i] == pos, (i, out["best_cand"][i], best)
        for c in range(C):
            if raw[c] is None:
                assert np.all(np.isnan(out["scores"][i, c])) and np.isnan(out["weighted"][i, c])
            else:
                np.testing.assert_allclose(out["scores"][i, c], raw[c], rtol=1e-12, atol=0)
        np.testing.assert_allclose(out["weighted"][i][valid[i] == 1], weighted, rtol=1e-12, equal_nan=True)
