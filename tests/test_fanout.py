"""Intent-hypothesis fan-out (findClosestObstacle + getIntentComb, mpcPlanner.cpp:663-769):
known answers of the restatement (oracle/fanout_ref.py) on the CPU, and the device kernels
(impc_intent_fanout) bit-exact against it on the GPU.  The reference holds no tests for these
functions, so the known answers are derived by hand from the cited statements (parity of the
restatement itself is unpinned, as for the rest of the path)."""
import numpy as np
import pytest

from oracle import fanout_ref as fr

F, Lf, R, S = fr.FORWARD, fr.LEFT, fr.RIGHT, fr.STOP


def probs(forward, left, right, stop):
    p = [0.0] * 4
    p[F], p[Lf], p[R], p[S] = forward, left, right, stop
    return p


def test_all_equal_weights_order_by_index_from_the_back():
    # std::sort of equal weights keeps index order; candidates are taken from the back (:753-756)
    types, _ = fr.intent_comb(0, [probs(0.25, 0.25, 0.25, 0.25)])
    assert types == [5, 4, 3, 2, 1, 0]


def test_forward_dominant_order():
    # weights: STOP .05, LEFT .2, RIGHT .05, FORWARD .7, max(L,F) .7, max(R,F) .7
    types, _ = fr.intent_comb(0, [probs(0.7, 0.2, 0.05, 0.05)])
    assert types == [5, 4, 3, 1, 2, 0]


def test_left_dominant_order():
    types, _ = fr.intent_comb(0, [probs(0.1, 0.6, 0.2, 0.1)])
    # STOP .1(0) LEFT .6(1) RIGHT .2(2) FORWARD .1(3) max(L,F) .6(4) max(R,F) .2(5)
    assert types == [4, 1, 5, 2, 3, 0]


def test_other_obstacles_take_first_maximum_intent():
    prob = [probs(0.25, 0.25, 0.25, 0.25), probs(0.1, 0.4, 0.4, 0.1), probs(0.5, 0.1, 0.1, 0.3)]
    _, others = fr.intent_comb(0, prob)
    assert others == [(1, Lf), (2, F)]  # LEFT (index 1) before RIGHT (index 2) on a tie


def test_closest_obstacle_first_call_is_nearest():
    dyn = [[5.0, 0.0, 1.0], [2.0, 1.0, 1.0], [-2.0, -1.0, 1.0]]
    assert fr.closest_obstacle([0.0, 0.0, 1.0], True, [], dyn) == 1  # first of the two at sqrt(5)


def test_closest_obstacle_prefers_the_one_ahead():
    # moving along +x: an obstacle 2 m ahead scores 2 (3 - cos 0) per unit weight, one 2 m behind 4
    prev = [[0, 0, 1] + [0] * 5, [1, 0, 1] + [0] * 5] + [[0] * 8] * 18
    dyn = [[-2.0, 0.0, 1.0], [2.0, 0.0, 1.0]]
    assert fr.closest_obstacle([0.0, 0.0, 1.0], False, prev, dyn) == 1
    # with fewer than 2 previous states it falls back to distance (first of the tie)
    assert fr.closest_obstacle([0.0, 0.0, 1.0], False, prev[:1], dyn) == 0


def test_candidate_contents():
    K, L = 3, 4
    pp = np.arange(K * 4 * L * 3, dtype=float).reshape(K, 4, L, 3)
    ps = pp + 0.5
    prob = [probs(0.1, 0.6, 0.2, 0.1), probs(0.7, 0.1, 0.1, 0.1), probs(0.1, 0.1, 0.1, 0.7)]
    out = fr.fanout([0, 0, 1], True, [], [[1, 0, 1], [5, 0, 1], [6, 0, 1]], pp.tolist(), ps.tolist(), prob)
    assert out["ob_idx"] == 0
    c0 = out["cands"][0]  # type 4: LEFT + FORWARD of obstacle 0, then obstacle 1 FORWARD, 2 STOP
    assert [np.asarray(t).tolist() for t in c0[0]] == [pp[0, Lf].tolist(), pp[0, F].tolist(), pp[1, F].tolist(),
                                                         pp[2, S].tolist()]
    assert len(out["cands"][1][0]) == K  # type 1: LEFT only


def random_instances(rng, I, K, L, P):
    curr = rng.uniform(-3, 3, (I, 3))
    first = (rng.random(I) < 0.25).astype(np.int8)
    pc = rng.choice([0, 1, 2, P, P], I).astype(np.int32)
    prev = rng.uniform(-3, 3, (I, P, 8))
    dyn_cur = rng.uniform(-8, 8, (I, K, 3))
    pred_pos = rng.uniform(-8, 8, (I, K, 4, L, 3))
    pred_size = rng.uniform(0.5, 2.0, (I, K, 4, L, 3))
    prob = rng.dirichlet(np.ones(4), (I, K))
    # exact ties in some instances (equal probabilities / duplicated obstacle positions)
    prob[::7] = 0.25
    if K > 1:
        dyn_cur[::5, 1] = dyn_cur[::5, 0]
    return curr, first, prev, pc, dyn_cur, pred_pos, pred_size, prob


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 3, 8])
def test_device_fanout_matches_restatement(ctx, K):
    import impc
    rng = np.random.default_rng(100 + K)
    I, L, P = 96, 31, 20
    curr, first, prev, pc, dyn_cur, pred_pos, pred_size, prob = random_instances(rng, I, K, L, P)
    out = impc.intent_fanout(ctx, curr, first, prev, pc, dyn_cur, pred_pos, pred_size, prob)
    for i in range(I):
        ref = fr.fanout(curr[i].tolist(), bool(first[i]), prev[i, :pc[i]].tolist(), dyn_cur[i].tolist(),
                        pred_pos[i], pred_size[i], prob[i].tolist())
        assert out["ob_idx"][i] == ref["ob_idx"], i
        assert out["cand_type"][i].tolist() == ref["types"], i
        np.testing.assert_array_equal(out["closest_prob"][i], prob[i, ref["ob_idx"]])
        for c, t in enumerate(ref["types"]):
            s = out["cand_slot"][i, c]
            pos, size = (out["single_pos"][i, s], out["single_size"][i, s]) if s < 4 else \
                (out["pair_pos"][i, s - 4], out["pair_size"][i, s - 4])
            np.testing.assert_array_equal(pos, np.asarray(ref["cands"][c][0]))
            np.testing.assert_array_equal(size, np.asarray(ref["cands"][c][1]))
            assert (s >= 4) == (t >= 4)
