"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of mpcPlanner's intent-hypothesis fan-out
(the oracle for impc_intent_fanout, include/impc_fanout.h).  Only tests/ may import it.

Follows trajectory_planner/include/trajectory_planner/mpcPlanner.cpp statement by statement:
  findClosestObstacle  :663-708  first call / fewer than 2 previous states: nearest current
                                 obstacle position to currPos_ (strict <, first minimum);
                                 otherwise sum over j < size()/3 of exp(-j) * d * (3 - cos(traj -
                                 obs)), every term at currentStatesSol_[0] / [1] as written, with
                                 the early break once the running sum exceeds the minimum
  getIntentComb        :710-769  weights (STOP, LEFT, RIGHT, FORWARD, max(L,F), max(R,F)) of the
                                 closest obstacle, std::sort of (weight, index) pairs, candidate i
                                 = combination weight[5-i].second; each candidate lists the
                                 closest obstacle's intent trajectories first (LEFT+FORWARD /
                                 RIGHT+FORWARD for the two pairs), then every other obstacle in
                                 index order at its maxCoeff intent (first maximum)
Intent indices follow dynamicPredictor's enum (FORWARD, LEFT, RIGHT, STOP = 0..3).
"""
import math

FORWARD, LEFT, RIGHT, STOP = 0, 1, 2, 3
COMB = [[STOP], [LEFT], [RIGHT], [FORWARD], [LEFT, FORWARD], [RIGHT, FORWARD]]  # :731-750


def _norm(a, b, c):
    return math.sqrt((a * a + b * b) + c * c)


def closest_obstacle(curr_pos, first_time, prev_states, dyn_cur):
    """prev_states: the previous plan's states (8-vectors, may be empty); dyn_cur: [K][3]."""
    ob, min_d = -1, math.inf
    if first_time or len(prev_states) < 2:
        for k, o in enumerate(dyn_cur):
            d = _norm(curr_pos[0] - o[0], curr_pos[1] - o[1], curr_pos[2] - o[2])
            if d < min_d:
                min_d, ob = d, k
        return ob
    s, ns = prev_states[0], prev_states[1]
    traj = math.atan2(ns[1] - s[1], ns[0] - s[0])
    for k, o in enumerate(dyn_cur):
        dist = 0.0
        for j in range(len(prev_states) // 3):
            obs = math.atan2(o[1] - s[1], o[0] - s[0])
            w = math.exp(-j)
            d = _norm(s[0] - o[0], s[1] - o[1], s[2] - o[2])
            dist += w * d * (3.0 - math.cos(traj - obs))
            if dist > min_d:
                break
        if dist < min_d:
            min_d, ob = dist, k
    return ob


def intent_comb(ob, prob):
    """prob: [K][4].  Returns (candidate combination types in candidate order, other obstacles'
    (index, intent) list)."""
    p = prob[ob]
    smax = lambda a, b: b if a < b else a  # noqa: E731  std::max
    w = [(p[STOP], 0), (p[LEFT], 1), (p[RIGHT], 2), (p[FORWARD], 3), (smax(p[LEFT], p[FORWARD]), 4),
         (smax(p[RIGHT], p[FORWARD]), 5)]
    w.sort()  # std::sort on std::pair<double, int>
    types = [w[5 - i][1] for i in range(6)]
    others = []
    for k in range(len(prob)):
        if k != ob:
            m = 0
            for q in range(1, 4):
                if prob[k][q] > prob[k][m]:
                    m = q
            others.append((k, m))
    return types, others


def fanout(curr_pos, first_time, prev_states, dyn_cur, pred_pos, pred_size, prob):
    """One instance.  pred_pos / pred_size: [K][4][L][3].  Returns dict(ob_idx, types, cands) with
    cands[c] = (positions [K'][L][3], sizes [K'][L][3]) as nested lists."""
    ob = closest_obstacle(curr_pos, first_time, prev_states, dyn_cur)
    types, others = intent_comb(ob, prob)
    cands = []
    for t in types:
        rows = [(ob, it) for it in COMB[t]] + others
        cands.append(([pred_pos[k][it] for k, it in rows], [pred_size[k][it] for k, it in rows]))
    return dict(ob_idx=ob, types=types, cands=cands)
