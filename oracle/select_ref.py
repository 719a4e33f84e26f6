"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of mpcPlanner's candidate scoring and
selection (the oracle for impc_select_best, include/impc_select.h).  Only tests/ may import it.

Follows trajectory_planner/include/trajectory_planner/mpcPlanner.cpp statement by statement:
  getTrajectoryScore   :771-778
  getConsistencyScore  :780-800   (first call / empty previous plan -> 0; 10 steps; floor 0.1)
  getDetourScore       :802-814   (floor 0.1)
  getSafetyScore       :816-848   (planar distances; dynamic obstacles use the FULL size in
                                   maxSize, static ones half of it -- as written in the reference)
  evaluateTraj         :850-887   (mean-normalised scores; the weight of candidate i is the i-th
                                   entry of (STOP, LEFT, RIGHT, FORWARD, max(L,F), max(R,F)) of the
                                   closest obstacle's intent probabilities, indexed by the
                                   candidate's position -- intentType.push_back(i), :617;
                                   first maximum wins, Eigen maxCoeff)
Intent indices follow dynamicPredictor's enum (FORWARD, LEFT, RIGHT, STOP = 0..3).
"""
import math

FORWARD, LEFT, RIGHT, STOP = 0, 1, 2, 3
NUM_CONSISTENCY_STEP = 10  # :781



def _sq(v):
    """pow(v, 2) of the reference C++: GCC folds pow(x, 2.0) to x * x at every optimisation level
    (no -ffast-math needed), so the reference binary squares by one correctly rounded multiply --
    libm's pow (math.pow) can differ from it by an ulp."""
    return v * v

def consistency_score(states, prev_states, first_time):
    """states, prev_states: lists of 8-vectors (prev may be empty)."""
    if first_time or len(prev_states) == 0 or len(states) == 0:
        return 0.0
    max_step = min(NUM_CONSISTENCY_STEP, min(len(prev_states), len(states)))
    if max_step == 0:
        return 0.0
    total = 0.0
    for i in range(max_step):
        dx = prev_states[i][0] - states[i][0]
        dy = prev_states[i][1] - states[i][1]
        dz = prev_states[i][2] - states[i][2]
        total += math.sqrt(dx * dx + dy * dy + dz * dz)
    total /= max_step
    return max(total, 0.1)


def detour_score(states, ref):
    total = 0.0
    for i in range(len(states)):
        dx = ref[i][0] - states[i][0]
        dy = ref[i][1] - states[i][1]
        dz = ref[i][2] - states[i][2]
        total += math.sqrt(dx * dx + dy * dy + dz * dz)
    total /= len(states)
    return max(total, 0.1)


def safety_score(states, static_obs, dyn_pos, dyn_size, dyn_safety, static_safety):
    """static_obs: list of (centroid[3], size[3]); dyn_pos/dyn_size: per obstacle, per step."""
    c = math.atanh(0.5)
    total = 0.0
    for i in range(len(states)):
        dist = 0.0
        total_w = 0.0
        px, py = states[i][0], states[i][1]
        for j in range(len(dyn_pos)):
            ox, oy = dyn_pos[j][i][0], dyn_pos[j][i][1]
            max_size = math.sqrt(_sq(dyn_size[j][i][0]) + _sq(dyn_size[j][i][1]))
            d = math.sqrt((px - ox) ** 2 + (py - oy) ** 2)
            w = 1 - math.tanh(c / (dyn_safety + max_size) * d)
            dist += d * w
            total_w += w
        for cen, size in static_obs:
            max_size = math.sqrt(_sq(size[0] / 2) + _sq(size[1] / 2))
            d = math.sqrt((px - cen[0]) ** 2 + (py - cen[1]) ** 2)
            w = 1 - math.tanh(c / (static_safety + max_size) * d)
            dist += d * w
            total_w += w
        dist = fdiv(dist, total_w)
        total += dist
    return total / len(states)


def fdiv(a, b):
    """IEEE double division (C++ semantics: x/0 -> +-inf, 0/0 -> nan)."""
    if b == 0:
        if a == 0 or math.isnan(a):
            return float("nan")
        return math.copysign(float("inf"), a) * math.copysign(1.0, b)
    return a / b


def evaluate(scores, intent_type, prob):
    """scores: [(consistency, detour, safety)] of the successful candidates; intent_type: their
    candidate indices; prob: closest obstacle's intent probabilities (FORWARD, LEFT, RIGHT, STOP).
    Returns (best position among the successful candidates, weighted scores)."""
    n = len(scores)
    ca = sum(s[0] for s in scores) / n
    da = sum(s[1] for s in scores) / n
    sa = sum(s[2] for s in scores) / n
    weight = [prob[STOP], prob[LEFT], prob[RIGHT], prob[FORWARD], max(prob[LEFT], prob[FORWARD]),
              max(prob[RIGHT], prob[FORWARD])]
    weighted = []
    for i in range(n):
        c = fdiv(ca, scores[i][0])
        d = fdiv(da, scores[i][1])
        s = fdiv(scores[i][2], sa)
        weighted.append(weight[intent_type[i]] * (1.0 * c + 1.0 * d + 1.0 * s))
    best = 0
    for i in range(1, n):
        if weighted[i] > weighted[best]:
            best = i
    return best, weighted


def select_instance(cand_states, valid, prev_states, first_time, ref, static_obs, cand_dyn_pos, cand_dyn_size,
                    prob, dyn_safety, static_safety):
    """One makePlanWithPred selection (:606-634).  Returns (best candidate index or -1,
    best position among valid candidates, raw scores [C][3] (None for invalid), weighted)."""
    scores, types = [], []
    raw = []
    for c in range(len(cand_states)):
        if not valid[c]:
            raw.append(None)
            continue
        st = cand_states[c]
        sc = (consistency_score(st, prev_states, first_time), detour_score(st, ref),
              safety_score(st, static_obs, cand_dyn_pos[c], cand_dyn_size[c], dyn_safety, static_safety))
        raw.append(sc)
        scores.append(sc)
        types.append(c)
    if not scores:
        return -1, -1, raw, []
    pos, weighted = evaluate(scores, types, prob)
    return types[pos], pos, raw, weighted
