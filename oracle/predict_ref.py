"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of dynamic_predictor's intent
probabilities (the oracle for impc_intent_prob, include/impc_predict.h).  Only tests/ may import it.

Follows dynamic_predictor/include/dynamic_predictor/dynamicPredictor.cpp statement by statement:
  initParam (intent part)  :66-115   paraml = paramr = (1 - maxFrontProb) / (3 maxFrontProb - 1),
                                     frontAngle deg -> rad, paramf = sqrt(fa^2 / (-2 log(paraml
                                     (1 + sin fa) - paraml))), params = atanh(0.5) / stopVel
  intentProb               :197-223  uniform start, one transition per history step, oldest first;
                                     the reference's last step (j = numHist - 1) reads entry -1 of the
                                     history (undefined behaviour) and is not taken
  genTransitionMatrix      :227-255  theta wrapped to (-pi, pi]; column i scaled by pscale at i
  genTransitionVector      :257-281
Intent indices: FORWARD, LEFT, RIGHT, STOP = 0..3.  pow(x, 2) is x * x (glibc's pow is correctly
rounded, so the two agree); the matrix-vector product accumulates columns in order.
"""
import math

FORWARD, LEFT, RIGHT, STOP = 0, 1, 2, 3


def params_from_config(max_front_prob, front_angle_deg, stop_velocity, prob_scale):
    paraml = paramr = (1 - max_front_prob) / (3 * max_front_prob - 1)
    fa = front_angle_deg * math.pi / 180
    paramf = math.sqrt(fa * fa / (-2 * math.log(paraml * (1 + math.sin(fa)) - paraml)))
    return dict(paramf=paramf, paraml=paraml, paramr=paramr, params=math.atanh(0.5) / stop_velocity,
                pscale=prob_scale)


def transition_vector(p, theta, r, si):
    s = [1.0] * 4
    s[si] = p["pscale"]
    tf = theta / p["paramf"]
    pf = s[0] * (math.exp(-0.5 * (tf * tf)) + p["paraml"])
    pl = s[1] * (p["paraml"] * (1 + math.sin(theta)))
    pr = s[2] * (p["paramr"] * (1 - math.sin(theta)))
    ps = 1 - math.tanh(p["params"] / s[3] * r)
    sm = pr + pl + pf
    pr = (1 - ps) * pr / sm
    pl = (1 - ps) * pl / sm
    pf = (1 - ps) * pf / sm
    out = [0.0] * 4
    out[FORWARD], out[LEFT], out[RIGHT], out[STOP] = pf, pl, pr, ps
    return out


def intent_prob(p, pos_hist, vel_hist):
    """pos_hist / vel_hist: lists of 3-vectors, entry 0 the newest.  Returns [4]."""
    P = [0.25] * 4
    nh = len(pos_hist)
    # j = nh - 1 would read history entry -1 (the reference's loop bound, :206, indexes
    # posHist_[i][numHist - j - 2] = [-1] there: out of bounds, undefined behaviour); stop before it
    for j in range(2, nh - 1):
        prev_pos, curr_pos, pp = pos_hist[nh - j - 1], pos_hist[nh - j - 2], pos_hist[nh - j]
        curr_vel = vel_hist[nh - j - 2]
        prev_angle = math.atan2(prev_pos[1] - pp[1], prev_pos[0] - pp[0])
        curr_angle = math.atan2(curr_pos[1] - prev_pos[1], curr_pos[0] - prev_pos[0])
        theta = curr_angle - prev_angle
        if theta > math.pi:
            theta = theta - 2 * math.pi
        elif theta <= -math.pi:
            theta = theta + 2 * math.pi
        r = math.sqrt(curr_vel[0] * curr_vel[0] + curr_vel[1] * curr_vel[1])
        T = [transition_vector(p, theta, r, i) for i in range(4)]  # columns
        nP = []
        for row in range(4):
            acc = 0.0
            for c in range(4):
                acc += T[c][row] * P[c]
            nP.append(acc)
        P = nP
    return P


# ---------------------------------------------------------------- trajectory prediction (predTraj)
# dynamicPredictor.cpp:283-566 with the occupancy map of map_manager (occupancyMap.h:218-269:
# posToIndex = floor((p - mapSizeMin) / res), outside [0, mapVoxelMax) counts as occupied,
# address = x * max_y * max_z + y * max_z + z).  Eigen's 4x4 state update is x + dt vx (the
# multiplications by the model's 0 / 1 entries are exact).

def occupied(m, occ, p):
    idx = [math.floor((p[a] - m["origin"][a]) / m["res"]) for a in range(3)]
    d = m["dims"]
    if not all(0 <= idx[a] < d[a] for a in range(3)):
        return True
    return occ[(idx[0] * d[1] + idx[1]) * d[2] + idx[2]] != 0


def _stop_sizes(tp, vel, size):
    v = math.sqrt(vel[0] * vel[0] + vel[1] * vel[1])
    s = list(size)
    out = []
    for _ in range(tp["num_pred"] + 1):
        out.append(list(s))
        g = 2 * min(v, tp["stop_vel"]) * tp["dt"]
        s[0] += g
        s[1] += g
    return out


def model_forward(tp, m, occ, pos, vel):
    """:351-396 -- for each angle, velocities ascend until the first colliding sample."""
    dt, P = tp["dt"], tp["num_pred"]
    v = math.sqrt(vel[0] * vel[0] + vel[1] * vel[1])
    a0 = math.atan2(vel[1], vel[0])
    fa = tp["front_angle_deg"] * math.pi / 180
    min_v, max_v = v - v, v + v
    samples = []
    i = a0 - fa
    while i < a0 + fa:
        j = min_v
        while j < max_v:
            st = [pos[0], pos[1], j * math.cos(i), j * math.sin(i)]
            pts, valid = [list(pos)], True
            for _ in range(P):
                nxt = [st[0] + dt * st[2], st[1] + dt * st[3], st[2], st[3]]
                p = [nxt[0], nxt[1], pos[2]]
                if occupied(m, occ, p):
                    valid = False
                    break
                pts.append(p)
                st = nxt
            if not valid:
                break
            samples.append(pts)
            j += 0.1
        i += 0.1
    return samples


def model_turning(tp, m, occ, intent, pos, vel):
    """:398-472 -- (speed, angular rate, end angle) grid; colliding samples are dropped."""
    dt, P = tp["dt"], tp["num_pred"]
    v = math.sqrt(vel[0] * vel[0] + vel[1] * vel[1])
    a0 = math.atan2(vel[1], vel[0])
    fa = tp["front_angle_deg"] * math.pi / 180
    if intent == LEFT:
        e_min, e_max = fa + a0, (math.pi - fa) + a0
        w_min, w_max = (math.pi / 2) / tp["max_turning_time"], (math.pi / 2) / tp["min_turning_time"]
    else:
        e_min, e_max = -(math.pi - fa) + a0, -fa + a0
        w_min, w_max = (-math.pi / 2) / tp["min_turning_time"], (-math.pi / 2) / tp["max_turning_time"]
    samples = []
    i = v - v
    while i < v + v:
        j = w_min
        while j < w_max:
            e = e_min
            while e < e_max:
                ang = a0
                st = [pos[0], pos[1], i * math.cos(ang), i * math.sin(ang)]
                pts, valid = [list(pos)], True
                for _ in range(P):
                    nxt = [st[0] + dt * st[2], st[1] + dt * st[3], st[2], st[3]]
                    p = [nxt[0], nxt[1], pos[2]]
                    if occupied(m, occ, p):
                        valid = False
                        break
                    pts.append(p)
                    st = nxt
                    ang += j * dt
                    ang = (e if e < ang else ang) if intent == LEFT else (e if ang < e else ang)
                    vv = math.sqrt(st[2] * st[2] + st[3] * st[3])
                    st[2], st[3] = vv * math.cos(ang), vv * math.sin(ang)
                if valid:
                    samples.append(pts)
                e += 0.2
            j += 0.2
        i += 0.2
    return samples


def gen_traj(tp, m, occ, samples, sizes):
    """:501-566 genTraj + positionCorrection (all samples have num_pred + 1 points)."""
    n = len(samples)
    mean = []
    for t in range(tp["num_pred"] + 1):
        sx = sy = 0.0
        for s in samples:
            sx += s[t][0]
            sy += s[t][1]
        mx, my = sx / n, sy / n
        vx = vy = 0.0
        for s in samples:
            vx += (s[t][0] - mx) * (s[t][0] - mx)
            vy += (s[t][1] - my) * (s[t][1] - my)
        mean.append([mx, my, samples[0][0][2]])
        sizes[t][0] += 2 * math.sqrt(vx / n) * tp["z_score"]
        sizes[t][1] += 2 * math.sqrt(vy / n) * tp["z_score"]
    if any(occupied(m, occ, p) for p in mean):
        min_sum, min_idx = math.inf, -1
        for k, s in enumerate(samples):
            sm = 0.0
            for t in range(len(mean)):
                dx, dy = s[t][0] - mean[t][0], s[t][1] - mean[t][1]
                sm += math.sqrt(dx * dx + dy * dy)
                if sm > min_sum:
                    break
            if sm < min_sum:
                min_sum, min_idx = sm, k
        mean = [list(p) for p in samples[min_idx]]
    return mean, sizes


def predict_traj(tp, m, occ, pos, vel, size):
    """predTraj for one obstacle (:283-330): per intent (FORWARD, LEFT, RIGHT, STOP) the predicted
    positions and sizes, num_pred + 1 each."""
    v = math.sqrt(vel[0] * vel[0] + vel[1] * vel[1])
    out_p, out_s = [], []
    for intent in (FORWARD, LEFT, RIGHT, STOP):
        if v <= tp["stop_vel"] or intent == STOP:
            samples, sizes = [[list(pos)] * (tp["num_pred"] + 1)], _stop_sizes(tp, vel, size)
        elif intent == FORWARD:
            samples, sizes = model_forward(tp, m, occ, pos, vel), [list(size) for _ in range(tp["num_pred"] + 1)]
        else:
            samples, sizes = model_turning(tp, m, occ, intent, pos, vel), [list(size) for _ in range(tp["num_pred"] + 1)]
        if samples:
            mean, sizes = gen_traj(tp, m, occ, samples, sizes)
        else:  # every sample collided (:312-326)
            mean, sizes = [list(pos)] * (tp["num_pred"] + 1), _stop_sizes(tp, vel, size)
        out_p.append(mean)
        out_s.append(sizes)
    return out_p, out_s
