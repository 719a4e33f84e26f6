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
