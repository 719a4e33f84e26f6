"""Obstacle intent probabilities (dynamic_predictor intentProb, dynamicPredictor.cpp:197-281):
known answers of the restatement (oracle/predict_ref.py) on the CPU, and the device kernel
(impc_intent_prob) against it on the GPU within 1e-13 (floating point; transcendental functions of
the device and glibc may differ by an ulp).  The reference holds no tests for this function, so
the known answers follow from the cited statements (parity of the restatement is unpinned)."""
import math

import numpy as np
import pytest

from oracle import predict_ref as pr

P = pr.params_from_config(0.5, 10.0, 0.1, 5.0)  # predictor_param.yaml


def track(heading, speed, n, turn=0.0, dt=0.1):
    """History of n samples, entry 0 the newest."""
    pos, vel = [], []
    x = y = 0.0
    h = heading
    for _ in range(n):
        vx, vy = speed * math.cos(h), speed * math.sin(h)
        pos.append([x, y, 1.0])
        vel.append([vx, vy, 0.0])
        x, y, h = x + vx * dt, y + vy * dt, h + turn * dt
    return pos[::-1], vel[::-1]


def test_params_from_config():
    assert P["paraml"] == P["paramr"] == 1.0
    fa = 10.0 * math.pi / 180
    assert P["paramf"] == math.sqrt(fa * fa / (-2 * math.log(math.sin(fa))))
    assert P["params"] == math.atanh(0.5) / 0.1


def test_short_history_stays_uniform():
    # fewer than 4 entries: no step with defined inputs (the reference's j = numHist - 1 step
    # reads entry -1, undefined behaviour, and is not taken)
    for n in (0, 1, 2, 3):
        pos, vel = track(0.3, 1.0, n)
        assert pr.intent_prob(P, pos, vel) == [0.25] * 4


def test_transition_columns_are_distributions():
    for theta in (-3.0, -0.5, 0.0, 0.4, 2.9):
        for r in (0.0, 0.05, 1.0):
            for si in range(4):
                v = pr.transition_vector(P, theta, r, si)
                assert abs(sum(v) - 1.0) < 1e-12 and min(v) >= 0


def test_straight_track_is_forward_stopped_is_stop():
    pos, vel = track(0.7, 1.5, 12)
    p = pr.intent_prob(P, pos, vel)
    assert max(range(4), key=lambda k: p[k]) == pr.FORWARD
    pos, vel = track(0.7, 0.0, 12)
    pos = [[0.0, 0.0, 1.0]] * 12
    p = pr.intent_prob(P, pos, vel)
    assert max(range(4), key=lambda k: p[k]) == pr.STOP


def test_left_turn_is_left():
    pos, vel = track(0.0, 1.5, 15, turn=1.2)
    p = pr.intent_prob(P, pos, vel)
    assert p[pr.LEFT] > p[pr.RIGHT]


@pytest.mark.gpu
def test_device_intent_prob_matches_restatement(ctx):
    import impc
    ip = impc.intent_params()
    assert (ip.paramf, ip.paraml, ip.params, ip.pscale) == (P["paramf"], P["paraml"], P["params"], P["pscale"])
    rng = np.random.default_rng(11)
    count, H = 300, 24
    ph, vh = np.zeros((count, H, 3)), np.zeros((count, H, 3))
    hl = rng.integers(0, H + 1, count).astype(np.int32)
    for o in range(count):
        pos, vel = track(rng.uniform(-math.pi, math.pi), rng.uniform(0, 2.5), H, turn=rng.uniform(-1.5, 1.5))
        ph[o], vh[o] = pos, vel
        ph[o] += rng.normal(0, 0.02, (H, 3))
    out = impc.intent_prob(ctx, ip, ph, vh, hl)
    for o in range(count):
        n = hl[o]
        ref = pr.intent_prob(P, ph[o, :n].tolist(), vh[o, :n].tolist())
        np.testing.assert_allclose(out[o], ref, rtol=1e-13, atol=1e-15)


# ---------------------------------------------------------------- predTraj
TP = dict(num_pred=33, dt=0.1, stop_vel=0.1, front_angle_deg=10.0, min_turning_time=2.0, max_turning_time=3.0,
          z_score=0.674)  # predictor_param.yaml


def world(rng=None):
    """A 20 x 20 x 5 m map at 0.1 m with a few inflated walls / pillars."""
    m = dict(origin=[-10.0, -10.0, 0.0], res=0.1, dims=[200, 200, 50])
    occ = np.zeros((200, 200, 50), np.uint8)
    occ[120:124, 40:160, :] = 1      # wall at x = 2.0 .. 2.4
    occ[60:160, 150:154, :] = 1      # wall at y = 5.0 .. 5.4
    occ[80:86, 80:86, :] = 1         # pillar around (-2, -2)
    return m, occ


def test_traj_stop_and_slow_obstacles_are_stationary():
    m, occ = world()
    pp, ps = pr.predict_traj(TP, m, occ.reshape(-1), [0.0, 0.0, 1.0], [0.05, 0.0, 0.0], [0.5, 0.5, 1.0])
    for it in range(4):
        assert all(p == [0.0, 0.0, 1.0] for p in pp[it])
        assert ps[it][1][0] == 0.5 + 2 * 0.05 * 0.1 and ps[it][-1][2] == 1.0


def test_traj_forward_is_straight_and_wall_stops_faster_samples():
    m, occ = world()
    pp, ps = pr.predict_traj(TP, m, occ.reshape(-1), [-5.0, -5.0, 1.0], [1.0, 0.0, 0.0], [0.5, 0.5, 1.0])
    fwd = pp[pr.FORWARD]
    assert fwd[-1][0] > -5.0 and abs(fwd[-1][1] - (-5.0)) < 0.5       # heads +x, spread +-10 deg
    assert ps[pr.FORWARD][-1][1] > 0.5                                  # lateral spread -> wider
    # toward the wall at x = 2: samples that would cross it are cut, the mean stays in front of it
    pp2, _ = pr.predict_traj(TP, m, occ.reshape(-1), [0.5, 0.0, 1.0], [2.0, 0.0, 0.0], [0.5, 0.5, 1.0])
    assert max(p[0] for p in pp2[pr.FORWARD]) < 2.0


def test_traj_left_turns_left():
    m, occ = world()
    pp, _ = pr.predict_traj(TP, m, occ.reshape(-1), [-5.0, -5.0, 1.0], [1.0, 0.0, 0.0], [0.5, 0.5, 1.0])
    assert pp[pr.LEFT][-1][1] > pp[pr.RIGHT][-1][1]


@pytest.mark.gpu
def test_device_predict_traj_matches_restatement(ctx):
    import impc
    m, occ = world()
    tp = impc.TrajParams(num_pred=TP["num_pred"], dt=TP["dt"], stop_velocity=TP["stop_vel"],
                         front_angle_deg=TP["front_angle_deg"], min_turning_time=TP["min_turning_time"],
                         max_turning_time=TP["max_turning_time"], z_score=TP["z_score"])
    om = impc.OccMap()
    om.origin[:] = m["origin"]
    om.resolution = m["res"]
    om.dims[:] = m["dims"]
    rng = np.random.default_rng(12)
    count = 24
    pos = np.stack([rng.uniform(-6, 4, count), rng.uniform(-6, 6, count), np.full(count, 1.0)], axis=1)
    hd = rng.uniform(-math.pi, math.pi, count)
    sp = rng.choice([0.05, 0.5, 1.0, 1.8], count)
    vel = np.stack([sp * np.cos(hd), sp * np.sin(hd), np.zeros(count)], axis=1)
    size = np.tile([0.5, 0.5, 1.0], (count, 1))
    pp, ps = impc.predict_traj(ctx, tp, om, occ.reshape(-1), pos, vel, size)
    flat = occ.reshape(-1)
    for o in range(count):
        rp, rs = pr.predict_traj(TP, m, flat, pos[o].tolist(), vel[o].tolist(), size[o].tolist())
        np.testing.assert_allclose(pp[o], np.asarray(rp), rtol=1e-12, atol=1e-12, err_msg=f"obstacle {o}")
        np.testing.assert_allclose(ps[o], np.asarray(rs), rtol=1e-12, atol=1e-12, err_msg=f"obstacle {o}")
