"""Seeded synthetic MPC workloads for tests and bench.py.

Produces the per-instance inputs mpcPlanner::solveTraj consumes (current state, reference
trajectory, previous plan, obstacles / intent predictions) and turns them into batched QPs with
the product builder (impc_mpc_build_values).  Synthetic data only: the reference's Gazebo /
DYNUS worlds are not available, so obstacle placement follows the distributions SURVEY.md 8d
derives from dynus_obstacles_node.cpp:74-133 and the predictor's 4-intent models
(dynamicPredictor.cpp:351-501: FORWARD / LEFT / RIGHT / STOP at 0.1 s steps).
"""
import math
import os

import numpy as np

from . import mpc_params, mpc_pattern, mpc_values

# dynamicPredictor utils.h:15-20 intent enum order
FORWARD, LEFT, RIGHT, STOP = 0, 1, 2, 3
PRED_STEPS = 30  # predictor_param.yaml:2 (30 steps @ 0.1 s) -> 31 positions


def _x0(rng, nb):
    pos = np.stack([np.zeros(nb), rng.uniform(-1, 1, nb), rng.uniform(1.5, 2.5, nb)], axis=1)
    vel = np.stack([rng.uniform(0, 5, nb), rng.uniform(-1, 1, nb), np.zeros(nb)], axis=1)
    return pos, vel


# Reference-path spacing per 0.1 s step: U(0.5, 2.5) m, i.e. 5-25 m/s -- the live
# benchmark path's raw points are 2.5 m apart and getReferenceTraj (mpcPlanner.cpp:1199-1231)
# samples them one per step, so most of this range is faster than vmax = 5 m/s and the QPs track a
# reference they cannot reach (iteration counts against the spacing).
STEP_RANGE = (0.5, 2.5)


def _xref(rng, pos, N, step_range=STEP_RANGE):
    nb = pos.shape[0]
    step = rng.uniform(step_range[0], step_range[1], nb)  # m per 0.1 s step
    xr = np.zeros((nb, N, 8))
    k = np.arange(N)
    xr[:, :, 0] = pos[:, None, 0] + k[None, :] * step[:, None]
    xr[:, :, 1] = pos[:, None, 1]
    xr[:, :, 2] = pos[:, None, 2]
    return xr


def _prev_plan(pos, vel, N, ts):
    """A previous receding-horizon plan (currentStatesSol_): constant-velocity rollout."""
    nb = pos.shape[0]
    st = np.zeros((nb, N, 8))
    k = np.arange(N) * ts
    st[:, :, 0:3] = pos[:, None, :] + k[None, :, None] * vel[:, None, :]
    st[:, :, 3:6] = vel[:, None, :]
    return st


def static_config(N=20, K=10, batch=4096, seed=2000, identical=True, params=None):
    """Config 2: batch of N=20 QPs with K static-style obstacle rows (copies of one seed if identical)."""
    p, pd = params if params is not None else mpc_params(horizon=N)
    rng = np.random.default_rng(seed)
    nb = 1 if identical else batch
    pos, vel = _x0(rng, nb)
    xref = _xref(rng, pos, N)
    cen = np.stack([pos[:, None, 0] + rng.uniform(2, 20, (nb, K)), rng.uniform(-5, 5, (nb, K)),
                    rng.uniform(0.5, 4.5, (nb, K))], axis=2)
    tall = rng.uniform(size=(nb, K)) < 0.5
    size = np.where(tall[:, :, None], np.array([0.4, 0.4, 4.0]), np.array([0.4, 4.0, 0.4]))
    yaw = rng.uniform(-math.pi, math.pi, (nb, K))
    if identical:
        rep = lambda a: np.repeat(a, batch, axis=0)
        pos, vel, xref, cen, size, yaw = map(rep, (pos, vel, xref, cen, size, yaw))
    pat = mpc_pattern(p, K, 0)
    vals = mpc_values(p, pos, vel, xref, None, st_centroid=cen, st_size=size, st_yaw=yaw)
    return dict(pattern=pat, values=vals, x_ws=None, params=pd, K=K, N=N)


def predict_intents(p0, v0, steps=PRED_STEPS, ts=0.1, omega=0.6, stop_time=1.0):
    """[..., 4 intents, steps+1, 3] kinematic predictions (FORWARD/LEFT/RIGHT/STOP)."""
    t = np.arange(steps + 1) * ts
    sp = np.linalg.norm(v0[..., :2], axis=-1)
    hd = np.arctan2(v0[..., 1], v0[..., 0])
    out = np.zeros(p0.shape[:-1] + (4, steps + 1, 3))
    # FORWARD: constant velocity
    out[..., FORWARD, :, :] = p0[..., None, :] + t[:, None] * v0[..., None, :]
    # LEFT / RIGHT: constant-speed turn at +-omega
    for idx, sgn in ((LEFT, 1.0), (RIGHT, -1.0)):
        w = sgn * omega
        h = hd[..., None] + w * t
        out[..., idx, :, 0] = p0[..., None, 0] + sp[..., None] / w * (np.sin(h) - np.sin(hd[..., None]))
        out[..., idx, :, 1] = p0[..., None, 1] - sp[..., None] / w * (np.cos(h) - np.cos(hd[..., None]))
        out[..., idx, :, 2] = p0[..., None, 2]
    # STOP: linear deceleration to rest over stop_time
    tt = np.minimum(t, stop_time)
    frac = tt - tt * tt / (2 * stop_time)
    out[..., STOP, :, :] = p0[..., None, :] + frac[:, None] * v0[..., None, :]
    return out


def intent_config(N=20, K=8, instances=8192, hyps=8, seed=3000, params=None, step_range=STEP_RANGE):
    """Config 3: `instances` planning instances x `hyps` hypotheses, K dynamic obstacles each.

    Hypotheses 0-5 are mpcPlanner::getIntentComb's six combinations for the closest obstacle
    (mpcPlanner.cpp:710-769, sorted by intent weight; the LEFT+FORWARD / RIGHT+FORWARD ones carry
    K+1 obstacle trajectories), 6-7 are extra argmax variants (all-argmax, all-FORWARD).
    Returns the QPs bucketed by obstacle count: {K: bucket, K+1: bucket}; each bucket has
    pattern, values, warm start and the (instance, hypothesis) of every QP.
    """
    p, pd = params if params is not None else mpc_params(horizon=N)
    rng = np.random.default_rng(seed)
    ts = pd["ts"]
    I = instances
    pos, vel = _x0(rng, I)
    xref = _xref(rng, pos, N, step_range)
    prev = _prev_plan(pos, vel, N, ts)
    obp = np.stack([pos[:, None, 0] + rng.uniform(3, 15, (I, K)), rng.uniform(-4, 4, (I, K)),
                    rng.uniform(1.0, 3.0, (I, K))], axis=2)
    spd = rng.uniform(0.5, 2.0, (I, K))
    hdg = rng.uniform(-math.pi, math.pi, (I, K))
    obv = np.stack([spd * np.cos(hdg), spd * np.sin(hdg), np.zeros((I, K))], axis=2)
    pred = predict_intents(obp, obv, ts=ts)                 # [I, K, 4, 31, 3]
    prob = rng.dirichlet(np.ones(4), size=(I, K))            # [I, K, 4]
    # The previous plan (the linearisation point, mpcPlanner.cpp:1042-1051) was the collision-free
    # answer of the last replan: re-draw obstacles whose most likely predicted track enters the
    # inflated ellipsoid around it (semi-axis size/2 + dynamic safety distance).
    clear = 0.4 + pd["dynamic_safety_dist"]
    for _ in range(64):
        am = np.argmax(prob, axis=2)
        steps = np.minimum(np.arange(N), pred.shape[3] - 1)  # prediction clamped to .back() (:1165-1184)
        track = np.take_along_axis(pred, am[:, :, None, None, None], axis=2)[:, :, 0][:, :, steps]  # [I, K, N, 3]
        bad = (np.linalg.norm(track - prev[:, None, :, :3], axis=3) < clear).any(axis=2)   # [I, K]
        if not bad.any():
            break
        nb_ = int(bad.sum())
        obp[bad] = np.stack([pos[np.nonzero(bad)[0], 0] + rng.uniform(3, 15, nb_), rng.uniform(-4, 4, nb_),
                             rng.uniform(1.0, 3.0, nb_)], axis=1)
        h2 = rng.uniform(-math.pi, math.pi, nb_)
        s2 = rng.uniform(0.5, 2.0, nb_)
        obv[bad] = np.stack([s2 * np.cos(h2), s2 * np.sin(h2), np.zeros(nb_)], axis=1)
        pred[bad] = predict_intents(obp[bad], obv[bad], ts=ts)
        prob[bad] = rng.dirichlet(np.ones(4), size=nb_)
    size = np.full(3, 0.8)                                   # dynus_obstacles_node.cpp:81 cubes
    # findClosestObstacle (first-time branch, :663-674): nearest current position
    d = np.linalg.norm(obp - pos[:, None, :], axis=2)
    ob = np.argmin(d, axis=1)
    argmax_int = np.argmax(prob, axis=2)                     # [I, K]
    buckets = {}
    for kk in (K, K + 1):
        buckets[kk] = dict(dyn_pos=[], inst=[], hyp=[])
    for i in range(I):
        o = ob[i]
        pr = prob[i, o]
        # getIntentComb weights (:722-728), std::sort ascending, take from the back (:753-756)
        weight = [(pr[STOP], 0), (pr[LEFT], 1), (pr[RIGHT], 2), (pr[FORWARD], 3),
                  (max(pr[LEFT], pr[FORWARD]), 4), (max(pr[RIGHT], pr[FORWARD]), 5)]
        weight.sort()
        combos = {0: [STOP], 1: [LEFT], 2: [RIGHT], 3: [FORWARD], 4: [LEFT, FORWARD], 5: [RIGHT, FORWARD]}
        others = [pred[i, j, argmax_int[i, j]] for j in range(K) if j != o]
        hyp_sets = []
        for h in range(6):
            cid = weight[5 - h][1]
            hyp_sets.append([pred[i, o, it] for it in combos[cid]] + others)
        hyp_sets.append([pred[i, o, argmax_int[i, o]]] + others)
        hyp_sets.append([pred[i, j, FORWARD] for j in range(K)])
        for h, sets in enumerate(hyp_sets[:hyps]):
            kk = len(sets)
            buckets[kk]["dyn_pos"].append(np.stack(sets))
            buckets[kk]["inst"].append(i)
            buckets[kk]["hyp"].append(h)
    # per-instance inputs of the candidate selection (makePlanWithPred / evaluateTraj)
    inst_data = dict(prev=prev, xref=xref, prob=prob[np.arange(I), ob], closest=ob,
                     pos=pos, vel=vel, obp=obp, pred=pred, prob_all=prob, size=size)
    out = {}
    for kk, bk in buckets.items():
        if not bk["inst"]:
            continue
        inst = np.array(bk["inst"])
        dp = np.stack(bk["dyn_pos"])                         # [nb, kk, 31, 3]
        ds = np.broadcast_to(size, dp.shape).copy()
        pat = mpc_pattern(p, 0, kk)
        vals = mpc_values(p, pos[inst], vel[inst], xref[inst], prev[inst], dyn_pos=dp, dyn_size=ds)
        nb = inst.size
        n = pat["n"]
        x_ws = np.zeros((nb, n))
        x_ws[:, : 8 * N] = prev[inst].reshape(nb, -1)          # solveTraj warm start (:489-498)
        out[kk] = dict(pattern=pat, values=vals, x_ws=x_ws, inst=inst, hyp=np.array(bk["hyp"]), K=kk, N=N,
                       params=pd, dyn_pos=dp, dyn_size=ds, instances=inst_data)
    return out


def slice_instances(buckets, lo, hi):
    """Planning instances [lo, hi) of intent_config buckets (one rank's share of config 3 split by
    instance, strong scaling): each bucket keeps the QPs of those instances, with instance indices
    local to the slice (``inst``) and global (``inst_global``), and the per-instance arrays sliced
    the same way.  Buckets left empty are dropped."""
    out = {}
    for kk, bk in buckets.items():
        sel = (bk["inst"] >= lo) & (bk["inst"] < hi)
        if not sel.any():
            continue
        nb = dict(bk)
        nb["values"] = {k: v[sel] for k, v in bk["values"].items()}
        for k in ("x_ws", "hyp", "dyn_pos", "dyn_size"):
            nb[k] = bk[k][sel]
        nb["inst_global"] = bk["inst"][sel]
        nb["inst"] = bk["inst"][sel] - lo
        nb["instances"] = {k: (v if k == "size" else v[lo:hi]) for k, v in bk["instances"].items()}
        out[kk] = nb
    return out


def queue_weight(pd, N):
    """q_weight of the longest-first work queue (impc_batch_set_queue_order) for mpcPlanner QPs:
    with q = -Q xRef (castMPCToQPGradient, mpcPlanner.cpp:952-966), ||q||_inf / (position weight
    x (N - 1)) is the reference's mean advance per step (m); the key weighs it 1:10 against the
    warm start's constraint violation (m), the measured ranking of the ADMM iteration count on
    config 3's QPs (tools/queue_order_study.py)."""
    return 1.0 / (10.0 * (N - 1) * pd["position_weight"])


def first_call_config(N=20, batch=1, seed=1000, params=None, step_range=STEP_RANGE):
    """Config 1: the first makePlan() QP -- no obstacles, cold start (mpcPlanner.cpp:543-569)."""
    p, pd = params if params is not None else mpc_params(horizon=N)
    rng = np.random.default_rng(seed)
    pos, vel = _x0(rng, batch)
    xref = _xref(rng, pos, N, step_range)
    pat = mpc_pattern(p, 0, 0)
    vals = mpc_values(p, pos, vel, xref, None)
    return dict(pattern=pat, values=vals, x_ws=None, params=pd, K=0, N=N)


def selection_arrays(buckets, ptr_by_bucket, C=6):
    """Inputs of impc.select_best for the intent_config buckets: hypotheses 0..C-1 of every
    instance are mpcPlanner's getIntentComb candidates.  ptr_by_bucket[K] is the device address
    of bucket K's QP-major solution array (Batch.device_results()[0])."""
    any_bk = next(iter(buckets.values()))
    inst = any_bk["instances"]
    I = inst["prev"].shape[0]
    N = any_bk["N"]
    kmax = max(buckets)
    L = any_bk["dyn_pos"].shape[2]
    x_ptrs = np.zeros(I * C, np.uint64)
    dyn_pos = np.zeros((I, C, kmax, L, 3))
    dyn_size = np.zeros((I, C, kmax, L, 3))
    dyn_count = np.zeros((I, C), np.int32)
    rows = {}
    for K, bk in buckets.items():
        n = bk["pattern"]["n"]
        sel = bk["hyp"] < C
        r = np.nonzero(sel)[0]
        i, h = bk["inst"][sel], bk["hyp"][sel]
        x_ptrs[i * C + h] = np.uint64(ptr_by_bucket[K]) + (r * n * 8).astype(np.uint64)
        dyn_pos[i, h, :K] = bk["dyn_pos"][r]
        dyn_size[i, h, :K] = bk["dyn_size"][r]
        dyn_count[i, h] = K
        rows[K] = (i, h, r)
    return dict(I=I, N=N, C=C, kmax=kmax, L=L, x_ptrs=x_ptrs, dyn_pos=dyn_pos, dyn_size=dyn_size,
                dyn_count=dyn_count, prev=inst["prev"], xref=inst["xref"], prob=inst["prob"], rows=rows)


# ---------------------------------------------------------------- config 4 (mixed K, sharded)
def config4_plan(total_qps=262144, hyps=8, kmax=20, N=20, seed=4000):
    """BASELINE.json configs[3]: total_qps QPs = total_qps / hyps planning instances, each with
    K ~ U{0..kmax} predicted dynamic obstacles and `hyps` intent hypotheses (two of them carry K + 1
    obstacle rows, as getIntentComb's two-intent candidates; K = 0 instances have no obstacle to
    branch on and solve `hyps` obstacle-free QPs).  Returns (K per instance, weight per instance):
    the weight is the instance's summed constraint count Sigma m, the shard-balancing measure."""
    I = total_qps // hyps
    K = np.random.default_rng(seed).integers(0, kmax + 1, I)
    m = lambda k: 21 * N - 5 + k * (N - 1)
    w = np.where(K > 0, (hyps - 2) * m(K) + 2 * m(K + 1), hyps * m(0))
    return K, w


def config4_rank(lo, hi, K, hyps=8, N=20, seed=4000, params=None):
    """The QP buckets of planning instances [lo, hi) of a config4_plan (one rank's shard).  Each
    bucket is one (generating K, obstacle count) pair -- pattern, values, warm start, and the
    GLOBAL instance index + hypothesis of every QP.  Seeds depend on the instance range only, so a
    shard's QPs are the same whatever process generates them."""
    out = []
    Ks = np.asarray(K)[lo:hi]
    for k in np.unique(Ks):
        idx = lo + np.nonzero(Ks == k)[0]                    # global instance ids with this K
        sd = seed + 101 * int(k) + 7919 * int(lo)
        if k == 0:
            c = first_call_config(N=N, batch=hyps * idx.size, seed=sd, params=params)
            c.update(inst=np.repeat(idx, hyps), hyp=np.tile(np.arange(hyps), idx.size))
            out.append(c)
            continue
        for kk, bk in sorted(intent_config(N=N, K=int(k), instances=idx.size, hyps=hyps, seed=sd,
                                           params=params).items()):
            bk = dict(bk)
            bk["inst"] = idx[bk["inst"]]
            out.append(bk)
    return out


def receding_update(bk, shift=1, params=None):
    """Config 5's receding window (BASELINE.json configs[4]) for a bucket of intent_config: the next
    replan's QP values -- xRef shifted by `shift` steps along the path (extended at its last
    spacing) and x0 moved to the previous plan's state `shift` -- with the same linearisation
    points (the previous plan), so P and A are unchanged and the step is a legal
    osqp_update_lin_cost (q) + osqp_update_bounds (l, u) on a persistent workspace
    (polyTrajSolver.cpp:225-237's pattern, OsqpEigen Solver.hpp:151-182)."""
    N = bk["N"]
    inst = bk["inst"]
    d = bk["instances"]
    xref, prev = d["xref"][inst], d["prev"][inst]
    step = xref[:, -1, :] - xref[:, -2, :]
    ext = xref[:, -1:, :] + step[:, None, :] * np.arange(1, shift + 1)[None, :, None]
    xr2 = np.concatenate([xref[:, shift:], ext], axis=1)
    p, _ = params if params is not None else mpc_params(horizon=N)
    return mpc_values(p, prev[:, shift, 0:3], prev[:, shift, 3:6], xr2, prev, dyn_pos=bk["dyn_pos"],
                      dyn_size=bk["dyn_size"])


# ------------------------------------------------------------------ the live replan loop
# The reference's predefined benchmark path (autonomous_flight/cfg/mpc_navigation/
# ref_trajectory_dynus_benchmark.txt: "t x y z" per line, read by mpcNavigation::getRefTraj,
# mpcNavigation.cpp:189-218, and handed to updatePath(path, 0.1) as is, :227-236), kept as a data
# fixture so no run reads /root/reference.
DYNUS_PATH_FILE = os.path.join(os.path.dirname(__file__), "..", "..", "..", "tests", "golden",
                               "ref_trajectory_dynus_benchmark.txt")


def dynus_path():
    """[P][3] points of the reference's benchmark path (the t column dropped, as getRefTraj does)."""
    rows = []
    with open(DYNUS_PATH_FILE) as f:
        for ln in f:
            parts = ln.split()
            if len(parts) < 4:
                break
            rows.append([float(parts[1]), float(parts[2]), float(parts[3])])
    return np.array(rows)


def live_loop(instances, K, replans, N=30, seed=4100, params=None):
    """R chained replans of I planning instances flying the reference's benchmark path, each
    instance's copy of the path shifted sideways / up by a seeded offset, K dynamic obstacles per
    instance crossing it at constant velocity (re-predicted every 0.1 s replan by the predictor's
    four kinematic intent models, predict_intents), constant intent probabilities per obstacle.
    The vehicle starts at rest at its path's first point on its first plan (firstTime_).
    Returns dict(paths [I][P][3], pos0 / vel0 [I][3], pred_pos [R][I][K][4][L][3] (the predictions
    handed to replan r), pred_size [I][K][4][L][3], prob [I][K][4], dyn_cur [R][I][K][3], size,
    params, pd, N, K, L)."""
    p, pd = params if params is not None else mpc_params(horizon=N)
    rng = np.random.default_rng(seed)
    I, ts = instances, pd["ts"]
    base = dynus_path()
    off = np.stack([np.zeros(I), rng.uniform(-1.5, 1.5, I), rng.uniform(-0.5, 0.5, I)], axis=1)
    paths = base[None, :, :] + off[:, None, :]
    pos0 = paths[:, 0, :].copy()
    vel0 = np.zeros((I, 3))
    # obstacles: ahead along x, 4-9 m to the side of the path, drifting across it or along it
    side = np.where(rng.uniform(size=(I, K)) < 0.5, -1.0, 1.0)
    obp = np.stack([pos0[:, None, 0] + rng.uniform(8, 60, (I, K)),
                    pos0[:, None, 1] + side * rng.uniform(4, 9, (I, K)),
                    pos0[:, None, 2] + rng.uniform(-0.3, 0.3, (I, K))], axis=2)
    spd = rng.uniform(0.2, 1.0, (I, K))
    hdg = np.where(side < 0, 0.5 * math.pi, -0.5 * math.pi) + rng.uniform(-1.0, 1.0, (I, K))
    obv = np.stack([spd * np.cos(hdg), spd * np.sin(hdg), np.zeros((I, K))], axis=2)
    prob = rng.dirichlet(np.full(4, 2.0), size=(I, K))
    L = PRED_STEPS + 1
    pred = np.empty((replans, I, K, 4, L, 3))
    for r in range(replans):
        pred[r] = predict_intents(obp + obv * (r * ts), obv, ts=ts)
    size = np.full(3, 0.8)
    pred_size = np.ascontiguousarray(np.broadcast_to(size, (I, K, 4, L, 3)))
    return dict(paths=paths, pos0=pos0, vel0=vel0, pred_pos=pred, pred_size=pred_size, prob=prob,
                dyn_cur=np.ascontiguousarray(pred[:, :, :, FORWARD, 0, :]), size=size, params=p, pd=pd, N=N, K=K, L=L)
