"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of mpcPlanner::makePlanWithPred
(trajectory_planner/include/trajectory_planner/mpcPlanner.cpp:571-661) for one planning instance,
composed of the other restatements (fanout_ref: findClosestObstacle / getIntentComb, mpc_qp_ref:
solveTraj's assembly, select_ref: getTrajectoryScore / evaluateTraj) and the OSQP oracle.  The
oracle for impc.replan.DeviceReplan; only tests/ may import it.

State of an instance (the members makePlanWithPred reads and writes):
  first_time  firstTime_
  plan_x      currentStatesSol_ followed by currentControlsSol_ (QP variable order, :489-508), or None
Branch (:593-606): predictions present (obPredPos_.size()) and not firstTime_ -> the fan-out
(:606-643); otherwise ONE solveTraj (:645-659) -- on a first plan with static and dynamic obstacles
cleared (:593-602), else with dynamicObstaclesPos_ (the current obstacles, each position held over
the horizon as updateDynamicObstacles / updatePredObstacles store them, :326-334 / :352-357; empty
when updatePredObstacles was handed no predictions, :364-371).
Static obstacles (obclustering_->getStaticObstacles(), :594): `static_obs` = [(centroid[3], size[3],
yaw)] enter every solveTraj not on a first plan (:593-602) -- after the dynamic obstacles, with the
isDyamic index quirk of updateObstacleParam (:1194, mpc_qp_ref) -- and getTrajectoryScore (:620).
solveTraj (:375-541): the time limit only when not firstTime_ (:442-444); warm start x = the
previous plan when not firstTime_, else zeros, y = 0 (:485-509); linearisation point = the previous
plan's states (currPos_ when there are none, :1042-1051); success = initSolver succeeded and
solveProblem returned NoError (:475-478, :513-518): osqp_solve's exitflag, 0 for every final status
(infeasible, max-iter, time limit and a NON_CVX from the residual test too, x = OSQP_NAN), 1 only
when an adaptive-rho refactorisation fails (status left UNSOLVED) -- solve_traj_ok.
"""
import numpy as np

from oracle import fanout_ref, mpc_qp_ref, select_ref
from oracle import osqp_oracle as ora

FANOUT, SINGLE_FIRST, SINGLE_CURRENT = 0, 1, 2
NON_CVX = -7
UNSOLVED = -10


def solve_traj_ok(info):
    """solveTraj's successSolve from one oracle solve's info record (module docstring)."""
    return int(info["setup_exitflag"]) == 0 and int(info["status_val"]) != UNSOLVED


def branch(first_time, has_pred, cur_count=0):
    """:606 -- `if (this->obPredPos_.size() and not this->firstTime_)`; the else branch keeps the
    current dynamic obstacles unless firstTime_ cleared them (:593-602)."""
    if has_pred and not first_time:
        return FANOUT
    if not first_time and cur_count > 0:
        return SINGLE_CURRENT
    return SINGLE_FIRST


def _states(plan_x, N):
    return [] if plan_x is None else [list(plan_x[8 * k: 8 * k + 8]) for k in range(N)]


def _qp(params, pos, vel, xref, lin, dyn_pos, dyn_size, static_obs=()):
    qp = mpc_qp_ref.build_qp(params, pos, vel, xref, lin, list(static_obs), dyn_pos, dyn_size)
    pat = dict(n=qp["n"], m=qp["m"], Pp=np.asarray(qp["P"][0]), Pi=np.asarray(qp["P"][1]), Ap=np.asarray(qp["A"][0]),
               Ai=np.asarray(qp["A"][1]))
    vals = dict(Px=np.asarray(qp["P"][2]), q=np.asarray(qp["q"]), Ax=np.asarray(qp["A"][2]), l=np.asarray(qp["l"]),
                u=np.asarray(qp["u"]))
    return pat, vals


def warm_start(first_time, plan_x, n):
    """solveTraj's primal warm start (:485-508): the previous plan unless firstTime_."""
    if first_time or plan_x is None:
        return np.zeros(n)
    return np.asarray(plan_x, np.float64)


def fanout_qps(params, first_time, plan_x, pos, vel, xref, dyn_cur, pred_pos, pred_size, prob, static_obs=()):
    """The fan-out branch's six candidate QPs (:606-615): (fanout dict, [(pattern, values, x_ws)])."""
    N = int(params["horizon"])
    prev = _states(plan_x, N)
    fo = fanout_ref.fanout(list(pos), first_time, prev, dyn_cur, pred_pos, pred_size, prob)
    qps = []
    for cpos, csize in fo["cands"]:
        pat, vals = _qp(params, pos, vel, xref, prev if prev else None, cpos, csize, static_obs)
        qps.append((pat, vals, warm_start(first_time, plan_x, pat["n"])))
    return fo, qps


def single_qp(params, first_time, plan_x, pos, vel, xref, cur_pos=None, cur_size=None, static_obs=()):
    """The single-solve branch's QP (:645-652): no obstacles on a first plan, else the static
    obstacles and the current dynamic obstacles (positions / sizes [K][3]) held over the horizon."""
    N = int(params["horizon"])
    prev = _states(plan_x, N)
    dp, ds = [], []
    if not first_time and cur_pos is not None:
        dp = [[list(cur_pos[k])] * N for k in range(len(cur_pos))]
        ds = [[list(cur_size[k])] * N for k in range(len(cur_size))]
    lin = None if first_time or not prev else prev
    pat, vals = _qp(params, pos, vel, xref, lin, dp, ds, () if first_time else static_obs)
    return pat, vals, warm_start(first_time, plan_x, pat["n"])


def select(params, pd, first_time, plan_x, xref, fo, cand_x, cand_ok, prob_closest, static_obs=()):
    """getTrajectoryScore per successful candidate + evaluateTraj (:617-634) on the candidates'
    solutions cand_x [6][n] (cand_ok [6]: solve_traj_ok of each): the chosen candidate index, or -1
    when none succeeded."""
    N = int(params["horizon"])
    prev = _states(plan_x, N)
    states = [[list(x[8 * k: 8 * k + 8]) for k in range(N)] for x in cand_x]
    valid = [bool(ok) for ok in cand_ok]
    stat = [] if first_time else [(c, z) for c, z, _ in static_obs]
    best, _, _, _ = select_ref.select_instance(states, valid, prev, first_time, [list(r) for r in xref], stat,
                                               [c[0] for c in fo["cands"]], [c[1] for c in fo["cands"]],
                                               prob_closest, pd["dynamic_safety_dist"], pd["static_safety_dist"])
    return best


def solve(pat, vals, x_ws, settings, time_limit=0.0):
    s = ora.settings_from(settings)
    s.time_limit = time_limit
    x, y, info = ora.solve_batch(pat, vals["Px"][None], vals["q"][None], vals["Ax"][None], vals["l"][None],
                                 vals["u"][None], s, x_ws=np.asarray(x_ws)[None])
    return x[0], y[0], info[0]


def make_plan_with_pred(params, pd, settings, state, pos, vel, xref, dyn_cur, pred_pos, pred_size, prob, has_pred,
                        cur_size=None, cur_count=0, static_obs=()):
    """One makePlanWithPred of one instance with oracle solves; `state` = dict(first_time, plan_x)
    is updated as the reference updates its members.  Returns dict(branch, valid, best, x)."""
    ft, px = state["first_time"], state["plan_x"]
    br = branch(ft, has_pred, cur_count)
    if br == FANOUT:
        fo, qps = fanout_qps(params, ft, px, pos, vel, xref, dyn_cur, pred_pos, pred_size, prob, static_obs)
        sols = [solve(p, v, w, settings) for p, v, w in qps]
        best = select(params, pd, ft, px, xref, fo, [s[0] for s in sols], [solve_traj_ok(s[2]) for s in sols],
                      prob[fo["ob_idx"]], static_obs)
        out = dict(branch=br, valid=best >= 0, best=best, x=sols[best][0] if best >= 0 else None)
    else:
        p, v, w = single_qp(params, ft, px, pos, vel, xref, dyn_cur if br == SINGLE_CURRENT else None,
                            cur_size if br == SINGLE_CURRENT else None, static_obs)
        x, _, info = solve(p, v, w, settings)
        ok = solve_traj_ok(info)
        out = dict(branch=br, valid=ok, best=-1, x=x if ok else None)
    if out["valid"]:  # currentStatesSol_ / currentControlsSol_ = the plan, firstTime_ = false
        state["plan_x"] = np.array(out["x"])
        state["first_time"] = 0
    return out
