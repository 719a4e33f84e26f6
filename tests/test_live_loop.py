"""The live replan loop on the reference's own input path (ISSUE item: a closed-loop replay):
planning instances fly autonomous_flight's benchmark path (ref_trajectory_dynus_benchmark.txt,
mpcNavigation::getRefTraj / updatePath(path, 0.1)) at the live planner horizon N = 30
(planner_param.yaml:25) for 30 chained replans, each replan as mpcNavigation::mpcCB runs it
(mpcNavigation.cpp:290-322): getXRef on the device (impc_reference_traj_device, lastRefStartIdx_
kept), impc_replan_run (makePlanWithPred: a first plan, then the intent fan-out every replan),
and the vehicle following its plan for one 0.1 s step (impc_replan_advance_device:
getPos / getVel(dt), mpc_node.cpp:216-224).  Dynamic obstacles move on and are re-predicted
every replan (the predictor's kinematic intent models, scenarios.live_loop).

Every replan is checked against the restatements: the reference trajectory bit for bit
(oracle/reftraj_ref.py), the branch, the closest obstacle and candidate order, every assembled QP
bit for bit, every solution against the OSQP oracle (identical status and iterations, 1e-5), the
selection bit for bit and the committed plan (oracle/replan_ref.py, tests/test_replan_branches.py
_check_replan).  Parity of the solutions is unpinned against the real libosqp."""
import numpy as np
import pytest

import impc
from impc import scenarios
from impc.replan import FANOUT, SINGLE_FIRST, DeviceReplan
from oracle.reftraj_ref import ReferencePath

from test_replan_branches import _check_replan

pytestmark = pytest.mark.gpu


def _dump_failure(rp, r, out, plan_x_before, ft_before, pos, vel, xref, sc):
    """A failed replan's inputs and device outputs, for offline analysis: the state the host checked
    against (plan_x before the replan), the device's state and linearisation points now, every
    assembled value and solution of the replan (gpurun_out/live_loop_failure_r<r>.npz)."""
    import os
    from impc.replan import _get
    try:
        v = rp.view()
        states = _get(rp.ctx, v.plan_states, (rp.I + 1, rp.N * 8), np.float64)
        px, ft, pc, valid = rp.plans()
        arrs = {k: np.asarray(val) for k, val in out.items()
                if isinstance(val, np.ndarray) and val.dtype != object}
        for k, val in out.items():
            if isinstance(val, (list, tuple)) and val and isinstance(val[0], np.ndarray):
                for j, a in enumerate(val):
                    arrs[f"{k}_{j}"] = a
        os.makedirs("gpurun_out", exist_ok=True)
        np.savez(f"gpurun_out/live_loop_failure_r{r}.npz", plan_x_before=plan_x_before, ft_before=ft_before,
                 pos=pos, vel=vel, xref=xref, plan_states_now=states, plan_x_now=px, pred_pos=sc["pred_pos"][r],
                 dyn_cur=sc["dyn_cur"][r], pred_size=sc["pred_size"], prob=sc["prob"], **arrs)
    except Exception as ex:  # the dump must not mask the assertion
        print("live-loop failure dump:", ex)


def test_live_loop_thirty_replans_on_the_benchmark_path(ctx):
    I, K, R, N = 6, 3, 30, 30
    sc = scenarios.live_loop(I, K, R, N=N, seed=4100)
    p, pd, L = sc["params"], sc["pd"], sc["L"]
    s = impc.default_settings(verbose=0)
    rp = DeviceReplan(ctx, p, pd, I, K, L, s)
    paths = impc.ReferencePaths(ctx, list(sc["paths"]), pd["ts"], N)
    refs = [ReferencePath(pth, pd["ts"], N) for pth in sc["paths"]]
    D = impc.DeviceArray
    pos_d, vel_d, xref_d = D(ctx, sc["pos0"]), D(ctx, sc["vel0"]), D(ctx, (I, N, 8))
    psize_d, prob_d = D(ctx, sc["pred_size"]), D(ctx, np.ascontiguousarray(sc["prob"]))
    pos, vel = sc["pos0"].copy(), sc["vel0"].copy()
    plan_x, ft = np.zeros((I, 13 * N - 5)), np.ones(I, np.int8)
    branches = []
    try:
        for r in range(R):
            pred_d, cur_d = D(ctx, np.ascontiguousarray(sc["pred_pos"][r])), D(ctx, sc["dyn_cur"][r])
            paths.xref_device(pos_d.ptr, xref_d.ptr)
            rp.run_device(pos_d.ptr, vel_d.ptr, xref_d.ptr, cur_d.ptr, pred_d.ptr, psize_d.ptr, prob_d.ptr)
            ctx.synchronize()
            out = rp.results()
            xref = xref_d.get()
            np.testing.assert_array_equal(pos_d.get(), pos)               # x0 replayed on the host
            exp_xref = np.array([refs[i].xref(pos[i]) for i in range(I)])
            np.testing.assert_array_equal(xref, exp_xref, err_msg=f"replan {r}: getXRef")
            try:
                expect, expect_first = _check_replan(out, (plan_x, ft, None, None), pos, vel, xref, sc["dyn_cur"][r],
                                                     sc["pred_pos"][r], sc["pred_size"], sc["prob"], np.ones(I, bool),
                                                     None, np.zeros(I, np.int32), pd, s)
            except AssertionError as e:
                _dump_failure(rp, r, out, plan_x, ft, pos, vel, xref, sc)
                raise AssertionError(f"replan {r}: {e}") from e
            plan_x, ft_new, _, valid = rp.plans()
            np.testing.assert_array_equal(plan_x, expect, err_msg=f"replan {r}: committed plans")
            np.testing.assert_array_equal(ft_new, expect_first)
            ft = ft_new
            branches.append(out["branch"].copy())
            rp.advance_device(pd["ts"], pos_d.ptr, vel_d.ptr)
            # getPos / getVel(dt) of a fresh plan: its state 1 (idx = floor(dt / ts) = 1, no interpolation)
            pos = np.where(valid[:, None] == 1, plan_x[:, 8:11], pos)
            vel = np.where(valid[:, None] == 1, plan_x[:, 11:14], vel)
            pred_d.free()
            cur_d.free()
        br = np.array(branches)
        assert (br[0] == SINGLE_FIRST).all() and (br[1:] == FANOUT).all()
        # the vehicles moved along the path: lastRefStartIdx_ advanced for every instance
        assert (paths.last_idx() > 0).all()
        assert (pos[:, 0] > sc["pos0"][:, 0] + 5.0).all()
    finally:
        for d in (pos_d, vel_d, xref_d, psize_d, prob_d):
            d.free()
        paths.close()
        rp.close()
