"""makePlanWithPred (trajectory_planner mpcPlanner.cpp:571-661) for a batch of planning instances,
with every stage on the device, both of its branches, and the planner state carried from one
replan to the next on the device.

Per instance, as the reference decides (:593-606):
  * fan-out branch -- not firstTime_ and predictions present (obPredPos_.size()): the intent fan-out
    (impc_intent_fanout_device, :663-769), the MPC -> QP assembly of the two candidate shapes
    (impc_mpc_build_values_device, :891-1197), the candidates' solves (solveTraj with timeLimit),
    scoring / selection (impc_select_best_device, :771-887); the chosen candidate is the plan
    (:629-639);
  * single-solve branch -- firstTime_ or no predictions (:645-659): ONE QP, no time limit
    (solveTraj's default 1e10, and none at all on a first plan, :442-444), no scoring; its solution
    is the plan when solveTraj succeeds.  On a first plan the static and dynamic obstacles are
    cleared (:593-602), so the QP has no obstacle rows and no warm start (:487-508, firstTime_);
    otherwise it takes the instance's current dynamic obstacles, dynamicObstaclesPos_, each
    position held over the horizon (updateDynamicObstacles :316-341) -- or none, when predictions
    were cleared (updatePredObstacles :364-371 clears them too, the live predictor loop's case).
All candidate and single-solve QPs of a replan go to ONE grouped launch.  The plan of every
instance that has one is then committed on the device (impc_replan_commit_device): it becomes
the next replan's warm start (the QP solution x: states then controls) and linearisation point,
and firstTime_ clears; an instance without a plan keeps its state (validTraj = false).

The replan's wall-clock budget (:609-628): the reference issues candidate i only while
`time = now - startTime < 0.15 s` and solves it with `timeLimit = max(solverTimeLimit_ - time,
solverTimeLimit_)` (solver_time_limit, 0.05 s by default, :166-167); a candidate enters the
selection only when solveTraj succeeded, i.e. solveProblem returned NoError (:513-518) -- every
status but a non-convex problem.  The batch issues all six candidates of every fan-out instance at
one instant, so the cut-off is one check before the grouped solve: past it no candidate is issued
and every fan-out instance selects nothing (best_cand -1, validTraj = false).  The single-solve
branch has no cut-off.
"""
import ctypes as C
import time

import numpy as np

from . import (NON_CVX, Batch, DeviceArray, MpcBuilder, ReferencePaths, SelectParams, _P, _check, gather_rows_device,
               lib, mpc_dims, mpc_pattern, repeat_rows_device, solve_group)

ISSUE_CUTOFF_S = 0.15  # makePlanWithPred: no candidate is issued 0.15 s after the replan started (:613)
FANOUT, SINGLE_FIRST, SINGLE_CURRENT = 0, 1, 2  # the branch an instance took (run()["branch"])


def candidate_valid(cand_slot, status_single, status_pair):
    """valid[i][c] of the selection: candidate c of instance i was solved without an OSQP error
    (solveTraj's successSolve, mpcPlanner.cpp:513-518 -- every status but OSQP_NON_CVX).  Candidate
    c sits at row 4i+slot of the single-intent batch (slot < 4) or 2i+slot-4 of the two-intent
    batch (fanout.hpp k_fanout_candidates)."""
    slot = np.asarray(cand_slot)
    ii = np.arange(slot.shape[0])[:, None]
    ok_s = np.asarray(status_single) != NON_CVX
    ok_p = np.asarray(status_pair) != NON_CVX
    return np.where(slot < 4, ok_s[4 * ii + np.minimum(slot, 3)], ok_p[2 * ii + np.clip(slot - 4, 0, 1)]).astype(np.int8)


def branches(first_time, has_pred, cur_count=None):
    """The makePlanWithPred branch of every instance (:606): FANOUT when not firstTime_ and
    predictions are present, else SINGLE_CURRENT when not firstTime_ and current dynamic obstacles
    are present (cur_count > 0), else SINGLE_FIRST (the obstacle-free QP)."""
    ft = np.asarray(first_time).astype(bool)
    hp = np.asarray(has_pred).astype(bool)
    cur = np.zeros_like(ft) if cur_count is None else np.asarray(cur_count) > 0
    return np.where(~ft & hp, FANOUT, np.where(~ft & cur, SINGLE_CURRENT, SINGLE_FIRST)).astype(np.int8)


class PlanState:
    """The planner state of I instances on the device (include/impc_replan.h): plan_x [I+1][n] --
    currentStatesSol_ and currentControlsSol_ in QP variable order, i.e. the warm start of the next
    solveTraj --, plan_states [I+1][N][8] (its states: the linearisation point), prev_count [I]
    (currentStatesSol_.size()), first_time [I] and valid [I] (the last replan's validTraj).  Row I
    of plan_x / plan_states stays zero: the warm start of a first-plan solve is gathered from it."""

    def __init__(self, ctx, I, N, prev=None, first_time=None, prev_count=None, prev_controls=None):
        self.ctx, self.I, self.N, self.n = ctx, int(I), int(N), 13 * int(N) - 5
        px = np.zeros((self.I + 1, self.n))
        if prev is not None:
            pv = np.asarray(prev, np.float64).reshape(self.I, -1, 8)
            assert pv.shape[1] == self.N, "the plan state holds N states per instance"
            px[: self.I, : 8 * self.N] = pv.reshape(self.I, -1)
        if prev_controls is not None:
            px[: self.I, 8 * self.N:] = np.asarray(prev_controls, np.float64).reshape(self.I, -1)
        self.first_time_h = (np.ones(self.I, np.int8) if first_time is None
                             else np.ascontiguousarray(first_time, np.int8).reshape(self.I).copy())
        pc = (np.full(self.I, self.N if prev is not None else 0, np.int32) if prev_count is None
              else np.ascontiguousarray(prev_count, np.int32).reshape(self.I))
        self.plan_x = DeviceArray(ctx, px)
        self.plan_states = DeviceArray(ctx, np.ascontiguousarray(px[:, : 8 * self.N]).reshape(self.I + 1, self.N, 8))
        self.prev_count = DeviceArray(ctx, pc)
        self.first_time = DeviceArray(ctx, self.first_time_h)
        self.valid = DeviceArray(ctx, np.zeros(self.I, np.int8))

    def refresh_flags(self):
        """Host copy of firstTime_ (the branch decision of the next replan) after a commit."""
        self.first_time_h = self.first_time.get()
        return self.first_time_h

    def plans(self):
        """(plan_x [I][n], first_time [I], prev_count [I], valid [I]) on the host."""
        return self.plan_x.get()[: self.I], self.first_time.get(), self.prev_count.get(), self.valid.get()

    def close(self):
        for d in (self.plan_x, self.plan_states, self.prev_count, self.first_time, self.valid):
            d.free()


class DeviceReplan:
    """Device buffers and solver batches for I instances with K dynamic obstacles each
    (L prediction steps, horizon N = params.horizon): the two candidate shapes of the fan-out
    branch (K and K + 1 obstacles, 4 I and 2 I QPs at most) and the single-solve shapes (no
    obstacles; K current obstacles held over the horizon), each batch created once at its capacity
    and run over the replan's instances of that branch (impc_batch_set_active)."""

    def __init__(self, ctx, params, pd, I, K, L, settings):
        self.ctx, self.params, self.pd, self.I, self.K, self.L = ctx, params, pd, I, K, L
        self.N = params.horizon
        N = self.N
        self.n = 13 * N - 5
        self.settings = settings
        self.fan = dict(ob_idx=DeviceArray(ctx, (I,), np.int32), cand_type=DeviceArray(ctx, (I, 6), np.int32),
                        cand_slot=DeviceArray(ctx, (I, 6), np.int32), closest_prob=DeviceArray(ctx, (I, 4)),
                        single_pos=DeviceArray(ctx, (I, 4, K, L, 3)), single_size=DeviceArray(ctx, (I, 4, K, L, 3)),
                        pair_pos=DeviceArray(ctx, (I, 2, K + 1, L, 3)),
                        pair_size=DeviceArray(ctx, (I, 2, K + 1, L, 3)))
        self.sel = dict(x_cand=DeviceArray(ctx, (I, 6), np.uint64), dyn_count=DeviceArray(ctx, (I, 6), np.int32),
                        dyn_pos=DeviceArray(ctx, (I, 6, K + 1, L, 3)), dyn_size=DeviceArray(ctx, (I, 6, K + 1, L, 3)),
                        valid=DeviceArray(ctx, np.ones((I, 6), np.int8)), best_cand=DeviceArray(ctx, (I,), np.int32),
                        best_pos=DeviceArray(ctx, (I,), np.int32), scores=DeviceArray(ctx, (I, 6, 3)),
                        weighted=DeviceArray(ctx, (I, 6)))
        # fan-out shapes (single-intent K, two-intent K + 1), then the single-solve shapes
        self.shapes = [self._shape(K, 4 * I, L, 4), self._shape(K + 1, 2 * I, L, 2)]
        self.first_shape = self._shape(0, I, 1, 1)
        self.cur_shape = None  # K current obstacles over the horizon, created on first use
        self._limits = {}  # per batch: the time limits last uploaded (re-uploaded only on change)

    def _shape(self, kk, cap, L, rep):
        n, m, nnzP, nnzA = mpc_dims(self.params, 0, kk)
        pat = mpc_pattern(self.params, 0, kk)
        b = Batch(self.ctx, n, m, pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], cap)
        b.set_settings(self.settings)
        outs = [DeviceArray(self.ctx, (cap, k)) for k in (nnzP, n, nnzA, m, m)]
        return dict(K=kk, cap=cap, rep=rep, n=n, m=m, batch=b, builder=MpcBuilder(self.ctx, self.params, 0, kk, L),
                    vals=outs, ws=DeviceArray(self.ctx, (cap, n)), count=0)

    def _set_limits(self, sh, limits):
        """Per-QP time limits of a batch (capacity-padded), uploaded only when they change (the
        upload waits for every launch in flight)."""
        full = np.zeros(sh["cap"])
        full[: limits.size] = limits
        key = id(sh["batch"])
        if key not in self._limits or not np.array_equal(self._limits[key], full):
            sh["batch"].set_time_limits(full)
            self._limits[key] = full

    def _stage(self, sh, count, pos_d, vel_d, xref_d, lin_d, ws_src_ptr, ws_idx_d, dyn_pos_d=None, dyn_size_d=None):
        """Per-QP inputs of `count` instances, each repeated sh["rep"] times on the device: x0 rows,
        reference, linearisation point, warm start (gathered from the plan state), then the
        assembly into the batch.  Returns the per-candidate copies (freed by the caller)."""
        rep, nq = sh["rep"], count * sh["rep"]
        sh["count"] = nq
        if nq == 0:
            return []
        tmp = []
        srcs = []
        for d in (pos_d, vel_d, xref_d, lin_d):
            if d is None:
                srcs.append(None)
                continue
            if rep == 1:
                srcs.append(d)
                continue
            r = DeviceArray(self.ctx, (count * rep,) + tuple(d.shape[1:]))
            repeat_rows_device(self.ctx, d.ptr, count, d.nbytes // d.shape[0], rep, r.ptr)
            tmp.append(r)
            srcs.append(r)
        # warm start: the plan state's rows of these instances (row I: zeros), repeated
        ws1 = DeviceArray(self.ctx, (count, self.n))
        tmp.append(ws1)
        gather_rows_device(self.ctx, ws_src_ptr, 8 * self.n, ws_idx_d.ptr, count, ws1.ptr)
        repeat_rows_device(self.ctx, ws1.ptr, count, 8 * self.n, rep, sh["ws"].ptr)
        sh["builder"].build(nq, *[s.ptr if s is not None else None for s in srcs], None, None, None,
                            dyn_pos_d.ptr if dyn_pos_d is not None else None,
                            dyn_size_d.ptr if dyn_size_d is not None else None, *[v.ptr for v in sh["vals"]])
        b = sh["batch"]
        b.set_values_device(*[v.ptr for v in sh["vals"]])
        b.warm_start_device(sh["ws"].ptr, None)
        b.set_active(nq)
        return tmp

    def run(self, pos, vel, xref, prev=None, first_time=None, prev_count=None, dyn_cur=None, pred_pos=None,
            pred_size=None, prob=None, timings=None, solver_time_limit=None, t_start=None,
            issue_cutoff_s=ISSUE_CUTOFF_S, profile=False, state=None, has_pred=None, cur_size=None, cur_count=None):
        """One makePlanWithPred over all instances.  Inputs: pos, vel [I][3] (updateCurrStates);
        xref [I][N][8] or an impc.ReferencePaths (getXRef on the device, from `pos`); dyn_cur
        [I][K][3] (the current obstacle positions, predPos[.][0][0]); pred_pos / pred_size
        [I][K][4][L][3], prob [I][K][4] (updatePredObstacles); has_pred [I] (obPredPos_.size() != 0,
        default all); cur_size [I][K][3] + cur_count [I] (0 or K): the current dynamic obstacles a
        no-prediction instance keeps (updateDynamicObstacles; default none, as updatePredObstacles
        leaves them).  The planner state: `state` (a PlanState, updated in place: the plans are
        committed on the device), or host arrays prev [I][N][8] / first_time [I] / prev_count [I]
        for a one-off replan from that state (committed into a temporary state).

        Returns dict(branch [I], valid [I], best_cand [I] (fan-out instances; -1 otherwise),
        cand_type, cand_slot, ob_idx [I] (-1 for single-solve instances), inst_fanout / inst_first /
        inst_current (the instances of each branch, in batch-row order), x_single, x_pair,
        info_single, info_pair (rows of the fan-out instances' candidates), x_first, info_first,
        x_current, info_current, xref, issued, time_limit, vals_*).  Budget: see the module
        docstring; t_start is the replan's startTime (perf_counter seconds, default: entry to
        run).  profile: each candidate QP's device latency as lat_single / lat_pair."""
        I, K, L, N = self.I, self.K, self.L, self.N
        t = {}
        t0 = time.perf_counter()
        if t_start is None:
            t_start = t0
        own = state is None
        if own:
            state = PlanState(self.ctx, I, N, prev, first_time, prev_count)
        ft = state.first_time_h
        hp = np.ones(I, bool) if has_pred is None else np.asarray(has_pred).astype(bool).reshape(I)
        cc = None if cur_size is None else (np.full(I, K) if cur_count is None else np.asarray(cur_count).reshape(I))
        br = branches(ft, hp, cc)
        F, S0, S1 = [np.flatnonzero(br == v).astype(np.int64) for v in (FANOUT, SINGLE_FIRST, SINGLE_CURRENT)]
        nf, n0, n1 = F.size, S0.size, S1.size
        tmp = []

        def dev(a, dt=np.float64):
            d = DeviceArray(self.ctx, np.ascontiguousarray(a, dt))
            tmp.append(d)
            return d

        def gathered(src, idx_d, count, shape, dt=np.float64):
            d = DeviceArray(self.ctx, (count,) + tuple(shape), dt)
            tmp.append(d)
            gather_rows_device(self.ctx, src.ptr, int(np.prod(shape)) * np.dtype(dt).itemsize, idx_d.ptr, count, d.ptr)
            return d

        pos = np.asarray(pos, np.float64).reshape(I, 3)
        vel = np.asarray(vel, np.float64).reshape(I, 3)
        pos_all = dev(pos)
        if isinstance(xref, ReferencePaths):  # getXRef of every instance, each replan (:603)
            xref_d = DeviceArray(self.ctx, (I, N, 8))
            xref.xref_device(pos_all.ptr, xref_d.ptr)
        else:
            xref_d = DeviceArray(self.ctx, np.ascontiguousarray(xref, np.float64).reshape(I, N, 8))
        tmp.append(xref_d)
        # ---- fan-out branch inputs, compacted to its instances
        f = self.fan
        if nf:
            Fd = dev(F, np.int64)
            fin = [dev(pos[F]), dev(np.zeros(nf, np.int8), np.int8),
                   gathered(state.plan_states, Fd, nf, (N, 8)), gathered(state.prev_count, Fd, nf, (), np.int32),
                   dev(np.asarray(dyn_cur, np.float64).reshape(I, K, 3)[F]),
                   dev(np.asarray(pred_pos, np.float64).reshape(I, K, 4, L, 3)[F]),
                   dev(np.asarray(pred_size, np.float64).reshape(I, K, 4, L, 3)[F]),
                   dev(np.asarray(prob, np.float64).reshape(I, K, 4)[F])]
            vel_f, xref_f = dev(vel[F]), gathered(xref_d, Fd, nf, (N, 8))
        self.ctx.synchronize()
        t["upload_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        if nf:
            _check(lib.impc_intent_fanout_device(
                self.ctx.h, nf, K, L, N, *[_P(d.ptr) for d in fin],
                *[_P(f[k].ptr) for k in ("ob_idx", "cand_type", "cand_slot", "closest_prob", "single_pos",
                                         "single_size", "pair_pos", "pair_size")], None), "impc_intent_fanout_device")
            for sh, dp, ds in zip(self.shapes, ("single_pos", "pair_pos"), ("single_size", "pair_size")):
                tmp += self._stage(sh, nf, fin[0], vel_f, xref_f, fin[2], state.plan_x.ptr, Fd, f[dp], f[ds])
        else:
            for sh in self.shapes:
                sh["count"] = 0
        # ---- single-solve branch: first plan / no predictions
        if n0:
            S0d = dev(S0, np.int64)
            # firstTime_: no warm start (:487-508) -- gathered from the zero row I
            ws_idx = dev(np.where(ft[S0] != 0, I, S0).astype(np.int64), np.int64)
            tmp += self._stage(self.first_shape, n0, dev(pos[S0]), dev(vel[S0]), gathered(xref_d, S0d, n0, (N, 8)),
                               None, state.plan_x.ptr, ws_idx)
        else:
            self.first_shape["count"] = 0
        if n1:
            if self.cur_shape is None:
                self.cur_shape = self._shape(K, I, N, 1)
            S1d = dev(S1, np.int64)
            cp = np.asarray(dyn_cur, np.float64).reshape(I, K, 3)[S1]
            cs = np.asarray(cur_size, np.float64).reshape(I, K, 3)[S1]
            # updateDynamicObstacles: each obstacle's position / size repeated horizon_ times (:326-334)
            hold = lambda a: np.ascontiguousarray(np.broadcast_to(a[:, :, None, :], (n1, K, N, 3)))  # noqa: E731
            tmp += self._stage(self.cur_shape, n1, dev(pos[S1]), dev(vel[S1]), gathered(xref_d, S1d, n1, (N, 8)),
                               gathered(state.plan_states, S1d, n1, (N, 8)), state.plan_x.ptr, S1d, dev(hold(cp)),
                               dev(hold(cs)))
        elif self.cur_shape is not None:
            self.cur_shape["count"] = 0
        self.ctx.synchronize()
        elapsed = time.perf_counter() - t_start
        issued = elapsed < issue_cutoff_s
        time_limit = self.settings.time_limit
        if solver_time_limit is not None:
            time_limit = max(solver_time_limit - elapsed, solver_time_limit)
        # fan-out candidates carry the limit (never on a first plan: those take the single branch);
        # the single-solve branch runs solveTraj's default 1e10 s / none (:442-444): no limit
        for sh in self.shapes:
            if sh["count"]:
                self._set_limits(sh, np.full(sh["count"], time_limit))
        singles = [sh for sh in (self.first_shape, self.cur_shape) if sh is not None and sh["count"]]
        for sh in singles:
            self._set_limits(sh, np.zeros(sh["count"]))
        launch = [sh for sh in self.shapes if sh["count"] and issued] + singles
        for sh in launch:
            if profile:
                sh["batch"].set_profiling(True)
        results = {}
        if launch:
            solve_group([sh["batch"] for sh in launch])
            self.ctx.synchronize()
            for sh in launch:
                x, y, info = sh["batch"].get()
                c = sh["count"]
                results[id(sh)] = (x[:c], y[:c], info[:c], sh["batch"].qp_latency()[:c] if profile else None)
            for sh in launch:
                if profile:
                    sh["batch"].set_profiling(False)
        t["fanout_build_solve_s"] = time.perf_counter() - t0
        # ---- selection over the fan-out instances, on the device; then the commit
        t0 = time.perf_counter()
        sel = self.sel
        fan_issued = nf and issued
        if nf:
            slot = f["cand_slot"].get()[:nf]
            valid = (candidate_valid(slot, results[id(self.shapes[0])][2]["status_val"],
                                     results[id(self.shapes[1])][2]["status_val"]) if fan_issued
                     else np.zeros((nf, 6), np.int8))
            vfull = np.zeros((I, 6), np.int8)
            vfull[:nf] = valid
            sel["valid"].set(vfull)
            xs = [sh["batch"].device_results()[0] for sh in self.shapes]
            _check(lib.impc_fanout_candidates_device(
                self.ctx.h, nf, K, L, _P(f["cand_slot"].ptr), _P(f["single_pos"].ptr), _P(f["single_size"].ptr),
                _P(f["pair_pos"].ptr), _P(f["pair_size"].ptr), _P(xs[0]), self.shapes[0]["n"], _P(xs[1]),
                self.shapes[1]["n"], _P(sel["x_cand"].ptr), _P(sel["dyn_count"].ptr), _P(sel["dyn_pos"].ptr),
                _P(sel["dyn_size"].ptr), None), "impc_fanout_candidates_device")
            sp = SelectParams(horizon=N, num_candidates=6, max_dynamic=K + 1, pred_len=L, num_static=0, prev_len=N,
                              dynamic_safety_dist=self.pd["dynamic_safety_dist"],
                              static_safety_dist=self.pd["static_safety_dist"])
            _check(lib.impc_select_best_device(
                self.ctx.h, C.byref(sp), nf, _P(sel["x_cand"].ptr), _P(sel["valid"].ptr), _P(fin[1].ptr),
                _P(fin[2].ptr), _P(fin[3].ptr), _P(xref_f.ptr), None, None, _P(sel["dyn_count"].ptr),
                _P(sel["dyn_pos"].ptr), _P(sel["dyn_size"].ptr), _P(f["closest_prob"].ptr), _P(sel["best_cand"].ptr),
                _P(sel["best_pos"].ptr), _P(sel["scores"].ptr), _P(sel["weighted"].ptr), None),
                "impc_select_best_device")
            _check(lib.impc_replan_commit_device(
                self.ctx.h, N, self.n, nf, _P(Fd.ptr), _P(sel["x_cand"].ptr), 6, _P(sel["best_cand"].ptr), None, None,
                _P(state.plan_x.ptr), _P(state.plan_states.ptr), _P(state.prev_count.ptr), _P(state.first_time.ptr),
                _P(state.valid.ptr), None), "impc_replan_commit_device")
        for sh, idx_d in ((self.first_shape, S0d if n0 else None), (self.cur_shape, S1d if n1 else None)):
            if idx_d is None:
                continue
            x_d, _, info_d = sh["batch"].device_results()
            _check(lib.impc_replan_commit_device(
                self.ctx.h, N, self.n, sh["count"], _P(idx_d.ptr), None, 0, None, _P(x_d), _P(info_d),
                _P(state.plan_x.ptr), _P(state.plan_states.ptr), _P(state.prev_count.ptr), _P(state.first_time.ptr),
                _P(state.valid.ptr), None), "impc_replan_commit_device")
        self.ctx.synchronize()
        xref_used = xref_d.get()
        t["select_s"] = time.perf_counter() - t0
        best = np.full(I, -1, np.int32)
        ob = np.full(I, -1, np.int32)
        ctype = np.full((I, 6), -1, np.int32)
        cslot = np.full((I, 6), -1, np.int32)
        if nf:
            best[F] = sel["best_cand"].get()[:nf]
            ob[F] = f["ob_idx"].get()[:nf]
            ctype[F] = f["cand_type"].get()[:nf]
            cslot[F] = slot
        out = dict(branch=br, best_cand=best, ob_idx=ob, cand_type=ctype, cand_slot=cslot, inst_fanout=F,
                   inst_first=S0, inst_current=S1, xref=xref_used, issued=issued, time_limit=time_limit,
                   valid=state.valid.get())
        if nf:
            out["valid_cand"] = valid
        for sh, nm in ((self.shapes[0], "single"), (self.shapes[1], "pair"), (self.first_shape, "first"),
                       (self.cur_shape, "current")):
            r = results.get(id(sh)) if sh is not None else None
            out["x_" + nm], out["y_" + nm], out["info_" + nm] = (r[0], r[1], r[2]) if r is not None else (None,) * 3
            out["lat_" + nm] = r[3] if r is not None else None
            if sh is not None and sh["count"]:
                out["vals_" + nm] = [v.get()[: sh["count"]] for v in sh["vals"]]
        state.refresh_flags()
        if own:
            out["plan_x"] = state.plans()[0]
            state.close()
        for d in tmp:
            d.free()
        if timings is not None:
            timings.update(t)
        return out

    def close(self):
        for d in list(self.fan.values()) + list(self.sel.values()):
            d.free()
        for sh in self.shapes + [self.first_shape] + ([self.cur_shape] if self.cur_shape is not None else []):
            sh["batch"].close()
            sh["builder"].close()
            for v in sh["vals"] + [sh["ws"]]:
                v.free()
