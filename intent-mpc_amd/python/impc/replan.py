"""makePlanWithPred (trajectory_planner mpcPlanner.cpp:571-661) for a batch of planning instances,
with every stage on the device: the intent fan-out (impc_intent_fanout_device, :663-769), the
MPC -> QP assembly of the two candidate shapes (impc_mpc_build_values_device, :891-1197), one
grouped solve of all candidate QPs (impc_batch_solve_group, the OSQP call of solveTraj) and the
candidate scoring / selection (impc_select_best, :771-887).

Host work is limited to the per-candidate repetition of the instance inputs (every candidate of
a replan is linearised at the same previous plan); the candidate table of the selection is built
on the device (impc_fanout_candidates_device).

The replan's wall-clock budget (mpcPlanner.cpp:609-628): the reference issues candidate i only
while `time = now - startTime < 0.15 s` and solves it with
`timeLimit = max(solverTimeLimit_ - time, solverTimeLimit_)` (solver_time_limit, 0.05 s by
default, :166-167); a candidate enters the selection only when solveTraj succeeded, i.e.
solveProblem returned NoError (:513-518) -- every status but a non-convex problem.  The batch
issues all six candidates of every instance at one instant, so the cut-off is one check before
the grouped solve: past it no candidate is issued and every instance selects nothing
(best_cand -1, the reference's validTraj = false).  solveTraj sets the time limit only when not
firstTime_ (:442-444), so the candidates of an instance with first_time set carry none (per-QP
limits, impc_batch_set_time_limits).  (The reference does not fan out a firstTime_ instance at
all -- it takes the single-solve branch :645-659; this class is the fan-out branch, and a
first_time instance's candidates are solved without a limit, as that branch's solve is.)
"""
import ctypes as C
import time

import numpy as np

from . import (NON_CVX, Batch, DeviceArray, MpcBuilder, ReferencePaths, SelectParams, _P, _check, lib,
               mpc_dims, mpc_pattern, repeat_rows_device, solve_group)

ISSUE_CUTOFF_S = 0.15  # makePlanWithPred: no candidate is issued 0.15 s after the replan started (:613)


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


class DeviceReplan:
    """Device buffers and solver batches for I instances with K dynamic obstacles each
    (L prediction steps, horizon N = params.horizon)."""

    def __init__(self, ctx, params, pd, I, K, L, settings):
        self.ctx, self.params, self.pd, self.I, self.K, self.L = ctx, params, pd, I, K, L
        self.N = params.horizon
        N = self.N
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
        self.shapes = []
        for kk, nb in ((K, 4 * I), (K + 1, 2 * I)):
            n, m, nnzP, nnzA = mpc_dims(params, 0, kk)
            pat = mpc_pattern(params, 0, kk)
            b = Batch(ctx, n, m, pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], nb)
            b.set_settings(settings)
            outs = [DeviceArray(ctx, (nb, k)) for k in (nnzP, n, nnzA, m, m)]
            self.shapes.append(dict(K=kk, nb=nb, n=n, m=m, batch=b, builder=MpcBuilder(ctx, params, 0, kk, L),
                                    vals=outs))

    def run(self, pos, vel, xref, prev, first_time, prev_count, dyn_cur, pred_pos, pred_size, prob, timings=None,
            solver_time_limit=None, t_start=None, issue_cutoff_s=ISSUE_CUTOFF_S, profile=False):
        """Returns dict(best_cand, cand_type, cand_slot, ob_idx, x_single, x_pair, info_single, info_pair,
        xref, issued, time_limit, valid).  xref: the reference of every instance [I][N][8], or an
        impc.ReferencePaths -- the instances' input paths and reference-tracking state, whose
        getReferenceTraj / getXRef then runs on the device (mpcPlanner.cpp:968-981, 1199-1231) from
        `pos`.  Budget (module docstring): t_start is the replan's startTime (perf_counter seconds,
        default: entry to run); solver_time_limit, when given, is solverTimeLimit_ and sets every
        candidate's OSQP time_limit to max(limit - elapsed, limit) -- on instances whose first_time is
        0 -- and the settings' own time_limit applies otherwise.  When the cut-off has passed, x_* /
        info_* are None.  profile: also return each candidate QP's device latency (ms, from the
        tick its time limit counts from) as lat_single / lat_pair."""
        I, K, L, N = self.I, self.K, self.L, self.N
        t = {}
        t0 = time.perf_counter()
        if t_start is None:
            t_start = t0
        din = [DeviceArray(self.ctx, np.ascontiguousarray(a, dt)) for a, dt in
               ((pos, np.float64), (first_time, np.int8), (prev, np.float64), (prev_count, np.int32),
                (dyn_cur, np.float64), (pred_pos, np.float64), (pred_size, np.float64), (prob, np.float64))]
        if isinstance(xref, ReferencePaths):
            xref_d = DeviceArray(self.ctx, (I, N, 8))
            xref.xref_device(din[0].ptr, xref_d.ptr)
        else:
            xref_d = DeviceArray(self.ctx, np.ascontiguousarray(xref, np.float64))
        vel_d = DeviceArray(self.ctx, np.ascontiguousarray(vel, np.float64))
        # per-candidate copies of the instance inputs on the device: 4 single-intent, 2 two-intent
        rep = {}
        for cnt in (4, 2):
            rep[cnt] = []
            for d in (din[0], vel_d, xref_d, din[2]):
                r = DeviceArray(self.ctx, (I * cnt,) + tuple(d.shape[1:]))
                repeat_rows_device(self.ctx, d.ptr, I, d.nbytes // I, cnt, r.ptr)
                rep[cnt].append(r)
        x_ws = {cnt: np.repeat(np.concatenate([prev.reshape(I, -1), np.zeros((I, 5 * (N - 1)))], axis=1), cnt, axis=0)
                for cnt in (4, 2)}
        for sh, cnt in zip(self.shapes, (4, 2)):
            sh["batch"].warm_start(x_ws[cnt], None)
        self.ctx.synchronize()
        t["upload_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        f = self.fan
        _check(lib.impc_intent_fanout_device(
            self.ctx.h, I, K, L, prev.shape[1], *[_P(d.ptr) for d in din],
            *[_P(f[k].ptr) for k in ("ob_idx", "cand_type", "cand_slot", "closest_prob", "single_pos",
                                     "single_size", "pair_pos", "pair_size")], None), "impc_intent_fanout_device")
        for sh, cnt, dp, ds in zip(self.shapes, (4, 2), ("single_pos", "pair_pos"), ("single_size", "pair_size")):
            r = rep[cnt]
            sh["builder"].build(sh["nb"], r[0].ptr, r[1].ptr, r[2].ptr, r[3].ptr, None, None, None, f[dp].ptr,
                                f[ds].ptr, *[v.ptr for v in sh["vals"]])
            sh["batch"].set_values_device(*[sh["vals"][k].ptr for k in (0, 1, 2, 3, 4)])
        self.ctx.synchronize()
        elapsed = time.perf_counter() - t_start
        issued = elapsed < issue_cutoff_s
        time_limit = self.settings.time_limit
        if solver_time_limit is not None:
            time_limit = max(solver_time_limit - elapsed, solver_time_limit)
        limited = np.asarray(first_time).reshape(I) == 0  # setTimeLimit only when not firstTime_ (:442-444)
        for sh, cnt in zip(self.shapes, (4, 2)):
            sh["batch"].set_settings(self.settings)
            sh["batch"].set_time_limits(np.repeat(np.where(limited, time_limit, 0.0), cnt))
            sh["batch"].set_profiling(profile)
        results = lat = None
        if issued:
            solve_group([sh["batch"] for sh in self.shapes])
            self.ctx.synchronize()
            results = [sh["batch"].get() for sh in self.shapes]
            if profile:
                lat = [sh["batch"].qp_latency() for sh in self.shapes]
        # candidate c of instance i sits at row 4i+slot of the single-intent batch (slot < 4) or
        # 2i+slot-4 of the two-intent batch (fanout.hpp k_fanout_candidates)
        slot = f["cand_slot"].get()
        valid = (candidate_valid(slot, results[0][2]["status_val"], results[1][2]["status_val"]) if issued
                 else np.zeros((I, 6), np.int8))
        self.sel["valid"].set(valid)
        t["fanout_build_solve_s"] = time.perf_counter() - t0
        # selection, on the device: the candidate table (solution pointers, obstacle sets in the
        # selection's padded layout) from the fan-out outputs, then scoring + evaluateTraj
        t0 = time.perf_counter()
        sel = self.sel
        xs = [sh["batch"].device_results()[0] for sh in self.shapes]
        _check(lib.impc_fanout_candidates_device(
            self.ctx.h, I, K, L, _P(f["cand_slot"].ptr), _P(f["single_pos"].ptr), _P(f["single_size"].ptr),
            _P(f["pair_pos"].ptr), _P(f["pair_size"].ptr), _P(xs[0]), self.shapes[0]["n"], _P(xs[1]),
            self.shapes[1]["n"], _P(sel["x_cand"].ptr), _P(sel["dyn_count"].ptr), _P(sel["dyn_pos"].ptr),
            _P(sel["dyn_size"].ptr), None), "impc_fanout_candidates_device")
        sp = SelectParams(horizon=N, num_candidates=6, max_dynamic=K + 1, pred_len=L, num_static=0,
                          prev_len=prev.shape[1], dynamic_safety_dist=self.pd["dynamic_safety_dist"],
                          static_safety_dist=self.pd["static_safety_dist"])
        _check(lib.impc_select_best_device(
            self.ctx.h, C.byref(sp), I, _P(sel["x_cand"].ptr), _P(sel["valid"].ptr), _P(din[1].ptr),
            _P(din[2].ptr), _P(din[3].ptr), _P(xref_d.ptr), None, None, _P(sel["dyn_count"].ptr),
            _P(sel["dyn_pos"].ptr), _P(sel["dyn_size"].ptr), _P(f["closest_prob"].ptr), _P(sel["best_cand"].ptr),
            _P(sel["best_pos"].ptr), _P(sel["scores"].ptr), _P(sel["weighted"].ptr), None),
            "impc_select_best_device")
        self.ctx.synchronize()
        xref_used = xref_d.get()
        din += [xref_d, vel_d]
        t["select_s"] = time.perf_counter() - t0
        for d in din + rep[4] + rep[2]:
            d.free()
        if timings is not None:
            timings.update(t)
        out = dict(best_cand=sel["best_cand"].get(), cand_type=f["cand_type"].get(), cand_slot=slot,
                   ob_idx=f["ob_idx"].get(), xref=xref_used, issued=issued, time_limit=time_limit, valid=valid)
        for k, (sh, nm) in enumerate(zip(self.shapes, ("single", "pair"))):
            out["x_" + nm], out["info_" + nm] = (results[k][0], results[k][2]) if issued else (None, None)
            out["lat_" + nm] = lat[k] if lat is not None else None
            out["vals_" + nm] = [v.get() for v in sh["vals"]]
        return out

    def close(self):
        for d in list(self.fan.values()) + list(self.sel.values()):
            d.free()
        for sh in self.shapes:
            sh["batch"].close()
            sh["builder"].close()
            for v in sh["vals"]:
                v.free()
