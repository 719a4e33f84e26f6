"""makePlanWithPred (trajectory_planner mpcPlanner.cpp:571-661) for a batch of planning instances:
a ctypes mirror of the C-ABI entry point impc_replan_run (include/impc_replan.h), which runs the
whole replan on the device -- branch table, fan-out, assembly, ONE grouped solve, candidate
validity, scoring / selection and the commit of every plan into the planner state the replan
object keeps on the device.

Per instance, as the reference decides (:593-606):
  * fan-out branch -- not firstTime_ and predictions present (obPredPos_.size()): the intent fan-out
    (:663-769), the MPC -> QP assembly of the two candidate shapes (:891-1197), the candidates'
    solves (solveTraj with timeLimit), scoring / selection (:771-887); the chosen candidate is the
    plan (:629-639);
  * single-solve branch -- firstTime_ or no predictions (:645-659): ONE QP, no time limit, no
    scoring; its solution is the plan when solveTraj succeeds.  On a first plan the static and
    dynamic obstacles are cleared (:593-602), so the QP has no obstacle rows and no warm start
    (:487-508, firstTime_); otherwise it takes the instance's current dynamic obstacles, each
    position held over the horizon (updateDynamicObstacles :316-341) -- or none, when predictions
    were cleared (updatePredObstacles :364-371 clears them too, the live predictor loop's case).
An instance without a plan keeps its state (validTraj = false).

The replan's wall-clock budget (:609-628): candidate i is issued only while `time = now -
startTime < 0.15 s`, with `timeLimit = max(solverTimeLimit_ - time, solverTimeLimit_)`; a
candidate enters the selection only when solveTraj succeeded (initSolver and solveProblem NoError,
:475-478, :513-518 -- solve_traj_ok).  The batch issues all six candidates of every fan-out instance at one instant (after
the device-side assembly), so the cut-off is one check: past it no candidate is issued and every
fan-out instance selects nothing (best_cand -1, validTraj = false).

Every instance may track its own number of obstacles, K_i = num_pred[i] (0..K; predPos.size(),
updatePredObstacles :343-373).  The QPs of a replan are grouped by obstacle count: shape k holds
every QP with k obstacle rows per stage (first plans k = 0, current-obstacle solves k = c_i,
single-intent candidates K_i, two-intent candidates K_i + 1), one solver batch per shape, all in
one grouped launch whose per-shape QP counts the device decides and the solver reads from device
memory -- the library call never waits for the device and reads nothing back.  With num_static
S_st > 0 every QP not on a first plan also carries the instance's S_st static obstacles
(obclustering_->getStaticObstacles(), :594; scored by getTrajectoryScore too) and the first plans
move to shape K + 2.

Everything here beyond impc_replan_run / impc_replan_set_state (input uploads, the per-shape
results and assembled values of run()'s return dict) is test plumbing.
"""
import ctypes as C
import time

import numpy as np

from . import (INFO_DTYPE, DeviceArray, MpcParams, ReferencePaths, Settings, _check, _P, lib,
               QUEUE_FIFO)

ISSUE_CUTOFF_S = 0.15  # makePlanWithPred: no candidate is issued 0.15 s after the replan started (:613)
FANOUT, SINGLE_FIRST, SINGLE_CURRENT = 0, 1, 2  # IMPC_REPLAN_* (run()["branch"])
ROW_FIRST, ROW_CURRENT = 6, 7  # impc_replan_shape row codes (0..3 single-intent slot, 4..5 two-intent slot)
CATEGORIES = ("single", "pair", "first", "current")  # the per-kind views of results()
UNSOLVED = -10


class ReplanConfig(C.Structure):
    """impc_replan_config (include/impc_replan.h)."""
    _fields_ = [("instances", C.c_int64), ("num_obstacles", C.c_int32), ("pred_len", C.c_int32),
                ("mpc", MpcParams), ("settings", Settings), ("issue_cutoff_s", C.c_double),
                ("queue_order", C.c_int32), ("num_static", C.c_int32)]


class ReplanInputs(C.Structure):
    """impc_replan_inputs: device pointers + the budget."""
    _fields_ = [(k, C.c_void_p) for k in ("pos", "vel", "xref", "dyn_cur", "pred_pos", "pred_size", "prob", "has_pred",
                                          "cur_size", "cur_count")] + \
               [("solver_time_limit", C.c_double), ("elapsed_s", C.c_double), ("num_pred", C.c_void_p),
                ("st_centroid", C.c_void_p), ("st_size", C.c_void_p), ("st_yaw", C.c_void_p)]


class ReplanStats(C.Structure):
    _fields_ = [("fanout", C.c_int64), ("single_first", C.c_int64), ("single_current", C.c_int64),
                ("issued", C.c_int32), ("reserved", C.c_int32), ("time_limit", C.c_double), ("stage_s", C.c_double),
                ("total_s", C.c_double)]


class ReplanView(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("plan_x", "plan_states", "prev_count", "first_time", "valid", "branch",
                                          "best_cand", "ob_idx", "cand_type", "cand_slot", "num_obs", "slot_row",
                                          "shape")]


def _sig(name, *args):
    f = getattr(lib, name)
    f.restype = C.c_int
    f.argtypes = list(args)


_sig("impc_replan_create", _P, C.POINTER(ReplanConfig), C.POINTER(_P))
_sig("impc_replan_destroy", _P)
_sig("impc_replan_set_state", _P, _P, _P)
_sig("impc_replan_run", _P, C.POINTER(ReplanInputs))
_sig("impc_replan_get_stats", _P, C.POINTER(ReplanStats))
_sig("impc_replan_view_device", _P, C.POINTER(ReplanView))
_sig("impc_replan_advance_device", _P, C.c_double, _P, _P)
_sig("impc_replan_shape", _P, C.c_int32, C.POINTER(_P), C.POINTER(C.c_int64), C.POINTER(_P), C.POINTER(_P),
     C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), C.POINTER(_P))


def solve_traj_ok(info):
    """solveTraj's successSolve per solved QP (host restatement of impc_lib::solve_traj_ok,
    mpcPlanner.cpp:475-478, :513-518): initSolver succeeded (setup_exitflag 0) and solveProblem
    returned NoError -- osqp_solve's exitflag, 0 for every final status (infeasible and a diverged
    NON_CVX included, x = OSQP_NAN) and 1 only after a failed adaptive-rho refactorisation (status
    left UNSOLVED)."""
    info = np.asarray(info)
    return (info["setup_exitflag"] == 0) & (info["status_val"] != UNSOLVED)


def candidate_valid(cand_slot, info_single, info_pair):
    """valid[i][c] of the selection (host restatement of the library's k_cand): candidate c of
    fan-out instance i succeeded (solve_traj_ok).  Candidate c sits at row 4i+slot of the
    single-intent rows (slot < 4) or 2i+slot-4 of the two-intent rows."""
    slot = np.asarray(cand_slot)
    ii = np.arange(slot.shape[0])[:, None]
    ok_s, ok_p = solve_traj_ok(info_single), solve_traj_ok(info_pair)
    return np.where(slot < 4, ok_s[4 * ii + np.minimum(slot, 3)], ok_p[2 * ii + np.clip(slot - 4, 0, 1)]).astype(np.int8)


def assemble(per_inst, shapes):
    """The per-kind views of one replan from its per-shape rows (shapes[k] = dict(x, y, info[, vals,
    lat]) of the rows shape k solved) and the per-instance outputs (branch, num_obs, slot_row, shape
    -- the single solve's shape, = num_obs without static obstacles):
    x_<kind>, y_<kind>, info_<kind>, vals_<kind>, lat_<kind> for the kinds single (the single-intent
    candidates, row 4 j + slot of the j-th fan-out instance), pair (two-intent, 2 j + slot - 4),
    first and current (row j of the j-th instance on that branch).  x and info are arrays; y and
    vals are arrays when every row has the same m (one obstacle count), else per-row lists.  A kind
    with no solved row is None.  Also cand_rows [I][6] = (shape, row) of candidate c (getIntentComb
    order) and single_rows [I] = (shape, row)."""
    br, K, R = per_inst["branch"], per_inst["num_obs"], per_inst["slot_row"]
    SH = per_inst.get("shape", K)
    I = br.shape[0]
    out = {"inst_fanout": np.flatnonzero(br == FANOUT), "inst_first": np.flatnonzero(br == SINGLE_FIRST),
           "inst_current": np.flatnonzero(br == SINGLE_CURRENT)}
    rows = {"single": [(int(K[i]), int(R[i, s])) for i in out["inst_fanout"] for s in range(4)],
            "pair": [(int(K[i]) + 1, int(R[i, s])) for i in out["inst_fanout"] for s in (4, 5)],
            "first": [(int(SH[i]), int(R[i, 0])) for i in out["inst_first"]],
            "current": [(int(SH[i]), int(R[i, 0])) for i in out["inst_current"]]}
    for nm in CATEGORIES:
        rr = rows[nm]
        ok = bool(rr) and all(k in shapes and r < shapes[k]["x"].shape[0] for k, r in rr)
        for key in ("x", "y", "info", "vals", "lat"):
            if not ok or shapes[rr[0][0]].get(key) is None:
                out[f"{key}_{nm}"] = None
                continue
            if key == "vals":
                parts = [[v[r] for v in shapes[k]["vals"]] for k, r in rr]
                same = len({k for k, _ in rr}) == 1
                out[f"vals_{nm}"] = [np.stack([p[j] for p in parts]) for j in range(5)] if same else parts
                continue
            parts = [shapes[k][key][r] for k, r in rr]
            same = key in ("x", "info", "lat") or len({k for k, _ in rr}) == 1
            out[f"{key}_{nm}"] = np.stack(parts) if same else parts
    slot = per_inst.get("cand_slot")
    out["cand_rows"] = [[((int(K[i]) + (1 if slot[i, c] >= 4 else 0)), int(R[i, slot[i, c]])) for c in range(6)]
                        if br[i] == FANOUT else None for i in range(I)] if slot is not None else None
    out["single_rows"] = [(int(SH[i]), int(R[i, 0])) if br[i] != FANOUT else None for i in range(I)]
    return out


def branches(first_time, has_pred, cur_count=None):
    """The makePlanWithPred branch of every instance (:606; host restatement of k_branch_table):
    FANOUT when not firstTime_ and predictions are present, else SINGLE_CURRENT when not firstTime_
    and current dynamic obstacles are present (cur_count > 0), else SINGLE_FIRST."""
    ft = np.asarray(first_time).astype(bool)
    hp = np.asarray(has_pred).astype(bool)
    cur = np.zeros_like(ft) if cur_count is None else np.asarray(cur_count) > 0
    return np.where(~ft & hp, FANOUT, np.where(~ft & cur, SINGLE_CURRENT, SINGLE_FIRST)).astype(np.int8)


def _get(ctx, ptr, shape, dtype):
    out = np.empty(shape, dtype)
    if out.nbytes:
        _check(lib.impc_copy_to_host(ctx.h, out.ctypes.data_as(_P), _P(ptr), out.nbytes), "impc_copy_to_host")
    return out


class DeviceReplan:
    """impc_replan: I planning instances with K dynamic obstacles each (L prediction steps, horizon
    N = params.horizon) and num_static static obstacles each; the planner state lives in the object
    on the device."""

    def __init__(self, ctx, params, pd, I, K, L, settings, issue_cutoff_s=ISSUE_CUTOFF_S, queue_order=QUEUE_FIFO,
                 num_static=0):
        self.ctx, self.params, self.pd, self.I, self.K, self.L = ctx, params, pd, int(I), int(K), int(L)
        self.S_st = int(num_static)
        self.num_shapes = self.K + 2 + (1 if self.S_st else 0)
        self.N = params.horizon
        self.n = 13 * self.N - 5
        self.settings = settings
        cfg = ReplanConfig(instances=self.I, num_obstacles=self.K, pred_len=self.L, mpc=params, settings=settings,
                           issue_cutoff_s=issue_cutoff_s, queue_order=queue_order, num_static=self.S_st)
        h = _P()
        _check(lib.impc_replan_create(ctx.h, C.byref(cfg), C.byref(h)), "impc_replan_create")
        self.h = h
        self.first_time_h = np.ones(self.I, np.int8)

    # ---- planner state
    def set_state(self, prev=None, first_time=None, prev_controls=None):
        """impc_replan_set_state from host arrays: prev [I][N][8] (currentStatesSol_), prev_controls
        [I][N-1][5] (currentControlsSol_; zeros if None), first_time [I] (all 1 if None)."""
        px = None
        if prev is not None:
            px = np.zeros((self.I, self.n))
            px[:, : 8 * self.N] = np.asarray(prev, np.float64).reshape(self.I, 8 * self.N)
            if prev_controls is not None:
                px[:, 8 * self.N:] = np.asarray(prev_controls, np.float64).reshape(self.I, -1)
        ft = None if first_time is None else np.ascontiguousarray(first_time, np.int8).reshape(self.I)
        _check(lib.impc_replan_set_state(self.h, None if px is None else px.ctypes.data_as(_P),
                                         None if ft is None else ft.ctypes.data_as(_P)), "impc_replan_set_state")
        self.first_time_h = np.ones(self.I, np.int8) if ft is None else ft.copy()

    def view(self):
        v = ReplanView()
        _check(lib.impc_replan_view_device(self.h, C.byref(v)), "impc_replan_view_device")
        return v

    def plans(self):
        """(plan_x [I][n], first_time [I], prev_count [I], valid [I]) on the host."""
        v = self.view()
        I = self.I
        return (_get(self.ctx, v.plan_x, (I + 1, self.n), np.float64)[:I], _get(self.ctx, v.first_time, I, np.int8),
                _get(self.ctx, v.prev_count, I, np.int32), _get(self.ctx, v.valid, I, np.int8))

    # ---- one replan
    def run_device(self, pos, vel, xref, dyn_cur, pred_pos, pred_size, prob, has_pred=None, cur_size=None,
                   cur_count=None, solver_time_limit=0.0, elapsed_s=0.0, num_pred=None, st_centroid=None,
                   st_size=None, st_yaw=None):
        """impc_replan_run on device addresses (ints); the product call."""
        inp = ReplanInputs(pos=pos, vel=vel, xref=xref, dyn_cur=dyn_cur, pred_pos=pred_pos, pred_size=pred_size,
                           prob=prob, has_pred=has_pred, cur_size=cur_size, cur_count=cur_count,
                           solver_time_limit=float(solver_time_limit or 0.0), elapsed_s=float(elapsed_s),
                           num_pred=num_pred, st_centroid=st_centroid, st_size=st_size, st_yaw=st_yaw)
        _check(lib.impc_replan_run(self.h, C.byref(inp)), "impc_replan_run")

    def advance_device(self, t, pos_ptr, vel_ptr):
        """impc_replan_advance_device: pos / vel [I][3] (device) = getPos(t) / getVel(t) of every
        instance with a plan (mpc_node.cpp:216-224)."""
        _check(lib.impc_replan_advance_device(self.h, float(t), _P(pos_ptr), _P(vel_ptr)), "impc_replan_advance_device")

    def stats(self):
        s = ReplanStats()
        _check(lib.impc_replan_get_stats(self.h, C.byref(s)), "impc_replan_get_stats")
        return {f: getattr(s, f) for f, _ in ReplanStats._fields_}

    def shape(self, k):
        """impc_replan_shape k (dynamic-obstacle count 0 .. K + 1; K + 2: the first plans with static
        obstacles): (batch handle, QP count solved, row_inst
        and row_code device pointers, device value pointers)."""
        b, cnt, ri, rc = _P(), C.c_int64(), _P(), _P()
        ptrs = [_P() for _ in range(5)]
        _check(lib.impc_replan_shape(self.h, k, C.byref(b), C.byref(cnt), C.byref(ri), C.byref(rc),
                                     *[C.byref(p) for p in ptrs]), "impc_replan_shape")
        return b.value, cnt.value, ri.value, rc.value, [p.value for p in ptrs]

    def _shape_results(self, k, with_values, profile=False):
        """Host copies of shape k's last results (its solved rows) -- inspection for tests."""
        b, cnt, ri, rc, ptrs = self.shape(k)
        if not cnt:
            return None
        st = self._stats_of(b)
        n, m = st["n"], st["m"]
        x = np.empty((st["batch"], n))
        y = np.empty((st["batch"], max(m, 1)))
        info = np.empty(st["batch"], INFO_DTYPE)
        _check(lib.impc_batch_get(_P(b), x.ctypes.data_as(C.POINTER(C.c_double)),
                                  y.ctypes.data_as(C.POINTER(C.c_double)), info.ctypes.data_as(_P)), "impc_batch_get")
        out = dict(x=x[:cnt], y=y[:cnt, :m], info=info[:cnt], row_inst=_get(self.ctx, ri, cnt, np.int32),
                   row_code=_get(self.ctx, rc, cnt, np.int8), batch=b)
        if with_values:
            out["vals"] = [_get(self.ctx, p, (cnt, ln), np.float64)
                           for p, ln in zip(ptrs, (st["nnzP"], n, st["nnzA"], m, m))]
        if profile:
            ms = np.empty(st["batch"])
            _check(lib.impc_batch_get_qp_latency(_P(b), ms.ctypes.data_as(C.POINTER(C.c_double))),
                   "impc_batch_get_qp_latency")
            out["lat"] = ms[:cnt]
        return out

    @staticmethod
    def _stats_of(bh):
        from . import Stats
        s = Stats()
        _check(lib.impc_batch_get_stats(_P(bh), C.byref(s)), "impc_batch_get_stats")
        return {f: getattr(s, f) for f, _ in Stats._fields_}

    def run(self, pos, vel, xref, prev=None, first_time=None, prev_count=None, dyn_cur=None, pred_pos=None,
            pred_size=None, prob=None, timings=None, solver_time_limit=None, t_start=None, profile=False,
            has_pred=None, cur_size=None, cur_count=None, values=True, num_pred=None, static=None):
        """One makePlanWithPred over all instances from host arrays (uploaded here; test plumbing
        around impc_replan_run).  Inputs: pos, vel [I][3]; xref [I][N][8] or an
        impc.ReferencePaths (getXRef on the device, from `pos`); dyn_cur [I][K][3]; pred_pos /
        pred_size [I][K][4][L][3], prob [I][K][4]; has_pred [I] (default all); num_pred [I] (K_i,
        0..K: each instance's first K_i obstacle slots; default K); cur_size [I][K][3] + cur_count [I]
        (0..K): the current dynamic obstacles a no-prediction instance keeps (default none).  static =
        (centroid [I][S_st][3], size [I][S_st][3], yaw [I][S_st]) with num_static > 0.  prev [I][N][8] / first_time [I]: when given, the planner state is set
        from them first (impc_replan_set_state; prev_count is implied -- 0 on a first plan, N
        otherwise -- and checked when passed); else the replan continues from the committed state.

        Returns dict(branch [I], valid [I], best_cand [I], cand_type, cand_slot, ob_idx [I], num_obs,
        slot_row, inst_fanout / inst_first / inst_current, x_* / y_* / info_* / vals_* (lat_* with
        profile) for the kinds single, pair, first, current (assemble(); None when a kind did not
        run), shapes, cand_rows, single_rows, xref, issued, time_limit).  t_start: the replan's startTime (perf_counter seconds)."""
        I, K, L, N = self.I, self.K, self.L, self.N
        t0 = time.perf_counter()
        if t_start is None:
            t_start = t0
        if prev is not None or first_time is not None:
            ft = np.ones(I, np.int8) if first_time is None else np.asarray(first_time, np.int8).reshape(I)
            if prev_count is not None:  # currentStatesSol_.size() is N once a plan exists, else 0
                pc = np.asarray(prev_count).reshape(I)
                assert ((pc == N) | (ft != 0)).all(), "a planner past its first plan holds a full plan (prev_count N)"
            self.set_state(prev, ft)
        tmp = []

        def dev(a, dt=np.float64):
            d = DeviceArray(self.ctx, np.ascontiguousarray(a, dt))
            tmp.append(d)
            return d.ptr

        pos = np.asarray(pos, np.float64).reshape(I, 3)
        pos_d = dev(pos)
        if isinstance(xref, ReferencePaths):  # getXRef of every instance, each replan (:603)
            xd = DeviceArray(self.ctx, (I, N, 8))
            tmp.append(xd)
            xref.xref_device(pos_d, xd.ptr)
            xref_d = xd.ptr
        else:
            xd = None
            xref_d = dev(np.asarray(xref, np.float64).reshape(I, N, 8))
        args = dict(pos=pos_d, vel=dev(np.asarray(vel).reshape(I, 3)), xref=xref_d,
                    dyn_cur=dev(np.asarray(dyn_cur).reshape(I, K, 3)),
                    pred_pos=dev(np.asarray(pred_pos).reshape(I, K, 4, L, 3)),
                    pred_size=dev(np.asarray(pred_size).reshape(I, K, 4, L, 3)),
                    prob=dev(np.asarray(prob).reshape(I, K, 4)),
                    has_pred=None if has_pred is None else dev(np.asarray(has_pred).reshape(I), np.int8),
                    cur_size=None if cur_size is None else dev(np.asarray(cur_size).reshape(I, K, 3)),
                    cur_count=None if (cur_size is None or cur_count is None) else dev(np.asarray(cur_count).reshape(I),
                                                                                      np.int32),
                    num_pred=None if num_pred is None else dev(np.asarray(num_pred).reshape(I), np.int32))
        if self.S_st:
            assert static is not None, "num_static > 0: static = (centroid, size, yaw) per instance"
            S = self.S_st
            args.update(st_centroid=dev(np.asarray(static[0]).reshape(I, S, 3)),
                        st_size=dev(np.asarray(static[1]).reshape(I, S, 3)),
                        st_yaw=dev(np.asarray(static[2]).reshape(I, S)))
        self.ctx.synchronize()
        t_up = time.perf_counter() - t0
        batches = [self.shape(k)[0] for k in range(self.num_shapes)]
        if profile:
            for b in batches:
                if b:
                    _check(lib.impc_batch_set_profiling(_P(b), 1), "impc_batch_set_profiling")
        t1 = time.perf_counter()
        self.run_device(**args, solver_time_limit=solver_time_limit or 0.0, elapsed_s=t1 - t_start)
        self.ctx.synchronize()
        t_run = time.perf_counter() - t1
        st = self.stats()
        out = self.results(values, profile)
        out["xref"] = xd.get() if xd is not None else np.asarray(xref, np.float64).reshape(I, N, 8)
        if profile:
            for b in batches:
                if b:
                    _check(lib.impc_batch_set_profiling(_P(b), 0), "impc_batch_set_profiling")
        for d in tmp:
            d.free()
        if timings is not None:
            timings.update(upload_s=t_up, run_s=t_run, stage_s=st["stage_s"], call_s=st["total_s"])
        return out

    def results(self, values=True, profile=False):
        """Host copies of the last replan's per-instance outputs, state and per-shape results
        (test / tool inspection after the call)."""
        I = self.I
        st = self.stats()
        v = self.view()
        out = dict(branch=_get(self.ctx, v.branch, I, np.int8), best_cand=_get(self.ctx, v.best_cand, I, np.int32),
                   ob_idx=_get(self.ctx, v.ob_idx, I, np.int32), cand_type=_get(self.ctx, v.cand_type, (I, 6), np.int32),
                   cand_slot=_get(self.ctx, v.cand_slot, (I, 6), np.int32), valid=_get(self.ctx, v.valid, I, np.int8),
                   num_obs=_get(self.ctx, v.num_obs, I, np.int32), slot_row=_get(self.ctx, v.slot_row, (I, 6), np.int32),
                   shape=_get(self.ctx, v.shape, I, np.int32),
                   issued=bool(st["issued"]), time_limit=st["time_limit"])
        shapes = {}
        for k in range(self.num_shapes):
            r = self._shape_results(k, values, profile)
            if r:
                shapes[k] = r
        out["shapes"] = shapes
        out.update(assemble(out, shapes))
        self.first_time_h = _get(self.ctx, v.first_time, I, np.int8)
        return out

    def close(self):
        if self.h:
            lib.impc_replan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
