"""polyTrajSolver (trajectory_planner polyTrajSolver.cpp) for a batch of paths on the device.

The reference keeps three persistent OsqpEigen solvers (x, y, z) per planner: setUpProblem
(:162-223) builds P, q = 0, A and the per-axis bounds once per path, updateProblem (:225-238)
only refreshes the bounds (updateBounds) on later solves, and solveX/Y/Z (:870-905) rescale the
normalised-time coefficients to real time.  Here the three axes of every path are one batch of
3 * nb QPs (shared pattern: all QPs of a path count have the same P / A structure), solved on
the generic kernel with its workspace kept between solves, so updateProblem is
impc_batch_update_bounds.

Corridor constraints (setCorridorConstraint, :960-1012): `corridor_size` [nb][W-1] (0 = none on a
segment) and `corridor_res` add one row per sample of each segment; corridor_num(...) gives each
path's numCorridor vector, and a batch holds paths with one vector (it fixes the pattern).
"""
import ctypes as C

import numpy as np

from . import Batch, Dims, MinsnapParams, _check, _d, _i, _i32p, lib

LIVE = dict(poly_degree=7, diff_degree=4, continuity_degree=3, desired_vel=1.0, soft_constraint=0,
            sc_deviation=(0.0, 0.0, 0.0))  # planner_param.yaml:11-14 (poly_traj/*)


def params(**kw):
    d = dict(LIVE)
    d.update(kw)
    p = MinsnapParams()
    for k, v in d.items():
        if k == "sc_deviation":
            p.sc_deviation[:] = list(v)
        else:
            setattr(p, k, v)
    return p


def _cn(cnum, W):
    if cnum is None:
        return None, None
    a = np.ascontiguousarray(cnum, np.int32)
    if a.shape != (W - 1,):
        raise ValueError(f"corridor_num has shape {a.shape}, expected ({W - 1},)")
    return a, a.ctypes.data_as(_i32p)


def corridor_num(p, path, corridor_size, corridor_res):
    """updateCorridorParam's numCorridor per segment of every path: [nb][W-1] int32."""
    path = np.ascontiguousarray(path, np.float64)
    nb, W = path.shape[0], path.shape[1]
    cs = np.ascontiguousarray(np.broadcast_to(corridor_size, (nb, W - 1)), np.float64)
    out = np.empty((nb, W - 1), np.int32)
    _check(lib.impc_minsnap_corridor_num(C.byref(p), nb, W, _d(path), _d(cs), corridor_res,
                                         out.ctypes.data_as(_i32p)), "impc_minsnap_corridor_num")
    return out


def dims(p, W, cnum=None):
    dm = Dims()
    keep, cp = _cn(cnum, W)
    _check(lib.impc_minsnap_corridor_dims(C.byref(p), W, cp, C.byref(dm)), "impc_minsnap_corridor_dims")
    return dm.n, dm.m, dm.nnzP, dm.nnzA


def pattern(p, W, cnum=None):
    n, m, nnzP, nnzA = dims(p, W, cnum)
    Pp, Pi = np.empty(n + 1, np.int64), np.empty(max(nnzP, 1), np.int64)
    Ap, Ai = np.empty(n + 1, np.int64), np.empty(max(nnzA, 1), np.int64)
    keep, cp = _cn(cnum, W)
    _check(lib.impc_minsnap_corridor_pattern(C.byref(p), W, cp, _i(Pp), _i(Pi), _i(Ap), _i(Ai)),
           "impc_minsnap_corridor_pattern")
    return dict(n=n, m=m, Pp=Pp, Pi=Pi[:nnzP], Ap=Ap, Ai=Ai[:nnzA])


def _opt(a, nb):
    return None if a is None else np.ascontiguousarray(np.broadcast_to(a, (nb, 3)), np.float64)


def _corridor_args(cnum, corridor_size, corridor_res, nb, W):
    keep, cp = _cn(cnum, W)
    if cp is None:
        return keep, None, cp, None, 0.0
    cs = np.ascontiguousarray(np.broadcast_to(corridor_size, (nb, W - 1)), np.float64)
    return keep, cs, cp, _d(cs), float(corridor_res)


def values(p, path, init_vel=None, end_vel=None, init_acc=None, end_acc=None, cnum=None, corridor_size=None,
           corridor_res=None):
    """path [nb][W][3] -> dict(Px, q, Ax, l, u) with 3 nb QPs (axis-minor) and seg_time [nb][W].
    cnum: the batch's numCorridor vector [W-1] (None: no corridor rows)."""
    path = np.ascontiguousarray(path, np.float64)
    nb, W = path.shape[0], path.shape[1]
    n, m, nnzP, nnzA = dims(p, W, cnum)
    out = dict(Px=np.empty((3 * nb, nnzP)), q=np.empty((3 * nb, n)), Ax=np.empty((3 * nb, nnzA)),
               l=np.empty((3 * nb, m)), u=np.empty((3 * nb, m)), seg_time=np.empty((nb, W)))
    ex = [_opt(a, nb) for a in (init_vel, end_vel, init_acc, end_acc)]
    k1, k2, cp, csp, res = _corridor_args(cnum, corridor_size, corridor_res, nb, W)
    _check(lib.impc_minsnap_corridor_values(C.byref(p), nb, W, _d(path), *[_d(a) for a in ex], cp, csp, res,
                                            *[_d(out[k]) for k in ("Px", "q", "Ax", "l", "u", "seg_time")]),
           "impc_minsnap_corridor_values")
    return out


def bounds(p, path, init_vel=None, end_vel=None, init_acc=None, end_acc=None, cnum=None, corridor_size=None,
           corridor_res=None):
    path = np.ascontiguousarray(path, np.float64)
    nb, W = path.shape[0], path.shape[1]
    n, m, _, _ = dims(p, W, cnum)
    l, u = np.empty((3 * nb, m)), np.empty((3 * nb, m))
    ex = [_opt(a, nb) for a in (init_vel, end_vel, init_acc, end_acc)]
    k1, k2, cp, csp, res = _corridor_args(cnum, corridor_size, corridor_res, nb, W)
    _check(lib.impc_minsnap_corridor_bounds(C.byref(p), nb, W, _d(path), *[_d(a) for a in ex], cp, csp, res, _d(l),
                                            _d(u)), "impc_minsnap_corridor_bounds")
    return l, u


def unscale(p, seg_time, x):
    """solveX/Y/Z's rescaling: x [3 nb][n] (copied) -> real-time polynomial coefficients."""
    seg_time = np.ascontiguousarray(seg_time, np.float64)
    x = np.array(x, np.float64, order="C")
    _check(lib.impc_minsnap_unscale(C.byref(p), seg_time.shape[0], seg_time.shape[1], _d(seg_time), _d(x)),
           "impc_minsnap_unscale")
    return x


class MinsnapBatch:
    """nb paths of W waypoints: setUpProblem on the first solve, updateProblem afterwards."""

    def __init__(self, ctx, p, nb, W, settings, cnum=None):
        """cnum: the numCorridor vector [W-1] of every path of the batch (corridor constraints), or
        None."""
        self.p, self.nb, self.W, self.cnum = p, nb, W, cnum
        self.corridor = None
        self.pat = pattern(p, W, cnum)
        pt = self.pat
        self.batch = Batch(ctx, pt["n"], pt["m"], pt["Pp"], pt["Pi"], pt["Ap"], pt["Ai"], 3 * nb)
        self.batch.set_settings(settings)
        self.init = False
        self.seg_time = None

    def update_path(self, path, corridor_size=None, corridor_res=None):
        """updatePath (:54-63), with setCorridorConstraint (:960-970) when the batch has corridor
        rows: a new path; the next solve sets the problem up again."""
        self.path = np.ascontiguousarray(path, np.float64)
        if (self.cnum is None) != (corridor_size is None):
            raise ValueError("corridor_size must be given exactly when the batch was built with cnum")
        self.corridor = None if corridor_size is None else (corridor_size, corridor_res)
        self.init = False

    def solve(self, init_vel=None, end_vel=None, init_acc=None, end_acc=None):
        """polyTrajSolver::solve (:849-868) with the end conditions of updateInit/EndVel/Acc:
        setUpProblem after a new path, else updateProblem (bounds only).  Returns (coefficients
        [nb][3][n] in real time, the normalised-time solutions [3 nb][n], info)."""
        cor = {} if self.corridor is None else dict(cnum=self.cnum, corridor_size=self.corridor[0],
                                                    corridor_res=self.corridor[1])
        if not self.init:
            v = values(self.p, self.path, init_vel, end_vel, init_acc, end_acc, **cor)
            self.batch.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
            self.seg_time = v["seg_time"]
            self.init = True
        else:
            l, u = bounds(self.p, self.path, init_vel, end_vel, init_acc, end_acc, **cor)
            self.batch.update_bounds(l, u)
        self.batch.solve()
        x, y, info = self.batch.get()
        return unscale(self.p, self.seg_time, x).reshape(self.nb, 3, -1), x, info

    def close(self):
        self.batch.close()
