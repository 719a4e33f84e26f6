"""TEST INFRASTRUCTURE ONLY -- ctypes front end of oracle/build/libosqp_oracle.so.

The oracle is the CPU restatement of OSQP 0.6.2 in oracle/osqp_oracle.c (see its header for
provenance and the "parity unpinned" status).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module, and only as the checker / CPU baseline.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libosqp_oracle.so")


class OraSettings(C.Structure):
    _fields_ = [
        ("rho", C.c_double), ("sigma", C.c_double), ("scaling", C.c_int64), ("adaptive_rho", C.c_int64),
        ("adaptive_rho_interval", C.c_int64), ("adaptive_rho_tolerance", C.c_double),
        ("adaptive_rho_fraction", C.c_double), ("max_iter", C.c_int64), ("eps_abs", C.c_double),
        ("eps_rel", C.c_double), ("eps_prim_inf", C.c_double), ("eps_dual_inf", C.c_double),
        ("alpha", C.c_double), ("linsys_solver", C.c_int64), ("delta", C.c_double), ("polish", C.c_int64),
        ("polish_refine_iter", C.c_int64), ("verbose", C.c_int64), ("scaled_termination", C.c_int64),
        ("check_termination", C.c_int64), ("warm_start", C.c_int64), ("time_limit", C.c_double),
    ]


INFO_DTYPE = np.dtype([("iter", np.int64), ("status_val", np.int64), ("rho_updates", np.int64),
                       ("setup_exitflag", np.int64), ("obj_val", np.float64), ("pri_res", np.float64),
                       ("dua_res", np.float64), ("rho_estimate", np.float64)])

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"oracle not built: {LIB_PATH} (run `make oracle`)")
        L = C.CDLL(LIB_PATH)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int64)
        L.ora_default_settings.argtypes = [C.POINTER(OraSettings)]
        L.ora_default_settings.restype = None
        L.ora_solve_batch.argtypes = [C.c_int64, C.c_int64, C.c_int64, ip, ip, dp, dp, ip, ip, dp, dp, dp,
                                      C.POINTER(OraSettings), dp, dp, dp, dp, C.c_void_p, C.c_int]
        L.ora_solve_batch.restype = C.c_int
        L.ora_setup.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_int64, ip, ip, dp, dp, ip, ip, dp, dp, dp,
                                C.POINTER(OraSettings)]
        L.ora_setup.restype = C.c_int
        L.ora_warm_start.argtypes = [C.c_void_p, dp, dp]
        L.ora_solve_ws.argtypes = [C.c_void_p]
        L.ora_get.argtypes = [C.c_void_p, dp, dp, C.c_void_p]
        L.ora_get.restype = None
        L.ora_update_lin_cost.argtypes = [C.c_void_p, dp]
        L.ora_update_bounds.argtypes = [C.c_void_p, dp, dp]
        L.ora_update_P_A.argtypes = [C.c_void_p, dp, dp]
        L.ora_rescale_raw.argtypes = [C.c_void_p, dp, dp, dp, dp, dp]
        L.ora_cleanup.argtypes = [C.c_void_p]
        L.ora_get_state.argtypes = [C.c_void_p, dp, dp, dp, dp]
        L.ora_get_state.restype = None
        L.ora_set_state.argtypes = [C.c_void_p, C.c_double, dp, dp, dp]
        L.ora_set_state.restype = C.c_int
        L.ora_get_setup.argtypes = [C.c_void_p, dp, ip, dp, dp, dp]
        L.ora_cleanup.restype = None
        _lib = L
    return _lib


def default_settings(**kw):
    s = OraSettings()
    lib().ora_default_settings(C.byref(s))
    for k, v in kw.items():
        setattr(s, k, v)
    return s


def settings_from(other):
    """Copy any struct with OSQPSettings field names (e.g. impc.Settings)."""
    s = OraSettings()
    for f, _ in OraSettings._fields_:
        setattr(s, f, getattr(other, f))
    return s


def _d(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int64))


def solve_batch(pattern, Px, q, Ax, l, u, settings=None, x_ws=None, y_ws=None, threads=1):
    """pattern: dict(n, m, Pp, Pi, Ap, Ai); values QP-major with a leading batch axis.
    Each QP follows the reference per-call pattern: setup -> [warm start] -> solve -> cleanup."""
    n, m = int(pattern["n"]), int(pattern["m"])
    Pp, Pi, Ap, Ai = [np.ascontiguousarray(pattern[k], dtype=np.int64) for k in ("Pp", "Pi", "Ap", "Ai")]
    if Pi.size == 0:
        Pi = np.zeros(1, np.int64)
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (Px, q, Ax, l, u)]
    nb = arrs[1].reshape(-1, n).shape[0]
    xw = None if x_ws is None else np.ascontiguousarray(x_ws, dtype=np.float64)
    yw = None if y_ws is None else np.ascontiguousarray(y_ws, dtype=np.float64)
    if xw is not None and yw is None:
        yw = np.zeros((nb, m))
    s = settings if settings is not None else default_settings()
    x = np.empty((nb, n))
    y = np.empty((nb, max(m, 1)))
    info = np.empty(nb, dtype=INFO_DTYPE)
    lib().ora_solve_batch(nb, n, m, _i(Pp), _i(Pi), _d(arrs[0]), _d(arrs[1]), _i(Ap), _i(Ai), _d(arrs[2]),
                          _d(arrs[3]), _d(arrs[4]), C.byref(s), _d(xw), _d(yw), _d(x), _d(y),
                          info.ctypes.data_as(C.c_void_p), int(threads))
    return x, y[:, :m], info


class Workspace:
    """Persistent OSQP workspace (osqp_setup once, then update_lin_cost / update_bounds / solve)."""

    def __init__(self, pattern, Px, q, Ax, l, u, settings=None):
        self.n, self.m = int(pattern["n"]), int(pattern["m"])
        self._pat = [np.ascontiguousarray(pattern[k], dtype=np.int64) for k in ("Pp", "Pi", "Ap", "Ai")]
        if self._pat[1].size == 0:
            self._pat[1] = np.zeros(1, np.int64)
        vals = [np.ascontiguousarray(a, dtype=np.float64) for a in (Px, q, Ax, l, u)]
        self.s = settings if settings is not None else default_settings()
        self.h = C.c_void_p()
        rc = lib().ora_setup(C.byref(self.h), self.n, self.m, _i(self._pat[0]), _i(self._pat[1]), _d(vals[0]),
                             _d(vals[1]), _i(self._pat[2]), _i(self._pat[3]), _d(vals[2]), _d(vals[3]),
                             _d(vals[4]), C.byref(self.s))
        if rc:
            raise RuntimeError(f"ora_setup failed: {rc}")

    def warm_start(self, x, y):
        lib().ora_warm_start(self.h, _d(np.ascontiguousarray(x, float)), _d(np.ascontiguousarray(y, float)))

    def update_lin_cost(self, q):
        lib().ora_update_lin_cost(self.h, _d(np.ascontiguousarray(q, float)))

    def update_bounds(self, l, u):
        lib().ora_update_bounds(self.h, _d(np.ascontiguousarray(l, float)), _d(np.ascontiguousarray(u, float)))

    def update_matrices(self, Px=None, Ax=None):
        """osqp_update_P / osqp_update_A / osqp_update_P_A with every value (ora_update_P_A)."""
        P = None if Px is None else np.ascontiguousarray(Px, float)
        A = None if Ax is None else np.ascontiguousarray(Ax, float)
        rc = lib().ora_update_P_A(self.h, _d(P), _d(A))
        if rc:
            raise RuntimeError(f"ora_update_P_A failed: {rc}")

    def rescale_raw(self, Px, q, Ax, l, u):
        """Study variant (not OSQP): new raw data scaled afresh, rho and scaled iterates kept."""
        a = [np.ascontiguousarray(v, float) for v in (Px, q, Ax, l, u)]
        rc = lib().ora_rescale_raw(self.h, *[_d(v) for v in a])
        if rc:
            raise RuntimeError(f"ora_rescale_raw failed: {rc}")

    def get_state(self):
        """(rho, x, z, y): settings rho and the SCALED iterates the workspace holds (ora_get_state)."""
        rho = C.c_double()
        x, z, y = np.empty(self.n), np.empty(max(self.m, 1)), np.empty(max(self.m, 1))
        lib().ora_get_state(self.h, C.byref(rho), _d(x), _d(z), _d(y))
        return rho.value, x, z[: self.m], y[: self.m]

    def set_state(self, rho, x, z, y):
        """Load another solver's persisted (rho, scaled x, z, y) into this workspace (ora_set_state:
        rho_vec by constraint type and a refactorisation when rho changes)."""
        a = [np.ascontiguousarray(v, float) for v in (x, z, y)]
        rc = lib().ora_set_state(self.h, float(rho), *[_d(v) for v in a])
        if rc:
            raise RuntimeError(f"ora_set_state failed: {rc}")

    def setup_state(self):
        """rho_vec, constr_type, D, E and c as osqp_setup left them (ora_get_setup)."""
        rho = np.empty(max(self.m, 1))
        ct = np.empty(max(self.m, 1), np.int64)
        D, E = np.empty(self.n), np.empty(max(self.m, 1))
        c = C.c_double()
        lib().ora_get_setup(self.h, _d(rho), _i(ct), _d(D), _d(E), C.byref(c))
        return dict(rho_vec=rho[: self.m], constr_type=ct[: self.m], D=D, E=E[: self.m], c=c.value)

    def solve(self):
        lib().ora_solve_ws(self.h)
        x = np.empty(self.n)
        y = np.empty(max(self.m, 1))
        info = np.empty(1, dtype=INFO_DTYPE)
        lib().ora_get(self.h, _d(x), _d(y), info.ctypes.data_as(C.c_void_p))
        return x, y[: self.m], info[0]

    def close(self):
        if self.h:
            lib().ora_cleanup(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
