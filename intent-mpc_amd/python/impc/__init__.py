"""ctypes bindings of libimpc_qp.so (include/impc_qp.h, include/impc_mpc.h).

Thin plumbing for tests and bench.py: every call goes straight to the C-ABI.  There is no
Python/CPU fallback -- if the shared library is missing, importing this module raises, and a
solve without a HIP device fails with IMPC_DEVICE_ERROR.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(os.path.dirname(_HERE))  # .../intent-mpc_amd
LIB_PATH = os.path.join(_PKG, "lib", "libimpc_qp.so")
if os.environ.get("IMPC_SECTION_PROF") == "1":  # profiling variant (tools/section_profile.py only)
    LIB_PATH = os.path.join(_PKG, "lib", "libimpc_qp_prof.so")
if os.environ.get("IMPC_LIB_VARIANT"):  # kernel-shape experiments (tools/ only): lib/libimpc_qp_<v>.so
    LIB_PATH = os.path.join(_PKG, "lib", "libimpc_qp_" + os.environ["IMPC_LIB_VARIANT"] + ".so")

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libimpc_qp.so not built at {LIB_PATH} (run __graft_entry__.build() or `make lib`)")
lib = C.CDLL(LIB_PATH)

# ---- status / error codes (constants.h:18-51)
SOLVED_INACCURATE, SOLVED = 2, 1
MAX_ITER_REACHED, PRIMAL_INFEASIBLE, DUAL_INFEASIBLE = -2, -3, -4
PRIMAL_INFEASIBLE_INACCURATE, DUAL_INFEASIBLE_INACCURATE = 3, 4
TIME_LIMIT_REACHED, NON_CVX, UNSOLVED = -6, -7, -10
OSQP_NAN = 2143289344.0


class Settings(C.Structure):
    """impc_settings == OSQPSettings (types.h:139-176)."""
    _fields_ = [
        ("rho", C.c_double), ("sigma", C.c_double), ("scaling", C.c_int64), ("adaptive_rho", C.c_int64),
        ("adaptive_rho_interval", C.c_int64), ("adaptive_rho_tolerance", C.c_double),
        ("adaptive_rho_fraction", C.c_double), ("max_iter", C.c_int64), ("eps_abs", C.c_double),
        ("eps_rel", C.c_double), ("eps_prim_inf", C.c_double), ("eps_dual_inf", C.c_double),
        ("alpha", C.c_double), ("linsys_solver", C.c_int64), ("delta", C.c_double), ("polish", C.c_int64),
        ("polish_refine_iter", C.c_int64), ("verbose", C.c_int64), ("scaled_termination", C.c_int64),
        ("check_termination", C.c_int64), ("warm_start", C.c_int64), ("time_limit", C.c_double),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class Info(C.Structure):
    _fields_ = [("iter", C.c_int64), ("status_val", C.c_int64), ("rho_updates", C.c_int64),
                ("setup_exitflag", C.c_int64), ("obj_val", C.c_double), ("pri_res", C.c_double),
                ("dua_res", C.c_double), ("rho_estimate", C.c_double)]


INFO_DTYPE = np.dtype([("iter", np.int64), ("status_val", np.int64), ("rho_updates", np.int64),
                       ("setup_exitflag", np.int64), ("obj_val", np.float64), ("pri_res", np.float64),
                       ("dua_res", np.float64), ("rho_estimate", np.float64)])


class Stats(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("n", "m", "nnzP", "nnzA", "batch", "batch_stride", "nnzL", "nnzLcol",
                                         "n_terms", "bandwidth", "device_bytes", "kernel",
                                         "structured_ok", "team_lanes", "var_slots", "row_slots")]


class MpcParams(C.Structure):
    """impc_mpc_params: mpcPlanner::initParam values (mpcPlanner.cpp:19-173)."""
    _fields_ = [("horizon", C.c_int32), ("num_half_space", C.c_int32), ("ts", C.c_double),
                ("max_vel", C.c_double), ("max_acc", C.c_double), ("y_range_min", C.c_double),
                ("y_range_max", C.c_double), ("z_range_min", C.c_double), ("z_range_max", C.c_double),
                ("static_safety_dist", C.c_double), ("dynamic_safety_dist", C.c_double),
                ("static_slack", C.c_double), ("dynamic_slack", C.c_double), ("position_weight", C.c_double),
                ("velocity_weight", C.c_double), ("acceleration_weight", C.c_double),
                ("half_max", C.c_double * 3), ("half_min", C.c_double * 3)]


class Dims(C.Structure):
    _fields_ = [("n", C.c_int64), ("m", C.c_int64), ("nnzP", C.c_int64), ("nnzA", C.c_int64)]


_P = C.c_void_p
_i64p = C.POINTER(C.c_int64)
_dp = C.POINTER(C.c_double)


def _sig(name, res, *args):
    if os.environ.get("IMPC_LIB_VARIANT") and not hasattr(lib, name):
        return None  # an older library kept for an A/B (tools only): entry points added since are absent
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_sig("impc_default_settings", None, C.POINTER(Settings))
_sig("impc_last_error", C.c_char_p)
_sig("impc_version", C.c_char_p)
_sig("impc_build_id", C.c_char_p)
_sig("impc_ctx_create", C.c_int, C.c_int, C.POINTER(_P))
_sig("impc_ctx_destroy", C.c_int, _P)
_sig("impc_ctx_stream", _P, _P)
_sig("impc_ctx_synchronize", C.c_int, _P)
_sig("impc_batch_create", C.c_int, _P, C.c_int64, C.c_int64, _i64p, _i64p, _i64p, _i64p, C.c_int64, C.POINTER(_P))
_sig("impc_batch_destroy", C.c_int, _P)
_sig("impc_batch_acquire", C.c_int, _P, C.c_int64, C.c_int64, _i64p, _i64p, _i64p, _i64p, C.c_int64, C.POINTER(_P))
_sig("impc_batch_release", C.c_int, _P)
_sig("impc_ctx_pool_stats", C.c_int, _P, C.POINTER(C.c_int64), C.POINTER(C.c_int64))
_sig("impc_host_alloc", C.c_int, _P, C.c_int64, C.POINTER(_P))
_sig("impc_host_free", C.c_int, _P, _P)
_sig("impc_stream_create", C.c_int, _P, C.POINTER(_P))
_sig("impc_stream_destroy", C.c_int, _P, _P)
_sig("impc_stream_wait", C.c_int, _P, _P, _P)
_sig("impc_stream_synchronize", C.c_int, _P, _P)
_sig("impc_batch_set_values_async", C.c_int, _P, _P, _P, _P, _P, _P, _P)
_sig("impc_batch_get_async", C.c_int, _P, _P, _P, _P, _P)
_sig("impc_batch_set_settings", C.c_int, _P, C.POINTER(Settings))
_sig("impc_batch_set_values", C.c_int, _P, _dp, _dp, _dp, _dp, _dp)
_sig("impc_batch_set_values_device", C.c_int, _P, _P, _P, _P, _P, _P)
_sig("impc_batch_set_values_shared", C.c_int, _P, _dp, _dp, C.c_int64, _i64p, _dp, _dp, _dp, _dp)
_sig("impc_batch_warm_start", C.c_int, _P, _dp, _dp)
_sig("impc_batch_warm_start_device", C.c_int, _P, _P, _P)
_sig("impc_batch_set_active", C.c_int, _P, C.c_int64)
_sig("impc_gather_rows_device", C.c_int, _P, _P, C.c_int64, _P, C.c_int64, _P, _P)
_sig("impc_replan_commit_device", C.c_int, _P, C.c_int32, C.c_int64, C.c_int64, _P, _P, C.c_int32, _P, _P, _P, _P, _P,
     _P, _P, _P, _P)
_sig("impc_batch_setup", C.c_int, _P, _P)
_sig("impc_batch_solve", C.c_int, _P, _P)
_sig("impc_batch_get", C.c_int, _P, _dp, _dp, C.c_void_p)
_sig("impc_batch_device_results", C.c_int, _P, C.POINTER(_P), C.POINTER(_P), C.POINTER(_P))
_sig("impc_batch_update_lin_cost", C.c_int, _P, _dp)
_sig("impc_batch_update_bounds", C.c_int, _P, _dp, _dp)
_sig("impc_batch_update_lin_cost_device", C.c_int, _P, _P)
_sig("impc_batch_update_bounds_device", C.c_int, _P, _P, _P)
_sig("impc_batch_update_matrices", C.c_int, _P, _dp, _dp)
_sig("impc_batch_update_matrices_device", C.c_int, _P, _P, _P)
_sig("impc_batch_get_stats", C.c_int, _P, C.POINTER(Stats))
_sig("impc_batch_get_perm", C.c_int, _P, _i64p)
_sig("impc_batch_set_profiling", C.c_int, _P, C.c_int)
_sig("impc_batch_get_timings", C.c_int, _P, _dp, _dp, _dp)
_sig("impc_batch_get_qp_latency", C.c_int, _P, _dp)
_sig("impc_batch_set_persistent", C.c_int, _P, C.c_int)
_sig("impc_batch_get_persistent", C.c_int, _P, _dp, _dp, _dp, _dp)
_sig("impc_batch_set_kernel", C.c_int, _P, C.c_int)
_sig("impc_batch_solve_group", C.c_int, C.POINTER(_P), C.c_int, _P)
_sig("impc_device_alloc", C.c_int, _P, C.c_int64, C.POINTER(_P))
_sig("impc_device_free", C.c_int, _P, _P)
_sig("impc_copy_to_device", C.c_int, _P, _P, _P, C.c_int64)
_sig("impc_copy_to_host", C.c_int, _P, _P, _P, C.c_int64)
_sig("impc_reference_traj_device", C.c_int, _P, C.c_int32, C.c_double, C.c_int64, _P, _P, _P, _P, C.c_int32, _P, _P)
_sig("impc_repeat_rows_device", C.c_int, _P, _P, C.c_int64, C.c_int64, C.c_int32, _P, _P)
_sig("impc_copy_rows_device", C.c_int, _P, _P, C.c_int64, _P, C.c_int64, C.c_int64, C.c_int64, _P)
_sig("impc_batch_follow_plan_device", C.c_int, _P, C.c_int32, C.c_double, C.c_double, _P, _P, _P)
# include/impc_comm.h
COMM_ID_BYTES = 128
_sig("impc_comm_unique_id", C.c_int, C.POINTER(C.c_ubyte))
_sig("impc_comm_create", C.c_int, _P, C.POINTER(C.c_ubyte), C.c_int, C.c_int, C.POINTER(_P))
_sig("impc_comm_destroy", C.c_int, _P)
_sig("impc_comm_allgather", C.c_int, _P, _P, _P, C.c_int64, _P)
_sig("impc_comm_gather_info", C.c_int, _P, C.POINTER(_P), C.c_int, C.c_int64, _P, _P)
_sig("impc_comm_max", C.c_int, _P, C.POINTER(C.c_double))
_sig("impc_ctx_timer_mark", C.c_int, _P, _P)
_sig("impc_batch_set_time_limits", C.c_int, _P, _dp)
_sig("impc_batch_set_queue_order", C.c_int, _P, C.c_int, C.c_double)
_sig("impc_ctx_clock_rate", C.c_int, _P, _dp)
_sig("impc_ctx_clock_check", C.c_int, _P, C.c_double, _dp)
_sig("impc_ctx_timer_read", C.c_int, _P, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_int64))


class SelectParams(C.Structure):
    """impc_select_params (include/impc_select.h)."""
    _fields_ = [("horizon", C.c_int32), ("num_candidates", C.c_int32), ("max_dynamic", C.c_int32),
                ("pred_len", C.c_int32), ("num_static", C.c_int32), ("prev_len", C.c_int32),
                ("dynamic_safety_dist", C.c_double), ("static_safety_dist", C.c_double)]


_sig("impc_select_best", C.c_int, _P, C.POINTER(SelectParams), C.c_int64, _P, _P, _P, _dp, _P, _dp, _dp, _dp, _P,
     _dp, _dp, _dp, _P, _P, _dp, _dp)
_sig("impc_select_best_device", C.c_int, _P, C.POINTER(SelectParams), C.c_int64, _P, _P, _P, _P, _P, _P, _P, _P, _P,
     _P, _P, _P, _P, _P, _P, _P, _P)
class MinsnapParams(C.Structure):
    """impc_minsnap_params (include/impc_minsnap.h)."""
    _fields_ = [("poly_degree", C.c_int32), ("diff_degree", C.c_int32), ("continuity_degree", C.c_int32),
                ("desired_vel", C.c_double), ("soft_constraint", C.c_int32), ("sc_deviation", C.c_double * 3)]


_sig("impc_minsnap_dims", C.c_int, C.POINTER(MinsnapParams), C.c_int32, C.POINTER(Dims))
_sig("impc_minsnap_build_pattern", C.c_int, C.POINTER(MinsnapParams), C.c_int32, _i64p, _i64p, _i64p, _i64p)
_sig("impc_minsnap_build_values", C.c_int, C.POINTER(MinsnapParams), C.c_int64, C.c_int32, _dp, _dp, _dp, _dp, _dp,
     _dp, _dp, _dp, _dp, _dp, _dp)
_sig("impc_minsnap_build_bounds", C.c_int, C.POINTER(MinsnapParams), C.c_int64, C.c_int32, _dp, _dp, _dp, _dp, _dp,
     _dp, _dp)
_i32p = C.POINTER(C.c_int32)
_sig("impc_minsnap_corridor_num", C.c_int, C.POINTER(MinsnapParams), C.c_int64, C.c_int32, _dp, _dp, C.c_double, _i32p)
_sig("impc_minsnap_corridor_dims", C.c_int, C.POINTER(MinsnapParams), C.c_int32, _i32p, C.POINTER(Dims))
_sig("impc_minsnap_corridor_pattern", C.c_int, C.POINTER(MinsnapParams), C.c_int32, _i32p, _i64p, _i64p, _i64p,
     _i64p)
_sig("impc_minsnap_corridor_values", C.c_int, C.POINTER(MinsnapParams), C.c_int64, C.c_int32, _dp, _dp, _dp, _dp, _dp,
     _i32p, _dp, C.c_double, _dp, _dp, _dp, _dp, _dp, _dp)
_sig("impc_minsnap_corridor_bounds", C.c_int, C.POINTER(MinsnapParams), C.c_int64, C.c_int32, _dp, _dp, _dp, _dp, _dp,
     _i32p, _dp, C.c_double, _dp, _dp)
_sig("impc_minsnap_unscale", C.c_int, C.POINTER(MinsnapParams), C.c_int64, C.c_int32, _dp, _dp)
_sig("impc_mpc_dims", C.c_int, C.POINTER(MpcParams), C.c_int32, C.c_int32, C.POINTER(Dims))
_sig("impc_mpc_build_pattern", C.c_int, C.POINTER(MpcParams), C.c_int32, C.c_int32, _i64p, _i64p, _i64p, _i64p)
_sig("impc_mpc_build_values", C.c_int, C.POINTER(MpcParams), C.c_int64, _dp, _dp, _dp, _dp, C.c_int32, _dp, _dp,
     _dp, C.c_int32, C.c_int32, _dp, _dp, _dp, _dp, _dp, _dp, _dp)
_sig("impc_mpc_builder_create", C.c_int, _P, C.POINTER(MpcParams), C.c_int32, C.c_int32, C.c_int32, C.POINTER(_P))
_sig("impc_mpc_builder_destroy", C.c_int, _P)
_sig("impc_mpc_build_values_device", C.c_int, _P, C.c_int64, *([_P] * 14), _P)
_sig("impc_mpc_warm_start", C.c_int, C.POINTER(MpcParams), C.c_int64, _dp, _dp, _dp)
_sig("impc_intent_fanout", C.c_int, _P, C.c_int64, C.c_int32, C.c_int32, C.c_int32, *([_P] * 16))
_sig("impc_intent_fanout_device", C.c_int, _P, C.c_int64, C.c_int32, C.c_int32, C.c_int32, *([_P] * 16), _P)
class IntentParams(C.Structure):
    """impc_intent_params (include/impc_predict.h)."""
    _fields_ = [("paramf", C.c_double), ("paraml", C.c_double), ("paramr", C.c_double), ("params", C.c_double),
                ("pscale", C.c_double)]


_sig("impc_intent_params_from_config", C.c_int, C.c_double, C.c_double, C.c_double, C.c_double,
     C.POINTER(IntentParams))
_sig("impc_intent_prob", C.c_int, _P, C.POINTER(IntentParams), C.c_int64, C.c_int32, _P, _P, _P, _P)
_sig("impc_intent_prob_device", C.c_int, _P, C.POINTER(IntentParams), C.c_int64, C.c_int32, _P, _P, _P, _P, _P)
class OccMap(C.Structure):
    """impc_occ_map (include/impc_predict.h)."""
    _fields_ = [("origin", C.c_double * 3), ("resolution", C.c_double), ("dims", C.c_int32 * 3),
                ("reserved", C.c_int32)]


class TrajParams(C.Structure):
    """impc_traj_params (include/impc_predict.h)."""
    _fields_ = [("num_pred", C.c_int32), ("reserved", C.c_int32), ("dt", C.c_double), ("stop_velocity", C.c_double),
                ("front_angle_deg", C.c_double), ("min_turning_time", C.c_double), ("max_turning_time", C.c_double),
                ("z_score", C.c_double)]


_sig("impc_predict_traj", C.c_int, _P, C.POINTER(TrajParams), C.POINTER(OccMap), _P, C.c_int64, _P, _P, _P, _P, _P)
_sig("impc_predict_traj_device", C.c_int, _P, C.POINTER(TrajParams), C.POINTER(OccMap), _P, C.c_int64, _P, _P, _P,
     _P, _P, _P)
_sig("impc_fanout_candidates_device", C.c_int, _P, C.c_int64, C.c_int32, C.c_int32, _P, _P, _P, _P, _P, _P,
     C.c_int64, _P, C.c_int64, _P, _P, _P, _P, _P)

# every symbol declared in include/*.h (checked by tests/test_abi.py)
KERNEL_AUTO, KERNEL_GENERIC, KERNEL_STRUCTURED = 0, 1, 2
QUEUE_FIFO, QUEUE_LONGEST_FIRST = 0, 1

EXPORTED = [
    "impc_default_settings", "impc_last_error", "impc_version", "impc_build_id", "impc_ctx_create", "impc_ctx_destroy",
    "impc_ctx_stream", "impc_ctx_synchronize", "impc_batch_create", "impc_batch_destroy", "impc_batch_set_settings",
    "impc_batch_set_values", "impc_batch_set_values_device", "impc_batch_set_values_shared", "impc_batch_warm_start", "impc_batch_setup",
    "impc_batch_solve", "impc_batch_get", "impc_batch_device_results", "impc_batch_update_lin_cost",
    "impc_batch_update_bounds", "impc_batch_get_stats", "impc_batch_get_perm", "impc_batch_set_profiling",
    "impc_batch_get_timings", "impc_batch_get_qp_latency", "impc_batch_set_persistent", "impc_batch_set_kernel", "impc_batch_solve_group", "impc_device_alloc", "impc_device_free",
    "impc_copy_to_device", "impc_copy_to_host", "impc_select_best", "impc_select_best_device", "impc_mpc_dims",
    "impc_mpc_build_pattern", "impc_mpc_build_values", "impc_mpc_warm_start", "impc_mpc_builder_create",
    "impc_mpc_builder_destroy", "impc_mpc_build_values_device", "impc_intent_fanout", "impc_intent_fanout_device",
    "impc_fanout_candidates_device", "impc_intent_params_from_config", "impc_intent_prob", "impc_intent_prob_device",
    "impc_predict_traj", "impc_predict_traj_device", "impc_minsnap_dims", "impc_minsnap_build_pattern",
    "impc_minsnap_build_values", "impc_minsnap_build_bounds", "impc_minsnap_unscale", "impc_minsnap_corridor_num",
    "impc_minsnap_corridor_dims", "impc_minsnap_corridor_pattern", "impc_minsnap_corridor_values",
    "impc_minsnap_corridor_bounds",
    "impc_reference_traj_device", "impc_repeat_rows_device", "impc_comm_unique_id", "impc_comm_create", "impc_comm_destroy", "impc_comm_allgather", "impc_comm_gather_info",
    "impc_comm_max", "impc_ctx_timer_mark", "impc_ctx_timer_read", "impc_batch_set_time_limits",
    "impc_ctx_clock_rate", "impc_ctx_clock_check", "impc_batch_set_queue_order", "impc_batch_warm_start_device",
    "impc_batch_set_active", "impc_gather_rows_device", "impc_replan_commit_device", "impc_batch_acquire",
    "impc_batch_release", "impc_host_alloc", "impc_host_free", "impc_stream_create", "impc_stream_destroy",
    "impc_stream_wait", "impc_stream_synchronize", "impc_batch_set_values_async", "impc_batch_get_async",
    "impc_batch_update_lin_cost_device", "impc_batch_update_bounds_device", "impc_ctx_pool_stats",
    "impc_replan_create", "impc_replan_destroy", "impc_replan_set_state", "impc_replan_run", "impc_replan_get_stats",
    "impc_replan_view_device", "impc_replan_shape", "impc_replan_advance_device", "impc_batch_follow_plan_device",
    "impc_copy_rows_device", "impc_batch_update_matrices", "impc_batch_update_matrices_device",
    "impc_batch_get_persistent",
]


class ImpcError(RuntimeError):
    def __init__(self, code, where):
        msg = lib.impc_last_error().decode()
        super().__init__(f"{where} failed with code {code}: {msg}")
        self.code = code


def _check(rc, where):
    if rc != 0:
        raise ImpcError(rc, where)


def _d(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _i(a):
    return None if a is None else a.ctypes.data_as(_i64p)


def default_settings(**kw):
    s = Settings()
    lib.impc_default_settings(C.byref(s))
    for k, v in kw.items():
        setattr(s, k, v)
    return s


class Context:
    def __init__(self, device=0):
        h = _P()
        _check(lib.impc_ctx_create(device, C.byref(h)), "impc_ctx_create")
        self.h = h

    @property
    def stream(self):
        return lib.impc_ctx_stream(self.h)

    def synchronize(self):
        _check(lib.impc_ctx_synchronize(self.h), "impc_ctx_synchronize")

    def timer_mark(self, stream=None):
        """impc_ctx_timer_mark: a HIP event on the launch stream (context stream if None)."""
        _check(lib.impc_ctx_timer_mark(self.h, _P(stream) if stream else None), "impc_ctx_timer_mark")

    def timer_read(self, max_pairs=4096):
        """impc_ctx_timer_read: ms between marks 2k and 2k+1 (synchronises, clears the marks)."""
        ms = np.zeros(max_pairs)
        n = C.c_int64()
        _check(lib.impc_ctx_timer_read(self.h, ms.ctypes.data_as(_dp), max_pairs, C.byref(n)), "impc_ctx_timer_read")
        return ms[: n.value]

    def clock_rate(self):
        """impc_ctx_clock_rate: Hz of the device clock time limits and latencies are read on."""
        hz = C.c_double()
        _check(lib.impc_ctx_clock_rate(self.h, C.byref(hz)), "impc_ctx_clock_rate")
        return hz.value

    def clock_check(self, seconds):
        """impc_ctx_clock_check: HIP-event seconds of a kernel that spins `seconds` on the device clock."""
        ev = C.c_double()
        _check(lib.impc_ctx_clock_check(self.h, float(seconds), C.byref(ev)), "impc_ctx_clock_check")
        return ev.value

    def close(self):
        if self.h:
            lib.impc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Batch:
    """B QPs with one shared (P, A) pattern, solved on the GPU."""

    def __init__(self, ctx, n, m, Pp, Pi, Ap, Ai, batch):
        self.ctx = ctx
        self.n, self.m, self.B = int(n), int(m), int(batch)
        self._pat = [np.ascontiguousarray(a, dtype=np.int64) for a in (Pp, Pi, Ap, Ai)]
        self.nnzP, self.nnzA = int(self._pat[0][-1]), int(self._pat[2][-1])
        h = _P()
        _check(lib.impc_batch_create(ctx.h, self.n, self.m, *[_i(a) for a in self._pat], self.B, C.byref(h)),
               "impc_batch_create")
        self.h = h

    def set_settings(self, s):
        _check(lib.impc_batch_set_settings(self.h, C.byref(s)), "impc_batch_set_settings")

    def set_values(self, Px, q, Ax, l, u):
        arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (Px, q, Ax, l, u)]
        assert arrs[0].size == self.B * self.nnzP and arrs[1].size == self.B * self.n
        assert arrs[2].size == self.B * self.nnzA and arrs[3].size == self.B * self.m == arrs[4].size
        _check(lib.impc_batch_set_values(self.h, *[_d(a) for a in arrs]), "impc_batch_set_values")

    def set_values_shared(self, Px, Ax, var_pos, Ax_var, q, l, u):
        """Shared P / A values (one copy) with per-QP overrides Ax_var [B][len(var_pos)] at the A
        positions var_pos, per-QP q, l, u (impc_batch_set_values_shared)."""
        Px, Ax, Axv, q, l, u = [np.ascontiguousarray(a, dtype=np.float64) for a in (Px, Ax, Ax_var, q, l, u)]
        vp = np.ascontiguousarray(var_pos, dtype=np.int64)
        assert Px.size == self.nnzP and Ax.size == self.nnzA and Axv.size == self.B * vp.size
        assert q.size == self.B * self.n and l.size == self.B * self.m == u.size
        _check(lib.impc_batch_set_values_shared(self.h, _d(Px), _d(Ax), vp.size,
                                                vp.ctypes.data_as(_i64p), _d(Axv), _d(q), _d(l), _d(u)),
               "impc_batch_set_values_shared")

    def set_values_device(self, Px, q, Ax, l, u):
        """Device pointers (ints) of QP-major float64 arrays, e.g. torch tensors' data_ptr()."""
        _check(lib.impc_batch_set_values_device(self.h, *[C.c_void_p(int(p)) for p in (Px, q, Ax, l, u)]),
               "impc_batch_set_values_device")

    def warm_start(self, x=None, y=None):
        xa = None if x is None else np.ascontiguousarray(x, dtype=np.float64)
        ya = None if y is None else np.ascontiguousarray(y, dtype=np.float64)
        # the C side copies B*n / B*m doubles from these pointers: shapes are checked here
        if xa is not None and xa.size != self.B * self.n:
            raise ValueError(f"warm_start: x has {xa.size} values, expected B*n = {self.B * self.n}")
        if ya is not None and ya.size != self.B * self.m:
            raise ValueError(f"warm_start: y has {ya.size} values, expected B*m = {self.B * self.m}")
        _check(lib.impc_batch_warm_start(self.h, _d(xa), _d(ya)), "impc_batch_warm_start")

    def warm_start_device(self, x_ptr, y_ptr=None):
        """impc_batch_warm_start_device: QP-major device arrays x [B][n] (y [B][m] or None = 0)."""
        _check(lib.impc_batch_warm_start_device(self.h, _P(x_ptr) if x_ptr else None, _P(y_ptr) if y_ptr else None),
               "impc_batch_warm_start_device")

    def set_values_async(self, Ax_var, q, l, u, x_ws=None, stream=None):
        """impc_batch_set_values_async: HostArray / pinned sources, queued on `stream` (a Stream)."""
        ptr = lambda a: None if a is None else _P(a.ptr if isinstance(a, HostArray) else a.ctypes.data)  # noqa: E731
        _check(lib.impc_batch_set_values_async(self.h, ptr(Ax_var), ptr(q), ptr(l), ptr(u), ptr(x_ws),
                                               _P(stream.h) if stream is not None else None),
               "impc_batch_set_values_async")

    def get_async(self, x, y, info, stream=None):
        """impc_batch_get_async into HostArrays (any may be None), queued on `stream`."""
        ptr = lambda a: None if a is None else _P(a.ptr)  # noqa: E731
        _check(lib.impc_batch_get_async(self.h, ptr(x), ptr(y), ptr(info), _P(stream.h) if stream is not None else None),
               "impc_batch_get_async")

    def set_active(self, count):
        """impc_batch_set_active: the solves take the first `count` QPs."""
        _check(lib.impc_batch_set_active(self.h, int(count)), "impc_batch_set_active")

    def setup(self, stream=None):
        _check(lib.impc_batch_setup(self.h, stream), "impc_batch_setup")

    def solve(self, stream=None):
        _check(lib.impc_batch_solve(self.h, stream), "impc_batch_solve")

    def get(self):
        x = np.empty(self.B * self.n)
        y = np.empty(self.B * max(self.m, 1))
        info = np.empty(self.B, dtype=INFO_DTYPE)
        _check(lib.impc_batch_get(self.h, _d(x), _d(y), info.ctypes.data_as(C.c_void_p)), "impc_batch_get")
        return x.reshape(self.B, self.n), y[: self.B * self.m].reshape(self.B, self.m), info

    def set_time_limits(self, limits):
        """impc_batch_set_time_limits: per-QP time limits [B] in seconds (0 = none); None clears."""
        if limits is None:
            _check(lib.impc_batch_set_time_limits(self.h, None), "impc_batch_set_time_limits")
            return
        a = np.ascontiguousarray(limits, dtype=np.float64)
        if a.size != self.B:
            raise ValueError(f"set_time_limits: {a.size} values, expected B = {self.B}")
        _check(lib.impc_batch_set_time_limits(self.h, _d(a)), "impc_batch_set_time_limits")

    def set_queue_order(self, mode, q_weight=0.0):
        """impc_batch_set_queue_order: QUEUE_FIFO or QUEUE_LONGEST_FIRST (device-estimated difficulty
        key = warm-start violation + q_weight * ||q||_inf, descending)."""
        _check(lib.impc_batch_set_queue_order(self.h, int(mode), float(q_weight)), "impc_batch_set_queue_order")

    def set_persistent(self, on=True):
        _check(lib.impc_batch_set_persistent(self.h, int(on)), "impc_batch_set_persistent")

    def get_persistent(self):
        """impc_batch_get_persistent: (rho [B], x [B][n], z [B][m], y [B][m]) of the persistent
        workspaces -- the SCALED iterates OSQP keeps between solves, in OSQP's variable / row order."""
        rho, x = np.empty(self.B), np.empty((self.B, self.n))
        z, y = np.empty((self.B, self.m)), np.empty((self.B, self.m))
        _check(lib.impc_batch_get_persistent(self.h, _d(rho), _d(x), _d(z), _d(y)), "impc_batch_get_persistent")
        return rho, x, z, y

    def qp_latency(self):
        """Per-QP device solve latency (ms) of the last profiled structured solve."""
        ms = np.empty(self.B)
        _check(lib.impc_batch_get_qp_latency(self.h, _d(ms)), "impc_batch_get_qp_latency")
        return ms

    def device_results(self):
        x, y, info = _P(), _P(), _P()
        _check(lib.impc_batch_device_results(self.h, C.byref(x), C.byref(y), C.byref(info)),
               "impc_batch_device_results")
        return x.value, y.value, info.value

    def update_lin_cost(self, q):
        qa = np.ascontiguousarray(q, dtype=np.float64)
        if qa.size != self.B * self.n:
            raise ValueError(f"update_lin_cost: q has {qa.size} values, expected B*n = {self.B * self.n}")
        _check(lib.impc_batch_update_lin_cost(self.h, _d(qa)), "impc_batch_update_lin_cost")

    def update_bounds(self, l, u):
        la = np.ascontiguousarray(l, dtype=np.float64)
        ua = np.ascontiguousarray(u, dtype=np.float64)
        if la.size != self.B * self.m or ua.size != self.B * self.m:
            raise ValueError(f"update_bounds: l / u have {la.size} / {ua.size} values, expected B*m = "
                             f"{self.B * self.m}")
        _check(lib.impc_batch_update_bounds(self.h, _d(la), _d(ua)), "impc_batch_update_bounds")

    def follow_plan_device(self, horizon, ts, t, pos_ptr, vel_ptr, lin_ptr=None):
        """impc_batch_follow_plan_device: pos / vel [B][3] (device) = getPos(t) / getVel(t) of each
        QP's own last solution, lin [B][N][8] = its states (QPs with a solution)."""
        _check(lib.impc_batch_follow_plan_device(self.h, int(horizon), float(ts), float(t), _P(pos_ptr), _P(vel_ptr),
                                                 _P(lin_ptr) if lin_ptr else None), "impc_batch_follow_plan_device")

    def update_matrices_device(self, Px_ptr=None, Ax_ptr=None):
        """impc_batch_update_matrices_device: new P / A values [B][nnz] in device memory (None = unchanged)."""
        _check(lib.impc_batch_update_matrices_device(self.h, _P(Px_ptr) if Px_ptr else None,
                                                     _P(Ax_ptr) if Ax_ptr else None), "impc_batch_update_matrices_device")

    def update_matrices(self, Px=None, Ax=None):
        """impc_batch_update_matrices: new P / A values [B][nnz] (host; None = unchanged)."""
        P = None if Px is None else np.ascontiguousarray(Px, np.float64)
        A = None if Ax is None else np.ascontiguousarray(Ax, np.float64)
        if P is not None and P.size != self.B * self.nnzP:
            raise ValueError("update_matrices: Px must be [B][nnzP]")
        if A is not None and A.size != self.B * self.nnzA:
            raise ValueError("update_matrices: Ax must be [B][nnzA]")
        _check(lib.impc_batch_update_matrices(self.h, _d(P), _d(A)), "impc_batch_update_matrices")

    def update_lin_cost_device(self, q_ptr):
        """impc_batch_update_lin_cost_device: q [B][n] in device memory (address)."""
        _check(lib.impc_batch_update_lin_cost_device(self.h, _P(q_ptr)), "impc_batch_update_lin_cost_device")

    def update_bounds_device(self, l_ptr, u_ptr):
        """impc_batch_update_bounds_device: l, u [B][m] in device memory (addresses)."""
        _check(lib.impc_batch_update_bounds_device(self.h, _P(l_ptr), _P(u_ptr)), "impc_batch_update_bounds_device")

    def stats(self):
        s = Stats()
        _check(lib.impc_batch_get_stats(self.h, C.byref(s)), "impc_batch_get_stats")
        return {f: getattr(s, f) for f, _ in Stats._fields_}

    def set_kernel(self, kernel):
        """impc_batch_set_kernel: KERNEL_AUTO / KERNEL_GENERIC / KERNEL_STRUCTURED."""
        _check(lib.impc_batch_set_kernel(self.h, int(kernel)), "impc_batch_set_kernel")
        return self

    def set_profiling(self, on=True):
        _check(lib.impc_batch_set_profiling(self.h, 1 if on else 0), "impc_batch_set_profiling")

    def timings(self):
        a, b, c = C.c_double(), C.c_double(), C.c_double()
        _check(lib.impc_batch_get_timings(self.h, C.byref(a), C.byref(b), C.byref(c)), "impc_batch_get_timings")
        return a.value, b.value, c.value

    def close(self):
        if self.h:
            lib.impc_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ MPC -> QP builder
LIVE_PARAMS = dict(  # planner_param.yaml:25-39 + flight_base.yaml:8-9, ts from mpcNavigation.cpp:229
    horizon=20, num_half_space=0, ts=0.1, max_vel=5.0, max_acc=20.0, y_range_min=-5.0, y_range_max=5.0,
    z_range_min=0.5, z_range_max=4.5, static_safety_dist=0.8, dynamic_safety_dist=1.5, static_slack=0.01,
    dynamic_slack=0.2, position_weight=1000.0, velocity_weight=0.0, acceleration_weight=10.0,
    half_max=(0.0, 0.0, 0.0), half_min=(0.0, 0.0, 0.0))


def mpc_params(**kw):
    d = dict(LIVE_PARAMS)
    d.update(kw)
    p = MpcParams()
    for k, v in d.items():
        if k in ("half_max", "half_min"):
            getattr(p, k)[:] = list(v)
        else:
            setattr(p, k, v)
    return p, d


def mpc_dims(params, num_static, num_dynamic):
    dm = Dims()
    _check(lib.impc_mpc_dims(C.byref(params), num_static, num_dynamic, C.byref(dm)), "impc_mpc_dims")
    return dm.n, dm.m, dm.nnzP, dm.nnzA


def mpc_pattern(params, num_static, num_dynamic):
    n, m, nnzP, nnzA = mpc_dims(params, num_static, num_dynamic)
    Pp = np.empty(n + 1, np.int64)
    Pi = np.empty(max(nnzP, 1), np.int64)
    Ap = np.empty(n + 1, np.int64)
    Ai = np.empty(nnzA, np.int64)
    _check(lib.impc_mpc_build_pattern(C.byref(params), num_static, num_dynamic, _i(Pp), _i(Pi), _i(Ap), _i(Ai)),
           "impc_mpc_build_pattern")
    return dict(n=n, m=m, Pp=Pp, Pi=Pi[:nnzP], Ap=Ap, Ai=Ai)


def mpc_values(params, curr_pos, curr_vel, xref, lin_states=None, st_centroid=None, st_size=None, st_yaw=None,
               dyn_pos=None, dyn_size=None):
    """Batched castMPCToQP*: arrays with a leading batch axis.  Returns dict(Px, q, Ax, l, u)."""
    curr_pos = np.ascontiguousarray(curr_pos, dtype=np.float64)
    nb = curr_pos.shape[0]
    ns = 0 if st_centroid is None else int(st_centroid.shape[1])
    nd = 0 if dyn_pos is None else int(dyn_pos.shape[1])
    L = 0 if dyn_pos is None else int(dyn_pos.shape[2])
    n, m, nnzP, nnzA = mpc_dims(params, ns, nd)
    out = dict(Px=np.empty((nb, nnzP)), q=np.empty((nb, n)), Ax=np.empty((nb, nnzA)), l=np.empty((nb, m)),
               u=np.empty((nb, m)))

    def c(a):
        return None if a is None else np.ascontiguousarray(a, dtype=np.float64)

    args = [c(curr_pos), c(curr_vel), c(xref), c(lin_states), c(st_centroid), c(st_size), c(st_yaw), c(dyn_pos),
            c(dyn_size)]
    rc = lib.impc_mpc_build_values(C.byref(params), nb, _d(args[0]), _d(args[1]), _d(args[2]), _d(args[3]), ns,
                                   _d(args[4]), _d(args[5]), _d(args[6]), nd, L, _d(args[7]), _d(args[8]),
                                   _d(out["Px"]), _d(out["q"]), _d(out["Ax"]), _d(out["l"]), _d(out["u"]))
    _check(rc, "impc_mpc_build_values")
    return out


# ------------------------------------------------------------------ candidate selection
def select_best(ctx, params, x_ptrs, valid, first_time, prev_states, prev_count, xref, st_centroid, st_size,
                dyn_count, dyn_pos, dyn_size, prob):
    """impc_select_best: scoring + evaluateTraj for I instances x C candidates on the device.

    params: dict of impc_select_params fields; x_ptrs: [I*C] device addresses of the candidates'
    QP solutions (e.g. Batch.device_results()[0] + row * n * 8).  Returns dict(best_cand,
    best_pos, scores [I][C][3], weighted [I][C])."""
    sp = SelectParams(**params)
    I, Cn = np.asarray(valid).shape
    xp = np.ascontiguousarray(x_ptrs, dtype=np.uint64)
    arr = lambda a, t: np.ascontiguousarray(a, dtype=t)  # noqa: E731
    keep = dict(valid=arr(valid, np.int8), first=arr(first_time, np.int8), prev=arr(prev_states, np.float64),
                pc=arr(prev_count, np.int32), xref=arr(xref, np.float64), sc=arr(st_centroid, np.float64),
                ss=arr(st_size, np.float64), dc=arr(dyn_count, np.int32), dp=arr(dyn_pos, np.float64),
                ds=arr(dyn_size, np.float64), prob=arr(prob, np.float64))
    best = np.empty(I, np.int32)
    pos = np.empty(I, np.int32)
    scores = np.empty((I, Cn, 3))
    weighted = np.empty((I, Cn))
    v = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    _check(lib.impc_select_best(ctx.h, C.byref(sp), I, v(xp), v(keep["valid"]), v(keep["first"]), _d(keep["prev"]),
                                v(keep["pc"]), _d(keep["xref"]), _d(keep["sc"]), _d(keep["ss"]), v(keep["dc"]),
                                _d(keep["dp"]), _d(keep["ds"]), _d(keep["prob"]), v(best), v(pos), _d(scores),
                                _d(weighted)), "impc_select_best")
    return dict(best_cand=best, best_pos=pos, scores=scores, weighted=weighted)


def intent_fanout(ctx, curr_pos, first_time, prev_states, prev_count, dyn_cur, pred_pos, pred_size, prob):
    """impc_intent_fanout: findClosestObstacle + getIntentComb for I instances on the device.

    Shapes: curr_pos [I][3], first_time [I], prev_states [I][P][8], prev_count [I], dyn_cur
    [I][K][3], pred_pos / pred_size [I][K][4][L][3], prob [I][K][4].  Returns dict(ob_idx,
    cand_type [I][6], cand_slot [I][6], closest_prob [I][4], single_pos / single_size
    [I][4][K][L][3], pair_pos / pair_size [I][2][K+1][L][3])."""
    arr = lambda a, t: np.ascontiguousarray(a, dtype=t)  # noqa: E731
    pp = arr(pred_pos, np.float64)
    I, K, _, L, _ = pp.shape
    prev = arr(prev_states, np.float64).reshape(I, -1, 8)
    keep = [arr(curr_pos, np.float64), arr(first_time, np.int8), prev, arr(prev_count, np.int32),
            arr(dyn_cur, np.float64), pp, arr(pred_size, np.float64), arr(prob, np.float64)]
    out = dict(ob_idx=np.empty(I, np.int32), cand_type=np.empty((I, 6), np.int32), cand_slot=np.empty((I, 6), np.int32),
               closest_prob=np.empty((I, 4)), single_pos=np.empty((I, 4, K, L, 3)),
               single_size=np.empty((I, 4, K, L, 3)), pair_pos=np.empty((I, 2, K + 1, L, 3)),
               pair_size=np.empty((I, 2, K + 1, L, 3)))
    v = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    _check(lib.impc_intent_fanout(ctx.h, I, K, L, prev.shape[1], *[v(a) for a in keep], *[v(a) for a in out.values()]),
           "impc_intent_fanout")
    return out


class MpcBuilder:
    """impc_mpc_builder: on-device castMPCToQP* for one (horizon, #static, #dynamic) shape.
    build() takes device addresses (ints, e.g. torch tensor data_ptr()) and fills device output
    arrays, asynchronously on the context stream."""

    def __init__(self, ctx, params, num_static, num_dynamic, pred_len):
        self.ctx, self.params = ctx, params
        self.h = _P()
        _check(lib.impc_mpc_builder_create(ctx.h, C.byref(params), num_static, num_dynamic, pred_len,
                                           C.byref(self.h)), "impc_mpc_builder_create")

    def build(self, nb, curr_pos, curr_vel, xref, lin_states, st_centroid, st_size, st_yaw, dyn_pos, dyn_size,
              Px, q, Ax, l, u):
        ptrs = [curr_pos, curr_vel, xref, lin_states, st_centroid, st_size, st_yaw, dyn_pos, dyn_size, Px, q, Ax, l, u]
        _check(lib.impc_mpc_build_values_device(self.h, nb, *[_P(p) if p else None for p in ptrs], None),
               "impc_mpc_build_values_device")

    def close(self):
        if self.h:
            lib.impc_mpc_builder_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostArray:
    """Pinned host memory of the library (impc_host_alloc) viewed as a numpy array: the source /
    destination of asynchronous transfers (Batch.set_values_async / get_async)."""

    def __init__(self, ctx, shape, dtype=np.float64):
        self.ctx, self.shape, self.dtype = ctx, tuple(shape), np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        p = _P()
        _check(lib.impc_host_alloc(ctx.h, self.nbytes, C.byref(p)), "impc_host_alloc")
        self.ptr = p.value
        buf = (C.c_char * max(self.nbytes, 1)).from_address(self.ptr)
        self.a = np.frombuffer(buf, self.dtype, count=int(np.prod(self.shape, dtype=np.int64))).reshape(self.shape)

    def free(self):
        if self.ptr:
            self.a = None
            lib.impc_host_free(self.ctx.h, _P(self.ptr))
            self.ptr = None


class Stream:
    """An extra HIP stream of a context (impc_stream_create), for copy / compute pipelines."""

    def __init__(self, ctx):
        self.ctx = ctx
        p = _P()
        _check(lib.impc_stream_create(ctx.h, C.byref(p)), "impc_stream_create")
        self.h = p.value

    def wait(self, other):
        """This stream waits for the work queued on `other` (a Stream, or None = the context's)."""
        _check(lib.impc_stream_wait(self.ctx.h, _P(self.h), _P(other.h) if other is not None else None),
               "impc_stream_wait")

    def synchronize(self):
        _check(lib.impc_stream_synchronize(self.ctx.h, _P(self.h)), "impc_stream_synchronize")

    def close(self):
        if self.h:
            lib.impc_stream_destroy(self.ctx.h, _P(self.h))
            self.h = None


def ctx_stream_wait(ctx, stream):
    """The context's stream waits for the work queued on `stream` so far."""
    _check(lib.impc_stream_wait(ctx.h, None, _P(stream.h)), "impc_stream_wait")


class DeviceArray:
    """A device allocation of the library (impc_device_alloc) holding one numpy array's bytes."""

    def __init__(self, ctx, shape_or_array, dtype=np.float64):
        self.ctx = ctx
        if isinstance(shape_or_array, np.ndarray):
            host = np.ascontiguousarray(shape_or_array)
            self.shape, self.dtype = host.shape, host.dtype
        else:
            host = None
            self.shape, self.dtype = tuple(shape_or_array), np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        p = _P()
        _check(lib.impc_device_alloc(ctx.h, self.nbytes, C.byref(p)), "impc_device_alloc")
        self.ptr = p.value
        if host is not None:
            _check(lib.impc_copy_to_device(ctx.h, _P(self.ptr), host.ctypes.data_as(_P), self.nbytes),
                   "impc_copy_to_device")

    def get(self):
        out = np.empty(self.shape, self.dtype)
        _check(lib.impc_copy_to_host(self.ctx.h, out.ctypes.data_as(_P), _P(self.ptr), self.nbytes),
               "impc_copy_to_host")
        return out

    def set(self, arr):
        host = np.ascontiguousarray(arr, self.dtype)
        if host.shape != self.shape:
            raise ValueError(f"DeviceArray.set: shape {host.shape}, expected {self.shape}")
        _check(lib.impc_copy_to_device(self.ctx.h, _P(self.ptr), host.ctypes.data_as(_P), self.nbytes),
               "impc_copy_to_device")

    def free(self):
        if self.ptr:
            lib.impc_device_free(self.ctx.h, _P(self.ptr))
            self.ptr = None


class ReferencePaths:
    """Device state of mpcPlanner's reference tracking for `ni` planning instances: their input
    paths (updatePath, CSR-packed) and lastRefStartIdx_; xref() runs getReferenceTraj / getXRef
    on the device (impc_reference_traj_device) and advances the state."""

    def __init__(self, ctx, paths, ts, horizon):
        self.ctx, self.ts, self.horizon, self.ni = ctx, float(ts), int(horizon), len(paths)
        lens = np.array([len(p) for p in paths], np.int64)
        ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        flat = np.concatenate([np.asarray(p, np.float64).reshape(-1, 3) for p in paths]) if lens.sum() else \
            np.zeros((1, 3))
        self.d_ptr = DeviceArray(ctx, ptr)
        self.d_path = DeviceArray(ctx, np.ascontiguousarray(flat))
        self.d_last = DeviceArray(ctx, np.zeros(self.ni, np.int32))  # updatePath: lastRefStartIdx_ = 0

    def xref_device(self, curr_pos_ptr, out_ptr, repeat=1, stream=None):
        _check(lib.impc_reference_traj_device(self.ctx.h, self.horizon, self.ts, self.ni, _P(self.d_ptr.ptr),
                                              _P(self.d_path.ptr), _P(curr_pos_ptr), _P(self.d_last.ptr),
                                              int(repeat), _P(out_ptr), _P(stream) if stream else None),
               "impc_reference_traj_device")

    def xref(self, curr_pos, repeat=1):
        """Host convenience: curr_pos [ni][3] -> xref [ni][repeat][horizon][8] (via the device)."""
        cp = DeviceArray(self.ctx, np.ascontiguousarray(curr_pos, np.float64).reshape(self.ni, 3))
        out = DeviceArray(self.ctx, (self.ni, repeat, self.horizon, 8))
        try:
            self.xref_device(cp.ptr, out.ptr, repeat)
            return out.get()
        finally:
            cp.free()
            out.free()

    def last_idx(self):
        return self.d_last.get()

    def close(self):
        for d in (self.d_ptr, self.d_path, self.d_last):
            d.free()


def repeat_rows_device(ctx, src_ptr, rows, row_bytes, repeat, dst_ptr, stream=None):
    """impc_repeat_rows_device: dst row r * repeat + c = src row r (device pointers)."""
    _check(lib.impc_repeat_rows_device(ctx.h, _P(src_ptr), int(rows), int(row_bytes), int(repeat), _P(dst_ptr),
                                       _P(stream) if stream else None), "impc_repeat_rows_device")


def copy_rows_device(ctx, dst_ptr, dpitch, src_ptr, spitch, width, rows, stream=None):
    """impc_copy_rows_device: rows x width bytes, strided, device to device."""
    _check(lib.impc_copy_rows_device(ctx.h, _P(dst_ptr), int(dpitch), _P(src_ptr), int(spitch), int(width), int(rows),
                                     _P(stream) if stream else None), "impc_copy_rows_device")


def gather_rows_device(ctx, src_ptr, row_bytes, idx_ptr, count, dst_ptr, stream=None):
    """impc_gather_rows_device: dst row r = src row idx[r] (device pointers, idx int64)."""
    _check(lib.impc_gather_rows_device(ctx.h, _P(src_ptr), int(row_bytes), _P(idx_ptr), int(count), _P(dst_ptr),
                                       _P(stream) if stream else None), "impc_gather_rows_device")


def comm_unique_id():
    """impc_comm_unique_id (ncclGetUniqueId): 128 bytes for rank 0 to hand to every rank."""
    buf = (C.c_ubyte * COMM_ID_BYTES)()
    _check(lib.impc_comm_unique_id(buf), "impc_comm_unique_id")
    return bytes(buf)


class Comm:
    """RCCL communicator on a context's device (include/impc_comm.h): the cost-record all-gather of
    the multi-GPU path."""

    def __init__(self, ctx, uid, rank, world):
        self.ctx, self.rank, self.world = ctx, int(rank), int(world)
        buf = (C.c_ubyte * COMM_ID_BYTES).from_buffer_copy(bytes(uid))
        h = _P()
        _check(lib.impc_comm_create(ctx.h, buf, self.rank, self.world, C.byref(h)), "impc_comm_create")
        self.h = h

    def gather_info(self, batches, max_qps, recv_ptr, stream=None):
        """impc_comm_gather_info: this rank's batches' impc_info records, packed to max_qps and
        all-gathered into recv_ptr (device, world * max_qps records), on `stream`."""
        arr = (_P * len(batches))(*[b.h for b in batches])
        _check(lib.impc_comm_gather_info(self.h, arr, len(batches), int(max_qps), _P(recv_ptr),
                                         _P(stream) if stream else None), "impc_comm_gather_info")

    def allgather(self, send_ptr, recv_ptr, nbytes, stream=None):
        _check(lib.impc_comm_allgather(self.h, _P(send_ptr), _P(recv_ptr), int(nbytes), _P(stream) if stream else None),
               "impc_comm_allgather")

    def max(self, v):
        d = C.c_double(float(v))
        _check(lib.impc_comm_max(self.h, C.byref(d)), "impc_comm_max")
        return d.value

    def close(self):
        if self.h:
            lib.impc_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def solve_group(batches, stream=None):
    """impc_batch_solve_group: one persistent launch over several structured batches."""
    arr = (_P * len(batches))(*[b.h for b in batches])
    _check(lib.impc_batch_solve_group(arr, len(batches), _P(stream) if stream else None), "impc_batch_solve_group")


def shared_split(Px, Ax):
    """For a batch's QP-major Px [B][nnzP], Ax [B][nnzA]: (Px0, Ax0, var_pos, Ax_var) when P is the
    same for every QP (None otherwise); var_pos are the A positions whose value differs between
    QPs, Ax_var their per-QP values -- the inputs of Batch.set_values_shared."""
    Px, Ax = np.asarray(Px), np.asarray(Ax)
    if not (Px == Px[0]).all():
        return None
    var = np.flatnonzero((Ax != Ax[0]).any(axis=0))
    return Px[0], Ax[0], var, np.ascontiguousarray(Ax[:, var])


def intent_params(max_front_prob=0.5, front_angle_deg=10.0, stop_velocity=0.1, prob_scale=5.0):
    """impc_intent_params_from_config (defaults: the reference's predictor_param.yaml)."""
    ip = IntentParams()
    _check(lib.impc_intent_params_from_config(max_front_prob, front_angle_deg, stop_velocity, prob_scale,
                                              C.byref(ip)), "impc_intent_params_from_config")
    return ip


def intent_prob(ctx, ip, pos_hist, vel_hist, hist_len):
    """impc_intent_prob: pos_hist / vel_hist [count][H][3] (entry 0 newest), hist_len [count]."""
    ph = np.ascontiguousarray(pos_hist, np.float64)
    vh = np.ascontiguousarray(vel_hist, np.float64)
    hl = np.ascontiguousarray(hist_len, np.int32)
    count, H = ph.shape[0], ph.shape[1]
    out = np.empty((count, 4))
    v = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    _check(lib.impc_intent_prob(ctx.h, C.byref(ip), count, H, v(hl), v(ph), v(vh), v(out)), "impc_intent_prob")
    return out


def predict_traj(ctx, tp, omap, occ, pos, vel, size):
    """impc_predict_traj: per obstacle [count][3] inputs -> pred_pos, pred_size [count][4][P+1][3]."""
    v = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    occ = np.ascontiguousarray(occ, np.uint8)
    pos, vel, size = [np.ascontiguousarray(a, np.float64) for a in (pos, vel, size)]
    count = pos.shape[0]
    pp = np.empty((count, 4, tp.num_pred + 1, 3))
    ps = np.empty_like(pp)
    _check(lib.impc_predict_traj(ctx.h, C.byref(tp), C.byref(omap), v(occ), count, v(pos), v(vel), v(size), v(pp),
                                 v(ps)), "impc_predict_traj")
    return pp, ps
