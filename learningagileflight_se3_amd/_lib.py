"""ctypes binding of liblafse3.so (the C ABI declared in include/lafse3.h).

The shared library is built in-tree by ``learningagileflight_se3_amd.build.build()`` (hipcc,
--offload-arch=gfx950).  There is no fallback: if the library is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# LAFSE3_LIB overrides the library path (A/B experiments with alternative builds of the same ABI)
LIB_PATH = os.environ.get("LAFSE3_LIB", os.path.join(_HERE, "liblafse3.so"))

NX, NU, MAX_N = 13, 4, 50
VARIANT_WAVE = 1   # include/lafse3.h LAFSE3_VARIANT_WAVE (the only kernel variant)
STATUS_NAMES = {0: "solved", 1: "acceptable", 2: "max_iter", 3: "line_search_failed", 4: "non_finite",
                5: "tiny_step", 6: "regularization_failed", 7: "device_error",
                8: "restoration_failed", 9: "infeasible"}


class Params(ctypes.Structure):
    """Mirror of ``lafse3_params`` (include/lafse3.h)."""
    _fields_ = [
        ("mass", ctypes.c_double), ("Jx", ctypes.c_double), ("Jy", ctypes.c_double), ("Jz", ctypes.c_double),
        ("arm_l", ctypes.c_double), ("c_tau", ctypes.c_double), ("grav", ctypes.c_double), ("dt", ctypes.c_double),
        ("wrt", ctypes.c_double), ("wqt", ctypes.c_double), ("wthrust", ctypes.c_double), ("wrf", ctypes.c_double),
        ("wvf", ctypes.c_double), ("wqf", ctypes.c_double), ("wwf", ctypes.c_double),
        ("tra_w_peak", ctypes.c_double), ("tra_w_decay", ctypes.c_double), ("du_weight", ctypes.c_double),
        ("u_lb", ctypes.c_double), ("u_ub", ctypes.c_double), ("w_lb", ctypes.c_double), ("w_ub", ctypes.c_double),
        ("wing_len", ctypes.c_double), ("d_min", ctypes.c_double),
        ("horizon", ctypes.c_int32), ("max_iter", ctypes.c_int32),
        ("tol", ctypes.c_double), ("acceptable_tol", ctypes.c_double),
        ("acceptable_iter", ctypes.c_int32),
        ("mu_init", ctypes.c_double), ("bound_relax", ctypes.c_double),
        ("lsq_mult_init", ctypes.c_int32), ("variant", ctypes.c_int32),
        ("max_soc", ctypes.c_int32), ("costate_option", ctypes.c_int32),
        ("grad_mode", ctypes.c_int32), ("restoration", ctypes.c_int32),
        ("watchdog", ctypes.c_int32),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# exported symbol -> (restype, argtypes)
_P = ctypes.POINTER
_vp, _d, _i32, _i64 = ctypes.c_void_p, ctypes.c_double, ctypes.c_int32, ctypes.c_int64
SIGNATURES = {
    "lafse3_default_params": (ctypes.c_int, [_P(Params)]),
    "lafse3_create": (ctypes.c_int, [_P(_vp), ctypes.c_int]),
    "lafse3_destroy": (ctypes.c_int, [_vp]),
    "lafse3_set_params": (ctypes.c_int, [_vp, _P(Params)]),
    "lafse3_get_params": (ctypes.c_int, [_vp, _P(Params)]),
    "lafse3_reserve": (ctypes.c_int, [_vp, _i64]),
    "lafse3_workspace_bytes_per_instance": (_i64, []),
    "lafse3_stream_create": (ctypes.c_int, [ctypes.c_int, _P(_vp)]),
    "lafse3_stream_destroy": (ctypes.c_int, [_vp]),
    "lafse3_ocp_solve": (ctypes.c_int, [_vp, _i64] + [_vp] * 6 + [_vp] * 6 + [_vp]),
    "lafse3_ocp_solve_f32": (ctypes.c_int, [_vp, _i64] + [_vp] * 6 + [_vp] * 6 + [_vp]),
    "lafse3_objective": (ctypes.c_int, [_vp, _i64] + [_vp] * 7 + [_vp, _vp, _vp]),
    "lafse3_sol_gradient": (ctypes.c_int, [_vp, _i64] + [_vp] * 5 + [_vp, _vp, _vp, _vp]),
    "lafse3_get_input": (ctypes.c_int, [_vp, _i64] + [_vp] * 4 + [_vp, _vp, _vp, _vp]),
    "lafse3_traversal_time": (ctypes.c_int, [_vp, _i64] + [_vp] * 4 + [ctypes.c_double] + [_vp] * 4),
    "lafse3_dnn2_weight_count": (ctypes.c_int, []),
    "lafse3_reward": (ctypes.c_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "lafse3_last_kernel_ms": (ctypes.c_float, [_vp]),
    "lafse3_last_counters": (ctypes.c_int, [_vp, _P(_i64)]),
    "lafse3_debug_trace": (ctypes.c_int, [_vp, _vp, ctypes.c_int]),
    "lafse3_debug_dump": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int]),
    "lafse3_debug_timers": (ctypes.c_int, [_vp, _vp]),
    "lafse3_record_iters": (ctypes.c_int, [_vp, _vp, _i64]),
    "lafse3_check_device": (ctypes.c_int, [_vp]),
    "lafse3_last_resto_counters": (ctypes.c_int, [_vp, _P(_i64)]),
    "lafse3_debug_drop_push": (ctypes.c_int, [_vp, _i64]),
    "lafse3_last_error": (ctypes.c_char_p, []),
    "lafse3_version": (ctypes.c_char_p, []),
}

_lib = None


class Lafse3Error(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load liblafse3.so; raises Lafse3Error (never falls back) when it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise Lafse3Error(f"{LIB_PATH} not built: run learningagileflight_se3_amd.build.build() "
                              "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        override = "LAFSE3_LIB" in os.environ   # A/B runs against an older build: its missing entry points stay unset
        for name, (res, args) in SIGNATURES.items():
            if override and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().lafse3_last_error().decode(errors="replace")
        raise Lafse3Error(f"{what} failed (rc={rc}): {msg}")


def default_params(**overrides) -> Params:
    p = Params()
    check(load().lafse3_default_params(ctypes.byref(p)), "lafse3_default_params")
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise KeyError(k)
        setattr(p, k, v)
    return p
