"""ctypes wrapper of the CPU oracle (oracle/lafse3_oracle.c).

TEST INFRASTRUCTURE ONLY.  Only tests/, ``__graft_entry__.smoke()`` and bench.py's
``cpu_baseline`` leg may import this module; it is the parity checker, never the product
path (learningagileflight_se3_amd/ never imports it).

Reference behaviour restated here (file:line in yanrui89/LearningAgileFlight_SE3):
  quad_OC.py:104-212 (OCSys.ocSolver), quad_policy.py:67-112 (objective / sol_gradient),
  solid_geometry.py:104-168 (collis_det), quad_model.py:35-276 (model, costs, rotor tips).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liblafse3_oracle.so")

NX, NU = 13, 4


class OrcParams(ctypes.Structure):
    _fields_ = [
        ("mass", ctypes.c_double), ("Jx", ctypes.c_double), ("Jy", ctypes.c_double), ("Jz", ctypes.c_double),
        ("arm_l", ctypes.c_double), ("c_tau", ctypes.c_double), ("grav", ctypes.c_double), ("dt", ctypes.c_double),
        ("wrt", ctypes.c_double), ("wqt", ctypes.c_double), ("wthrust", ctypes.c_double), ("wrf", ctypes.c_double),
        ("wvf", ctypes.c_double), ("wqf", ctypes.c_double), ("wwf", ctypes.c_double),
        ("tra_w_peak", ctypes.c_double), ("tra_w_decay", ctypes.c_double), ("du_weight", ctypes.c_double),
        ("u_lb", ctypes.c_double), ("u_ub", ctypes.c_double), ("w_lb", ctypes.c_double), ("w_ub", ctypes.c_double),
        ("wing_len", ctypes.c_double), ("d_min", ctypes.c_double),
        ("horizon", ctypes.c_int32),
        ("max_iter", ctypes.c_int32),
        ("tol", ctypes.c_double), ("acceptable_tol", ctypes.c_double),
        ("acceptable_iter", ctypes.c_int32),
        ("mu_init", ctypes.c_double), ("bound_relax", ctypes.c_double),
        ("lsq_mult_init", ctypes.c_int32), ("t_probe_f32", ctypes.c_int32),
        ("max_soc", ctypes.c_int32),
        ("restoration", ctypes.c_int32),
        ("watchdog", ctypes.c_int32),
        ("grad_mode", ctypes.c_int32),
    ]


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc, no reference sources involved)."""
    src = os.path.join(_HERE, "lafse3_oracle.c")
    fast = os.path.join(_HERE, "liblafse3_oracle_fast.so")
    stale = [p for p in (_LIB_PATH, fast) if not os.path.exists(p) or os.path.getmtime(p) < os.path.getmtime(src)]
    if force or stale:
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


_lib = None
_lib_fast = None
_LIB_FAST_PATH = os.path.join(_HERE, "liblafse3_oracle_fast.so")


def lib(fast: bool = False):
    """The parity build (default) or, with fast=True, the -O3 / FMA timing build used by bench.py's
    cpu_baseline leg (same source, same algorithm; results agree to rounding)."""
    global _lib, _lib_fast
    if fast:
        if _lib_fast is None:
            build()
            _lib_fast = _bind(ctypes.CDLL(_LIB_FAST_PATH))
        return _lib_fast
    if _lib is None:
        build()
        _lib = _bind(ctypes.CDLL(_LIB_PATH))
    return _lib


def _bind(L):
    if True:
        P = ctypes.POINTER
        d, i32, i64 = ctypes.c_double, ctypes.c_int32, ctypes.c_int64
        pd, pi, pf = P(d), P(i32), P(ctypes.c_float)
        L.orc_default_params.argtypes = [P(OrcParams)]
        L.orc_params_size.restype = ctypes.c_int
        L.orc_pow15.restype = ctypes.c_double
        L.orc_pow15.argtypes = [ctypes.c_double]
        L.orc_solve_q.argtypes = [P(OrcParams), i64, pd, pd, pd, pd, pd, pd, pd, pd, pd, pd, pi, pi]
        L.orc_reward.argtypes = [P(OrcParams), i64, pd, pd, pd, pd, pi]
        L.orc_collis_det.argtypes = [i64, ctypes.c_int, pd, pd, pd, pi, pi]
        L.orc_model_eval.argtypes = [P(OrcParams), i64, pd, pd, pd, pd, pd, pd, pd, pd]
        L.orc_cost_eval.argtypes = [P(OrcParams), i64, pd, pd, pd, pd, pd, pd, pd, pd, pd]
        L.orc_sol_gradient.argtypes = [P(OrcParams), i64, pd, pd, pd, pf, pd, pd, pd, pi]
        L.orc_rd2quat.argtypes = [d, pd, pd]
        L.orc_grad_params.argtypes = [P(OrcParams), i64, pf, pd, pd, pd, pi]
        L.orc_assemble.argtypes = [P(OrcParams), i64, pd, pf, pd]
        L.orc_num_threads.restype = ctypes.c_int
        L.orc_debug_trace.argtypes = [pd, ctypes.c_int]
        L.orc_debug_dump.argtypes = [pd, ctypes.c_int, ctypes.c_int]
        L.orc_debug_final_err.argtypes = [pd]
        L.orc_debug_grad_iters.argtypes = [pi]
        L.orc_set_num_threads.argtypes = [ctypes.c_int]
        assert L.orc_params_size() == ctypes.sizeof(OrcParams), "OrcParams layout mismatch"
    return L


def default_params(**kw) -> OrcParams:
    p = OrcParams()
    lib().orc_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _ptr(a, ct=ctypes.c_double):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ct))


def _c(a, dt=np.float64):
    if a is None:
        return None
    return np.ascontiguousarray(a, dtype=dt)


def rd2quat(a, a_norm=None):
    """Rd2Rp + toQuaternion (quad_policy.py:10-13, quad_model.py:818-825)."""
    a = _c(a).reshape(3)
    if a_norm is None:
        a_norm = float(np.sqrt(a @ a))
    q = np.zeros(4)
    lib().orc_rd2quat(float(a_norm), _ptr(a), _ptr(q))
    return q


def solve(ini, goal, ptra, qtra, t, ulast=None, params=None, fast=False):
    """Batched OCSys.ocSolver restatement (quaternion traversal attitude). Returns dict of arrays.
    fast=True runs the -O3 / FMA timing build (bench.py cpu_baseline)."""
    p = params or default_params()
    ini, goal, ptra, qtra = _c(ini).reshape(-1, NX), _c(goal).reshape(-1, 3), _c(ptra).reshape(-1, 3), _c(qtra).reshape(-1, 4)
    B = ini.shape[0]
    t = _c(np.broadcast_to(np.asarray(t, dtype=np.float64), (B,)))
    ulast = None if ulast is None else _c(np.broadcast_to(ulast, (B, 4)))
    N = p.horizon
    x = np.zeros((B, N + 1, NX)); u = np.zeros((B, N, NU)); lam = np.zeros((B, N, NX))
    cost = np.zeros(B); st = np.zeros(B, np.int32); cnt = np.zeros((B, 3), np.int32)
    rc = lib(fast).orc_solve_q(ctypes.byref(p), B, _ptr(ini), _ptr(goal), _ptr(ptra), _ptr(qtra), _ptr(t), _ptr(ulast),
                           _ptr(x), _ptr(u), _ptr(lam), _ptr(cost), _ptr(st, ctypes.c_int32), _ptr(cnt, ctypes.c_int32))
    assert rc == 0
    return {"x": x, "u": u, "lam": lam, "cost": cost, "status": st, "iters": cnt[:, 0], "sweeps": cnt[:, 1],
            "trials": cnt[:, 2]}


def reward(x, goal, gate12, params=None):
    p = params or default_params()
    x, goal, gate12 = _c(x), _c(goal).reshape(-1, 3), _c(gate12).reshape(-1, 12)
    B = goal.shape[0]
    r = np.zeros(B); br = np.zeros((B, 4), np.int32)
    lib().orc_reward(ctypes.byref(p), B, _ptr(x), _ptr(goal), _ptr(gate12), _ptr(r), _ptr(br, ctypes.c_int32))
    return r, br


def collis_det(gate12, tracks):
    gate12, tracks = _c(gate12).reshape(-1, 12), _c(tracks)
    B, H1 = tracks.shape[0], tracks.shape[1]
    out = np.zeros(B); br = np.zeros(B, np.int32); co = np.zeros(B, np.int32)
    lib().orc_collis_det(B, H1 - 1, _ptr(gate12), _ptr(tracks), _ptr(out), _ptr(br, ctypes.c_int32), _ptr(co, ctypes.c_int32))
    return out, br, co


def model_eval(x, u, lam, params=None):
    p = params or default_params()
    x, u, lam = _c(x).reshape(-1, NX), _c(u).reshape(-1, NU), _c(lam).reshape(-1, NX)
    n = x.shape[0]
    f = np.zeros((n, NX)); A = np.zeros((n, NX, NX)); B = np.zeros((n, NX, NU))
    Hxx = np.zeros((n, NX, NX)); Hxu = np.zeros((n, NX, NU))
    lib().orc_model_eval(ctypes.byref(p), n, _ptr(x), _ptr(u), _ptr(lam), _ptr(f), _ptr(A), _ptr(B), _ptr(Hxx), _ptr(Hxu))
    return f, A, B, Hxx, Hxu


def cost_eval(x, goal, ptra, qtra, wk, params=None):
    p = params or default_params()
    x = _c(x).reshape(-1, NX)
    n = x.shape[0]
    goal, ptra, qtra = _c(goal).reshape(n, 3), _c(ptra).reshape(n, 3), _c(qtra).reshape(n, 4)
    wk = _c(np.broadcast_to(wk, (n,)))
    path = np.zeros(n); tra = np.zeros(n); g = np.zeros((n, NX)); H = np.zeros((n, NX, NX))
    lib().orc_cost_eval(ctypes.byref(p), n, _ptr(x), _ptr(goal), _ptr(ptra), _ptr(qtra), _ptr(wk), _ptr(path), _ptr(tra),
                        _ptr(g), _ptr(H))
    return path, tra, g, H


def sol_gradient(ini, goal, gate12, dnn_out, ulast=None, params=None, fast=False, iters=None):
    """Batched run_quad.sol_gradient restatement (quad_policy.py:94-112); dnn_out float32 (B,7).
    fast=True runs the -O3 / FMA timing build (bench.py cpu_baseline).  iters: optional int32 (B, 9) array
    that receives every job's IPM iteration count (rewards9 slot order)."""
    p = params or default_params()
    ini, goal, gate12 = _c(ini).reshape(-1, NX), _c(goal).reshape(-1, 3), _c(gate12).reshape(-1, 12)
    dnn = _c(dnn_out, np.float32).reshape(-1, 7)
    B = ini.shape[0]
    ulast = None if ulast is None else _c(np.broadcast_to(ulast, (B, 4)))
    out8 = np.zeros((B, 8)); R = np.zeros((B, 9)); st = np.zeros((B, 9), np.int32)
    if iters is not None:
        assert iters.dtype == np.int32 and iters.shape == (B, 9) and iters.flags.c_contiguous
        lib(fast).orc_debug_grad_iters(_ptr(iters, ctypes.c_int32))
    try:
        rc = lib(fast).orc_sol_gradient(ctypes.byref(p), B, _ptr(ini), _ptr(goal), _ptr(gate12),
                                        _ptr(dnn, ctypes.c_float), _ptr(ulast), _ptr(out8), _ptr(R),
                                        _ptr(st, ctypes.c_int32))
    finally:
        if iters is not None:
            lib(fast).orc_debug_grad_iters(None)
    assert rc == 0
    return out8, R, st


def grad_params(dnn_out, params=None):
    """Per-solve (p_tra, q_tra, t, uses_Ulast) of the 9 solves of sol_gradient (quad_policy.py:97-110)."""
    p = params or default_params()
    dnn = _c(dnn_out, np.float32).reshape(-1, 7)
    B = dnn.shape[0]
    pp = np.zeros((B, 9, 3)); qq = np.zeros((B, 9, 4)); tt = np.zeros((B, 9)); uu = np.zeros((B, 9), np.int32)
    lib().orc_grad_params(ctypes.byref(p), B, _ptr(dnn, ctypes.c_float), _ptr(pp), _ptr(qq), _ptr(tt),
                          _ptr(uu, ctypes.c_int32))
    return pp, qq, tt, uu


def assemble(R9, dnn_out, params=None):
    """out8 of sol_gradient from the 9 rewards per sample (quad_policy.py:97-112)."""
    p = params or default_params()
    R9 = _c(R9).reshape(-1, 9)
    dnn = _c(dnn_out, np.float32).reshape(-1, 7)
    out8 = np.zeros((R9.shape[0], 8))
    lib().orc_assemble(ctypes.byref(p), R9.shape[0], _ptr(R9), _ptr(dnn, ctypes.c_float), _ptr(out8))
    return out8


def debug_trace(buf=None, iters=0):
    """Debug: per-iteration trace of subsequent solve() calls into buf (B, iters, 12)."""
    global _trace_keep
    _trace_keep = buf
    lib().orc_debug_trace(_ptr(buf), int(iters))


def debug_dump(buf=None, it=-1, after_refine=False):
    """Debug: Newton step [dx 51x13 | du 50x4 | lam+ 50x13] of iteration `it` into buf (B, 1513)."""
    global _dump_keep
    _dump_keep = buf
    lib().orc_debug_dump(_ptr(buf), int(it), int(after_refine))


def debug_final_err(buf=None, fast: bool = False):
    """Debug: [overall NLP error, unscaled dual inf, primal inf, unscaled compl] at the last iterate of
    subsequent solve() calls into buf (B, 4) (None disables)."""
    global _final_keep
    _final_keep = buf
    lib(fast).orc_debug_final_err(_ptr(buf))


def num_threads(fast: bool = False) -> int:
    return int(lib(fast).orc_num_threads())


def set_num_threads(n: int, fast: bool = False):
    lib(fast).orc_set_num_threads(int(n))
