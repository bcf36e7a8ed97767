"""Batched MPC solve / objective / gradient on MI355X through liblafse3.so.

``Engine`` owns one C-ABI context (device workspace + parameters) and takes torch tensors that
already live in HBM.  Every method is asynchronous on the current torch stream and returns tensors
allocated on the same device.  Host numpy inputs are accepted for convenience (copied to the device).

Reference interfaces mirrored (yanrui89/LearningAgileFlight_SE3):
  Engine.ocp_solve     OCSys.ocSolver          quad_OC.py:104-212
  Engine.objective     run_quad.objective      quad_policy.py:67-91
  Engine.sol_gradient  run_quad.sol_gradient   quad_policy.py:94-112
  Engine.get_input     run_quad.get_input      quad_policy.py:202-211
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import NU, NX, Params, check, load


def _dev_tensor(a, shape_tail, dtype, device, name, allow_none=False):
    if a is None:
        if allow_none:
            return None
        raise ValueError(f"{name} is required")
    t = a if isinstance(a, torch.Tensor) else torch.as_tensor(np.asarray(a))
    t = t.to(device=device, dtype=dtype)
    if t.dim() == len(shape_tail):
        t = t.unsqueeze(0)
    if tuple(t.shape[1:]) != tuple(shape_tail):
        raise ValueError(f"{name}: expected (B, {', '.join(map(str, shape_tail))}), got {tuple(t.shape)}")
    return t.contiguous()


def _same_batch(B, **named):
    """Every per-sample argument must carry the batch of ini_state (the kernels index row b < B of each);
    u_last alone may be one row, broadcast to the batch.  Returns the (possibly expanded) tensors."""
    out = []
    for name, v in named.items():
        if v is not None and v.shape[0] != B:
            if name == "u_last" and v.shape[0] == 1:
                v = v.expand(B, *v.shape[1:]).contiguous()
            else:
                raise ValueError(f"{name}: batch {v.shape[0]} != {B} (the batch of ini_state)")
        out.append(v)
    return out


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class QueueStream:
    """A torch stream (``.stream``, a torch.cuda.ExternalStream) on a hardware queue of its own
    (lafse3_stream_create): for contexts whose launches are meant to overlap, e.g. the episode groups of the
    moving-gate loop.  Two ordinary torch streams can share one of HIP's pooled hardware queues and then run
    their kernels back to back (profiles/r05_moving_trace.log).  ``close()`` synchronizes and destroys the stream;
    the solver contexts that launched on it stay usable (their counters are read on a stream of their own after the
    launch's end event, api.hip read_counters)."""

    def __init__(self, device=None):
        d = torch.device("cuda") if device is None else torch.device(device)
        # a device without an index ("cuda") is the current device, as torch reads it
        self.device = torch.device("cuda", torch.cuda.current_device() if d.index is None else d.index)
        self._L = load()
        self._h = ctypes.c_void_p()
        check(self._L.lafse3_stream_create(self.device.index, ctypes.byref(self._h)), "lafse3_stream_create")
        self.stream = torch.cuda.ExternalStream(self._h.value, device=self.device)

    def close(self):
        if self._h.value:
            self.stream.synchronize()
            check(self._L.lafse3_stream_destroy(self._h), "lafse3_stream_destroy")
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    """One solver context on one HIP device (``device=None``: torch's current device)."""

    def __init__(self, params: Params | None = None, device=None, **overrides):
        if not torch.cuda.is_available():
            raise _lib.Lafse3Error("no HIP device visible: the MI355X engine has no CPU fallback")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        self._L = load()
        self._ctx = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self._L.lafse3_create(ctypes.byref(self._ctx), self.device.index), "lafse3_create")
        p = params if params is not None else _lib.default_params()
        for k, v in overrides.items():
            setattr(p, k, v)
        self.set_params(p)

    # ------------------------------------------------------------------ params / resources
    def set_params(self, p: Params):
        check(self._L.lafse3_set_params(self._ctx, ctypes.byref(p)), "lafse3_set_params")
        self.params = p

    @property
    def horizon(self) -> int:
        return int(self.params.horizon)

    def reserve(self, n_instances: int):
        check(self._L.lafse3_reserve(self._ctx, int(n_instances)), "lafse3_reserve")

    def close(self):
        if getattr(self, "_ctx", None) is not None and self._ctx.value:
            self._L.lafse3_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_kernel_ms(self) -> float:
        return float(self._L.lafse3_last_kernel_ms(self._ctx))

    def last_counters(self) -> dict:
        c = (ctypes.c_int64 * 3)()
        check(self._L.lafse3_last_counters(self._ctx, c), "lafse3_last_counters")
        return {"iterations": int(c[0]), "sweeps": int(c[1]), "trials": int(c[2])}

    def last_resto_counters(self) -> dict:
        """Restoration-phase entries and successful returns of the last launch (lafse3_last_resto_counters)."""
        c = (ctypes.c_int64 * 2)()
        check(self._L.lafse3_last_resto_counters(self._ctx, c), "lafse3_last_resto_counters")
        return {"resto_entries": int(c[0]), "resto_returns": int(c[1])}

    def debug_trace(self, buf=None, iters: int = 0):
        """Debug: per-iteration IPM trace into a (instances, iters, 16) float64 device tensor."""
        self._trace_buf = buf
        check(self._L.lafse3_debug_trace(self._ctx, _ptr(buf), int(iters)), "lafse3_debug_trace")

    def debug_dump(self, buf=None, it: int = -1, after_refine: bool = False):
        """Debug: Newton step of iteration `it` into a (instances, 1513) float64 device tensor."""
        self._dump_buf = buf
        check(self._L.lafse3_debug_dump(self._ctx, _ptr(buf), int(it), int(after_refine)), "lafse3_debug_dump")

    def debug_timers(self, buf=None):
        """Debug: per-instance phase timers + placement record into an (instances, 32) int64 device tensor (None disables)."""
        self._timer_buf = buf
        check(self._L.lafse3_debug_timers(self._ctx, _ptr(buf)), "lafse3_debug_timers")

    def record_iters(self, buf=None):
        """Per-instance IPM iteration counts of later launches into an int32 device tensor (one entry per NLP
        instance, sol_gradient: (B, 9) in rewards9 order); None disables.  A launch that would write more
        entries than buf holds raises."""
        if buf is not None and (buf.dtype != torch.int32 or not buf.is_contiguous() or buf.device != self.device):
            raise ValueError("record_iters: a contiguous int32 tensor on the engine's device is required")
        self._iters_buf = buf
        check(self._L.lafse3_record_iters(self._ctx, _ptr(buf), 0 if buf is None else buf.numel()),
              "lafse3_record_iters")

    def check_device(self):
        """Wait for the last launch and raise Lafse3Error if the kernel raised its device error word (a lost
        sol_gradient probe task: its rewards9 slot is NaN and its status9 entry 7)."""
        check(self._L.lafse3_check_device(self._ctx), "lafse3_check_device")

    def debug_drop_push(self, sample: int = -1):
        """Debug: withhold the probe-queue entry of `sample` in later sol_gradient launches (-1 disables)."""
        check(self._L.lafse3_debug_drop_push(self._ctx, int(sample)), "lafse3_debug_drop_push")

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ hot path
    def ocp_solve(self, ini_state, goal, p_tra, a_tra, t, u_last=None, want=("x", "u", "lam", "cost"),
                  costate_option: int | None = None, dtype=torch.float64):
        """Batched OCSys.ocSolver. Returns dict of device tensors (x, u, lam, cost, status, iters).

        ``costate_option`` (quad_OC.py:104 argument): 0 = IPOPT lam_g, 1 = PMP costates (quad_OC.py:188-201);
        None keeps the context's parameter.  ``dtype=torch.float32`` uses the fp32 twin
        (lafse3_ocp_solve_f32: float32 buffers at the boundary, fp64 solve inside).
        """
        if costate_option is not None and int(costate_option) != int(self.params.costate_option):
            saved = self.params.costate_option
            self.params.costate_option = int(costate_option)
            self.set_params(self.params)
            try:
                return self.ocp_solve(ini_state, goal, p_tra, a_tra, t, u_last, want, dtype=dtype)
            finally:
                self.params.costate_option = saved
                self.set_params(self.params)
        f32 = dtype == torch.float32
        d, f64 = self.device, (torch.float32 if f32 else torch.float64)
        ini = _dev_tensor(ini_state, (NX,), f64, d, "ini_state")
        B = ini.shape[0]
        goal = _dev_tensor(goal, (3,), f64, d, "goal")
        p = _dev_tensor(p_tra, (3,), f64, d, "p_tra")
        a = _dev_tensor(a_tra, (3,), f64, d, "a_tra")
        tt = torch.as_tensor(t, dtype=f64).to(d).reshape(-1).expand(B).contiguous()
        ul = _dev_tensor(u_last, (NU,), f64, d, "u_last", allow_none=True)
        goal, p, a, ul = _same_batch(B, goal=goal, p_tra=p, a_tra=a, u_last=ul)
        N = self.horizon
        out = {
            "x": torch.empty((B, N + 1, NX), dtype=f64, device=d) if "x" in want else None,
            "u": torch.empty((B, N, NU), dtype=f64, device=d) if "u" in want else None,
            "lam": torch.empty((B, N, NX), dtype=f64, device=d) if "lam" in want else None,
            "cost": torch.empty((B,), dtype=f64, device=d) if "cost" in want else None,
            "status": torch.empty((B,), dtype=torch.int32, device=d),
            "iters": torch.empty((B,), dtype=torch.int32, device=d),
        }
        fn = self._L.lafse3_ocp_solve_f32 if f32 else self._L.lafse3_ocp_solve
        check(fn(self._ctx, B, _ptr(ini), _ptr(goal), _ptr(p), _ptr(a), _ptr(tt), _ptr(ul),
                 _ptr(out["x"]), _ptr(out["u"]), _ptr(out["lam"]), _ptr(out["cost"]),
                 _ptr(out["status"]), _ptr(out["iters"]), self._stream()),
              "lafse3_ocp_solve_f32" if f32 else "lafse3_ocp_solve")
        return {k: v for k, v in out.items() if v is not None}

    def objective(self, ini_state, goal, gate12, p_tra, a_tra, t, u_last=None):
        """Batched run_quad.objective -> (reward (B,), status (B,))."""
        d, f64 = self.device, torch.float64
        ini = _dev_tensor(ini_state, (NX,), f64, d, "ini_state")
        B = ini.shape[0]
        goal = _dev_tensor(goal, (3,), f64, d, "goal")
        g12 = _dev_tensor(gate12, (12,), f64, d, "gate12")
        p = _dev_tensor(p_tra, (3,), f64, d, "p_tra")
        a = _dev_tensor(a_tra, (3,), f64, d, "a_tra")
        tt = torch.as_tensor(t, dtype=f64).to(d).reshape(-1).expand(B).contiguous()
        ul = _dev_tensor(u_last, (NU,), f64, d, "u_last", allow_none=True)
        goal, g12, p, a, ul = _same_batch(B, goal=goal, gate12=g12, p_tra=p, a_tra=a, u_last=ul)
        R = torch.empty((B,), dtype=f64, device=d)
        st = torch.empty((B,), dtype=torch.int32, device=d)
        check(self._L.lafse3_objective(self._ctx, B, _ptr(ini), _ptr(goal), _ptr(g12), _ptr(p), _ptr(a), _ptr(tt),
                                       _ptr(ul), _ptr(R), _ptr(st), self._stream()), "lafse3_objective")
        return R, st

    def sol_gradient(self, ini_state, goal, gate12, dnn_out, u_last=None, want_rewards=False, grad_mode=None,
                     verify=True):
        """Batched run_quad.sol_gradient: dnn_out (B,7) float32 -> out8 (B,8) float64 [+ rewards9, status9].
        ``grad_mode``: None = the context's setting, 0 = FD (9 solves, the reference), 1 = IFT (3 solves +
        six sensitivity sweeps, lafse3.h).  ``verify``: wait for the launch and raise Lafse3Error when a probe
        task was lost (its out8 row would carry a NaN into the DNN1 update); False leaves the launch
        asynchronous -- the caller then checks (check_device / last_counters) before using out8."""
        if grad_mode is not None and int(grad_mode) != int(self.params.grad_mode):
            saved = self.params.grad_mode
            self.params.grad_mode = int(grad_mode)
            self.set_params(self.params)
            try:
                return self.sol_gradient(ini_state, goal, gate12, dnn_out, u_last, want_rewards, verify=verify)
            finally:
                self.params.grad_mode = saved
                self.set_params(self.params)
        d, f64 = self.device, torch.float64
        ini = _dev_tensor(ini_state, (NX,), f64, d, "ini_state")
        B = ini.shape[0]
        goal = _dev_tensor(goal, (3,), f64, d, "goal")
        g12 = _dev_tensor(gate12, (12,), f64, d, "gate12")
        dnn = _dev_tensor(dnn_out, (7,), torch.float32, d, "dnn_out")
        ul = _dev_tensor(u_last, (NU,), f64, d, "u_last", allow_none=True)
        goal, g12, dnn, ul = _same_batch(B, goal=goal, gate12=g12, dnn_out=dnn, u_last=ul)
        out8 = torch.empty((B, 8), dtype=f64, device=d)
        R9 = torch.empty((B, 9), dtype=f64, device=d) if want_rewards else None
        S9 = torch.empty((B, 9), dtype=torch.int32, device=d) if want_rewards else None
        check(self._L.lafse3_sol_gradient(self._ctx, B, _ptr(ini), _ptr(goal), _ptr(g12), _ptr(dnn), _ptr(ul),
                                          _ptr(out8), _ptr(R9), _ptr(S9), self._stream()), "lafse3_sol_gradient")
        if verify:
            self.check_device()
        if want_rewards:
            return out8, R9, S9
        return out8

    def dnn2_weights(self, net):
        """DNN2 (18-128-128-7 nn.Module, e.g. nn3_1.pth's weights) packed as lafse3_traversal_time expects:
        l1.weight, l1.bias, l2.weight, l2.bias, l3.weight row 6, l3.bias[6] (float32, device).
        Cached per module until its parameters change."""
        key = (id(net), tuple(p._version for p in net.parameters()))
        cached = getattr(self, "_dnn2_cache", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        sd = {k: v.detach().to(device=self.device, dtype=torch.float32) for k, v in net.state_dict().items()}
        if sd["l1.weight"].shape != (128, 18) or sd["l2.weight"].shape != (128, 128) or sd["l3.weight"].shape[1] != 128:
            raise _lib.Lafse3Error("dnn2_weights: expected the 18-128-128-7 DNN2 of nn3_1.pth")
        w = torch.cat([sd["l1.weight"].reshape(-1), sd["l1.bias"], sd["l2.weight"].reshape(-1),
                       sd["l2.bias"], sd["l3.weight"][6], sd["l3.bias"][6:7]]).contiguous()
        if w.numel() != self._L.lafse3_dnn2_weight_count():
            raise _lib.Lafse3Error("dnn2_weights: packed size mismatch")
        self._dnn2_cache = (key, w)
        return w

    def traversal_time(self, state, final_point, gate12, velo, w, net, want_iters=False):
        """quad_moving.solver (quad_moving.py:29-57) for B episodes in one kernel: (B,) traversal times
        [+ (B,) fixed-point updates].  gate12: (B, 12) or (B, 4, 3) corners; velo (B, 3); w the pitch rate;
        net the DNN2 module."""
        d, f64 = self.device, torch.float64
        st = _dev_tensor(state, (NX,), f64, d, "state")
        B = st.shape[0]
        fin = _dev_tensor(final_point, (3,), f64, d, "final_point")
        g = torch.as_tensor(gate12, dtype=f64, device=d).reshape(-1, 12).contiguous()
        ve = _dev_tensor(velo, (3,), f64, d, "velo")
        fin, g, ve = _same_batch(B, final_point=fin, gate12=g, velo=ve)
        W = self.dnn2_weights(net)
        t = torch.empty((B,), dtype=f64, device=d)
        it = torch.empty((B,), dtype=torch.int32, device=d) if want_iters else None
        check(self._L.lafse3_traversal_time(self._ctx, B, _ptr(st), _ptr(fin), _ptr(g), _ptr(ve), float(w), _ptr(W),
                                            _ptr(t), _ptr(it), self._stream()), "lafse3_traversal_time")
        return (t, it) if want_iters else t

    def reward(self, x, goal, gate12):
        """Score given trajectories (B, N+1, 13) as run_quad.objective does -> reward (B,)."""
        d, f64 = self.device, torch.float64
        xs = _dev_tensor(x, (self.horizon + 1, NX), f64, d, "x")
        B = xs.shape[0]
        goal = _dev_tensor(goal, (3,), f64, d, "goal")
        g12 = _dev_tensor(gate12, (12,), f64, d, "gate12")
        goal, g12 = _same_batch(B, goal=goal, gate12=g12)
        R = torch.empty((B,), dtype=f64, device=d)
        check(self._L.lafse3_reward(self._ctx, B, _ptr(xs), _ptr(goal), _ptr(g12), _ptr(R), self._stream()),
              "lafse3_reward")
        return R

    def get_input(self, ini_state, goal, dnn_out, u_last=None, want_x=False):
        """Batched run_quad.get_input: first control (B,4) [+ state trajectory (B,N+1,13)]."""
        d, f64 = self.device, torch.float64
        ini = _dev_tensor(ini_state, (NX,), f64, d, "ini_state")
        B = ini.shape[0]
        goal = _dev_tensor(goal, (3,), f64, d, "goal")
        dnn = _dev_tensor(dnn_out, (7,), torch.float32, d, "dnn_out")
        ul = _dev_tensor(u_last, (NU,), f64, d, "u_last", allow_none=True)
        goal, dnn, ul = _same_batch(B, goal=goal, dnn_out=dnn, u_last=ul)
        u0 = torch.empty((B, NU), dtype=f64, device=d)
        x = torch.empty((B, self.horizon + 1, NX), dtype=f64, device=d) if want_x else None
        st = torch.empty((B,), dtype=torch.int32, device=d)
        check(self._L.lafse3_get_input(self._ctx, B, _ptr(ini), _ptr(goal), _ptr(ul), _ptr(dnn), _ptr(u0), _ptr(x),
                                       _ptr(st), self._stream()), "lafse3_get_input")
        return (u0, x, st) if want_x else (u0, st)
