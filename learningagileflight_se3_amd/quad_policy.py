"""Drop-in mirror of the reference's optimal-control interface, backed by the MI355X engine.

Same class / method names, argument meaning and return shapes as the reference, so a caller of
yanrui89/LearningAgileFlight_SE3 switches by changing an import:

  ``OCSys.ocSolver``        quad_OC.py:104-212  -> dict(state_traj_opt, control_traj_opt,
                            costate_traj_opt, auxvar_value, time, horizon, cost)
  ``run_quad.objective``    quad_policy.py:67-91  -> float reward
  ``run_quad.sol_gradient`` quad_policy.py:94-112 -> ndarray(8)
  ``run_quad.get_input``    quad_policy.py:202-211 -> ndarray(4)

plus batched twins (``*_batch``) that take (B, ...) arrays and return device tensors — the form the
batched training loop uses.  Every call runs the HIP kernels through the C ABI (liblafse3.so); there
is no CPU solver behind this module (missing library -> ``_lib.Lafse3Error``).

Differences from the reference, by design:
  * the NLP is fixed to the quadrotor problem run_quad configures (quad_policy.py:35-56); OCSys is not
    a general CasADi front end, its cost is set with ``setTraCost(tra_pos, tra_ang, t)`` (the
    arguments of init_TraCost + setTraCost, quad_policy.py:74-75) instead of a CasADi expression;
  * ``costate_option=1`` recomputes the costates by the reference's PMP recursion (quad_OC.py:188-201)
    on the GPU (lafse3_params.costate_option), path-cost gradient only, as the reference does.
"""
from __future__ import annotations

import numpy as np
import torch

from . import scenario
from .engine import Engine


def _as_np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


class OCSys:
    """OCSys restricted to the run_quad problem (quad_OC.py:18-212, configured as quad_policy.py:35-56)."""

    def __init__(self, project_name="quadrotor", goal_pos=(0, 8, 0), horizon=50, engine: Engine | None = None,
                 device=None):
        self.project_name = project_name
        self.goal_pos = np.asarray(goal_pos, dtype=np.float64)
        self.horizon = horizon
        self.engine = engine if engine is not None else Engine(device=device, horizon=horizon)
        self.tra_pos = np.zeros(3)
        self.tra_ang = np.zeros(3)
        self.t = 1.0

    def setTraCost(self, tra_pos, tra_ang, t=3):
        """init_TraCost(tra_pos, Rd2Rp(tra_ang)) + setTraCost(tra_cost, t)  quad_model.py:200-213, quad_OC.py:98-101."""
        self.tra_pos = np.asarray(tra_pos, dtype=np.float64)
        self.tra_ang = np.asarray(tra_ang, dtype=np.float64)
        self.t = float(t)

    def ocSolver(self, ini_state, Ulast=None, horizon=None, auxvar_value=1, print_level=0, dt=0.1, costate_option=0):
        """quad_OC.py:104-212.  Returns the reference's dict keys and shapes (numpy, float64)."""
        if horizon is not None and horizon != self.horizon:
            raise ValueError(f"OCSys was built for horizon {self.horizon}")
        if costate_option not in (0, 1):
            raise ValueError("costate_option is 0 (IPOPT lam_g) or 1 (PMP recursion)")
        if abs(dt - self.engine.params.dt) > 1e-12:
            raise ValueError("dt is fixed by the engine parameters")
        out = self.engine.ocp_solve(np.asarray(ini_state, dtype=np.float64)[None], self.goal_pos[None],
                                    self.tra_pos[None], self.tra_ang[None], np.array([self.t]),
                                    None if Ulast is None else np.asarray(Ulast, dtype=np.float64)[None],
                                    costate_option=costate_option)
        N = self.horizon
        return {
            "state_traj_opt": _as_np(out["x"])[0],
            "control_traj_opt": _as_np(out["u"])[0],
            "costate_traj_opt": _as_np(out["lam"])[0],
            "auxvar_value": auxvar_value,
            "time": np.array([k for k in range(N + 1)]),
            "horizon": N,
            "cost": _as_np(out["cost"]).reshape(1, 1),
            "status": int(_as_np(out["status"])[0]),
            "iters": int(_as_np(out["iters"])[0]),
        }


class run_quad:
    """quad_policy.py:15-211 (run_quad) on the MI355X engine."""

    def __init__(self, goal_pos=[0, 8, 0], goal_atti=[0, [1, 0, 0]], ini_r=[0, -8, 0], ini_v_I=[0.0, 0.0, 0.0],
                 ini_q=None, horizon=50, engine: Engine | None = None, device=None):
        self.winglen = 1.5
        self.goal_pos = list(goal_pos)
        self.goal_atti = goal_atti
        if not isinstance(ini_r, list):
            ini_r = list(np.asarray(ini_r).tolist())
        if ini_q is None:
            ini_q = scenario.to_quaternion(0.0, [3, 3, 5]).tolist()
        self.ini_r = ini_r
        self.ini_v_I = list(ini_v_I)
        self.ini_q = list(ini_q)
        self.ini_w = [0.0, 0.0, 0.0]
        self.ini_state = self.ini_r + self.ini_v_I + self.ini_q + self.ini_w
        self.horizon = horizon
        self.dt = 0.1
        self.engine = engine if engine is not None else Engine(device=device, horizon=horizon)
        self.gate12 = None

    # quad_policy.py:60-65
    def init_obstacle(self, gate_point):
        g = np.asarray(gate_point, dtype=np.float64).reshape(12)
        self.point1, self.point2, self.point3, self.point4 = g[0:3], g[3:6], g[6:9], g[9:12]
        self.gate12 = g

    def _gate(self):
        if self.gate12 is None:
            raise RuntimeError("init_obstacle(gate_point) must be called first (quad_policy.py:60)")
        return self.gate12

    def _ini(self, ini_state):
        return np.asarray(self.ini_state if ini_state is None else ini_state, dtype=np.float64)

    # quad_policy.py:67-91
    def objective(self, ini_state=None, tra_pos=None, tra_ang=None, t=3, Ulast=None):
        R, st = self.engine.objective(self._ini(ini_state)[None], np.asarray(self.goal_pos, np.float64)[None],
                                      self._gate()[None], np.asarray(tra_pos, np.float64)[None],
                                      np.asarray(tra_ang, np.float64)[None], np.array([float(t)]),
                                      None if Ulast is None else np.asarray(Ulast, np.float64)[None])
        return float(_as_np(R)[0])

    # quad_policy.py:94-112
    def sol_gradient(self, ini_state=None, tra_pos=None, tra_ang=None, t=None, Ulast=None):
        tra_pos = np.asarray(tra_pos)
        tra_ang = np.asarray(tra_ang)
        ini = self._ini(ini_state)
        goal = np.asarray(self.goal_pos, np.float64)
        if tra_pos.dtype == np.float32 and tra_ang.dtype == np.float32 and np.asarray(t).dtype == np.float32:
            # DNN outputs (deep_learning.py:55-56): the fused 9-solve kernel reproduces the float32 quirks
            dnn = np.concatenate([tra_pos, tra_ang, np.asarray(t, np.float32).reshape(1)]).astype(np.float32)
            out8 = self.engine.sol_gradient(ini[None], goal[None], self._gate()[None], dnn[None],
                                            None if Ulast is None else np.asarray(Ulast, np.float64)[None])
            return _as_np(out8)[0]
        # float64 inputs: the same 9 objective evaluations, batched into one launch
        return self._sol_gradient_f64(ini, goal, tra_pos.astype(np.float64), tra_ang.astype(np.float64),
                                      float(t), Ulast)

    def _sol_gradient_f64(self, ini, goal, p, a, t, Ulast):
        delta = 1e-3
        P = np.repeat(p[None], 9, 0)
        A = np.repeat(a[None], 9, 0)
        T = np.full(9, t)
        for e in range(3):
            P[1 + e, e] += delta
            A[4 + e, e] += delta
        T[7], T[8] = t - 0.1, t + 0.1
        UL = np.zeros((9, 4))
        if Ulast is not None:
            UL[1:7] = np.asarray(Ulast, np.float64)
        R, _ = self.engine.objective(np.repeat(ini[None], 9, 0), np.repeat(goal[None], 9, 0),
                                     np.repeat(self._gate()[None], 9, 0), P, A, T, UL)
        R = _as_np(R)
        j = R[0]
        d = np.zeros(8)
        for e in range(3):
            d[e] = np.clip(R[1 + e] - j, -0.5, 0.5) * 0.1
            d[3 + e] = np.clip(R[4 + e] - j, -0.5, 0.5) * (1 / (500 * a[e] ** 2 + 5))
        drdt = 0
        if R[7] - j > 2:
            drdt = -0.05
        if R[8] - j > 2:
            drdt = 0.05
        return np.array([-d[0], -d[1], -d[2], -d[3], -d[4], -d[5], -drdt, j])

    # quad_policy.py:202-211
    def get_input(self, ini_state, Ulast, tra_pos, tra_ang, t):
        tra_pos = np.asarray(tra_pos)
        tra_ang = np.asarray(tra_ang)
        goal = np.asarray(self.goal_pos, np.float64)
        ul = None if Ulast is None else np.asarray(Ulast, np.float64)[None]
        if tra_pos.dtype == np.float32 and tra_ang.dtype == np.float32:
            dnn = np.concatenate([tra_pos, tra_ang, np.asarray(t, np.float32).reshape(1)]).astype(np.float32)
            u0, st = self.engine.get_input(self._ini(ini_state)[None], goal[None], dnn[None], ul)
            return _as_np(u0)[0]
        out = self.engine.ocp_solve(self._ini(ini_state)[None], goal[None], tra_pos.astype(np.float64)[None],
                                    tra_ang.astype(np.float64)[None], np.array([float(t)]), ul, want=("u",))
        self.sol1 = {"control_traj_opt": _as_np(out["u"])[0]}
        return self.sol1["control_traj_opt"][0, :]

    # ---- batched twins (device tensors in/out) -------------------------------------------------------
    def sol_gradient_batch(self, ini_state, goal, gate12, dnn_out, Ulast=None):
        return self.engine.sol_gradient(ini_state, goal, gate12, dnn_out, Ulast)

    def get_input_batch(self, ini_state, goal, dnn_out, Ulast=None):
        return self.engine.get_input(ini_state, goal, dnn_out, Ulast)[0]
