#!/usr/bin/env python3
"""Generate the committed golden vectors under tests/golden/ from the REFERENCE's own Python code.

Runs only in the build container (it needs /root/reference, which never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_golden.py

What is imported from /root/reference (read-only, no bytecode written):
  * solid_geometry.py            — imported unmodified (numpy only): plane / line / obstacle.collis_det
  * quad_model.py, quad_policy.py, quad_OC.py, quad_nn.py
                                 — need CasADi 3.5.5, which is absent from this image
                                   (``import casadi`` -> ModuleNotFoundError, an ordinary import error).
                                   For these we register, in sys.modules, a sympy-backed module named
                                   ``casadi`` that provides only casadi's *symbolic algebra* primitives the
                                   reference uses (SX.sym, vertcat, horzcat, vcat, diag, inv, mtimes,
                                   transpose, trace, dot) plus an inert ``Function``.  The reference's own
                                   Quadrotor.initDyn / initCost / init_TraCost then build the reference's
                                   expressions as sympy expressions, which we differentiate and evaluate.
                                   The NLP solve (``nlpsol('ipopt')``) is NOT emulated: wherever the reference
                                   calls ``OCSys.ocSolver`` we substitute the C oracle's solution for the exact
                                   parameters the reference passed (captured), so the reference's reward and
                                   finite-difference code runs around the oracle ("oracle in the loop").

Output files (small .npz, < 1 MB total):
  model.npz     f, A=d f_d/dx, B=d f_d/du, sum_i lam_i Hess(f_d,i) at 64 seeded points
  costs.npz     path/final/thrust/traversal cost values, gradient and Hessian of w*tra+path
  rd2quat.npz   Rd2Rp + toQuaternion on fp64 and fp32 angle vectors
  geometry.npz  obstacle.collis_det (+ co flag) and get_quadrotor_position on seeded tracks
  scenario.npz  nn_sample under np.random.seed + gate.rotate_y_out corners + run_quad.ini_state
  policy.npz    run_quad.objective and run_quad.sol_gradient with oracle-in-the-loop for 8 samples:
                per-call captured (p_tra, q_tra, t, Ulast), the 9 state trajectories the reference's
                reward code scored, its 9 rewards and its out8 (the NLP solutions themselves are the
                oracle's and are pinned only by the KKT certificate)
  last_inputs.npz  the scenario vector held by gym_pybullet_drone/last_inputs.npy (allow_pickle=False)
  dnn2_nn3_1.npz  the trained DNN2 of main.py:41-42 (nn3_1.pth): its six float32 parameter storages read raw
                from the checkpoint's zip archive (load_nn3_1; the checkpoint is not unpickled)
  moving.npz    main.py's moving-gate receding-horizon loop (gate.move/translate/rotate_y/transform/t_final,
                quad_moving.solver, run_quad.get_input) for 2 episodes x 120 plant steps (12 MPC solves each;
                episode 0 = last_inputs.npy's scenario): the reference's own gate / solver / run_quad code with
                the trained DNN2 (dnn2_nn3_1.npz), the C oracle substituted for ocSolver, and the plant dyn_fn
                (setDyn(0.01)) evaluated from the reference's own f expression (sympy)
  moving500.npz the same loop for episode 0 at main.py's full length: 500 plant steps, 50 MPC solves
                (main.py:65); ``make_golden.py moving500`` regenerates only this file
"""
from __future__ import annotations

import math
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

import numpy as np  # noqa: E402
import sympy as sp  # noqa: E402

sys.path.insert(0, REPO)
from oracle import oracle as O  # noqa: E402


# ---------------------------------------------------------------------------------------------
# sympy-backed stand-in for casadi's symbolic layer (only what quad_model/quad_OC/quad_policy use)
# ---------------------------------------------------------------------------------------------
class SXM:
    __array_ufunc__ = None  # make numpy defer (np.identity(3) - SXM -> SXM.__rsub__)

    def __init__(self, m):
        if isinstance(m, SXM):
            m = m.m
        if not isinstance(m, sp.MatrixBase):
            m = sp.Matrix([[sp.sympify(m)]])
        self.m = sp.Matrix(m)

    @staticmethod
    def _wrap(o):
        if isinstance(o, SXM):
            return o.m
        if isinstance(o, (list, tuple, np.ndarray)):
            a = np.asarray(o, dtype=object)
            if a.ndim == 1:
                return sp.Matrix([[sp.sympify(float(v) if isinstance(v, (np.floating, float)) else v)] for v in a])
            return sp.Matrix([[sp.sympify(float(v) if isinstance(v, (np.floating, float)) else v) for v in row] for row in a])
        if isinstance(o, (np.floating,)):
            return sp.Float(float(o))
        return sp.sympify(o)

    def _bin(self, o, f):
        a, b = self.m, self._wrap(o)
        if isinstance(b, sp.MatrixBase):
            if a.shape == (1, 1) and b.shape != (1, 1):
                return SXM(b.applyfunc(lambda e: f(a[0, 0], e)))
            if b.shape == (1, 1) and a.shape != (1, 1):
                return SXM(a.applyfunc(lambda e: f(e, b[0, 0])))
            return SXM(sp.Matrix(a.shape[0], a.shape[1], lambda i, j: f(a[i, j], b[i, j])))
        return SXM(a.applyfunc(lambda e: f(e, b)))

    def __add__(self, o): return self._bin(o, lambda x, y: x + y)
    def __radd__(self, o): return self._bin(o, lambda x, y: y + x)
    def __sub__(self, o): return self._bin(o, lambda x, y: x - y)
    def __rsub__(self, o): return self._bin(o, lambda x, y: y - x)
    def __mul__(self, o): return self._bin(o, lambda x, y: x * y)
    def __rmul__(self, o): return self._bin(o, lambda x, y: y * x)
    def __truediv__(self, o): return self._bin(o, lambda x, y: x / y)
    def __rtruediv__(self, o): return self._bin(o, lambda x, y: y / x)
    def __pow__(self, o): return self._bin(o, lambda x, y: x ** y)
    def __neg__(self): return SXM(-self.m)

    def __getitem__(self, i):
        if isinstance(i, tuple):
            return SXM(self.m[i])
        return SXM(self.m[i])

    def numel(self): return self.m.shape[0] * self.m.shape[1]

    def full(self): return np.array(self.m.evalf(), dtype=np.float64)

    @property
    def scalar(self):
        assert self.m.shape == (1, 1)
        return self.m[0, 0]


def _cat(args, axis):
    mats = [SXM._wrap(a) if not isinstance(a, SXM) else a.m for a in args]
    mats = [m if isinstance(m, sp.MatrixBase) else sp.Matrix([[m]]) for m in mats]
    return SXM(sp.Matrix.vstack(*mats) if axis == 0 else sp.Matrix.hstack(*mats))


class _SX:
    @staticmethod
    def sym(name, n=1):
        if n == 1:
            return SXM(sp.Symbol(name))
        return SXM(sp.Matrix([sp.Symbol(f"{name}_{i}") for i in range(n)]))


class _Function:
    def __init__(self, name, ins, outs):
        self.name, self.ins, self.outs = name, ins, outs


def _make_casadi():
    m = types.ModuleType("casadi")
    m.numpy = np
    m.SX = _SX
    m.MX = _SX
    m.vertcat = lambda *a: _cat(a, 0)
    m.horzcat = lambda *a: _cat(a, 1)
    m.vcat = lambda lst: _cat(lst, 0) if len(lst) else SXM(sp.zeros(0, 1))
    m.diag = lambda v: SXM(sp.diag(*list(SXM(v).m)))
    m.inv = lambda M: SXM(SXM(M).m.inv())
    m.mtimes = lambda A, B: SXM(SXM._wrap(A) * SXM._wrap(B))
    m.transpose = lambda A: SXM(SXM(A).m.T)
    m.trace = lambda A: SXM(SXM(A).m.trace())
    m.dot = lambda a, b: SXM((SXM._wrap(a).T * SXM._wrap(b))[0, 0])
    m.exp = lambda a: SXM(sp.exp(SXM._wrap(a))) if not isinstance(a, (float, int)) else np.exp(a)
    m.Function = _Function
    m.atan = math.atan            # numeric use only (quad_moving.solver, main.py)
    m.pi = math.pi
    m.jacobian = lambda e, x: SXM(SXM(e).m.jacobian(SXM(x).m))
    m.__all__ = ["numpy", "SX", "MX", "vertcat", "horzcat", "vcat", "diag", "inv", "mtimes", "transpose",
                 "trace", "dot", "exp", "Function", "jacobian", "atan", "pi"]
    return m


def import_reference():
    sys.modules["casadi"] = _make_casadi()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import solid_geometry as SG  # noqa: F401  (pure numpy, unmodified)
    import quad_model as QM
    import quad_policy as QP
    return SG, QM, QP


# ---------------------------------------------------------------------------------------------
def sym_vec(x: SXM):
    return list(x.m)


def gen_model(QM, rng, n=64):
    quad = QM.Quadrotor()
    quad.initDyn(Jx=0.0023, Jy=0.0023, Jz=0.004, mass=0.5, l=0.35, c=0.0245)  # quad_policy.py:37
    X, U = sym_vec(quad.X), sym_vec(quad.U)
    f = quad.f.m
    dt = 0.1
    fd = sp.Matrix(X) + dt * f
    A = fd.jacobian(X)
    Bm = fd.jacobian(U)
    lam = sp.symbols("lam0:13")
    L = sum(lam[i] * fd[i] for i in range(13))
    Hxx = sp.hessian(L, X)
    Hxu = sp.Matrix(13, 4, lambda i, j: sp.diff(L, X[i], U[j]))
    args = X + U + list(lam)
    fn = sp.lambdify(args, [f, A, Bm, Hxx, Hxu], "numpy")
    xs = np.zeros((n, 13)); us = np.zeros((n, 4)); ls = rng.normal(0, 1, size=(n, 13))
    xs[:, 0:3] = rng.uniform(-6, 6, (n, 3)); xs[:, 3:6] = rng.normal(0, 2, (n, 3))
    xs[:, 6:10] = rng.normal(0, 0.6, (n, 4)); xs[:, 10:13] = rng.uniform(-1.5, 1.5, (n, 3))
    us[:] = rng.uniform(0, 2.44, (n, 4))
    out = {k: [] for k in ("f", "A", "B", "Hxx", "Hxu")}
    for i in range(n):
        r = fn(*xs[i], *us[i], *ls[i])
        for k, v in zip(("f", "A", "B", "Hxx", "Hxu"), r):
            out[k].append(np.array(v, dtype=np.float64))
    out = {k: np.stack(v) for k, v in out.items()}
    out["f"] = out["f"].reshape(n, 13)
    np.savez_compressed(os.path.join(HERE, "model.npz"), x=xs, u=us, lam=ls, **out)
    print("model.npz", {k: v.shape for k, v in out.items()})


def gen_costs(QM, QP, rng, n=64):
    res = {k: [] for k in ("path", "final", "thrust", "tra", "grad", "hess", "qtra")}
    xs = np.zeros((n, 13)); us = rng.uniform(0, 2.44, (n, 4))
    xs[:, 0:3] = rng.uniform(-6, 6, (n, 3)); xs[:, 3:6] = rng.normal(0, 2, (n, 3))
    xs[:, 6:10] = rng.normal(0, 0.6, (n, 4)); xs[:, 10:13] = rng.uniform(-1.5, 1.5, (n, 3))
    goals = rng.uniform(-2, 2, (n, 3)) + np.array([0, 6, 0])
    ptra = rng.uniform(-0.5, 0.5, (n, 3))
    atra = rng.uniform(-0.8, 0.8, (n, 3))
    wks = 60 * np.exp(-10 * rng.uniform(-1, 1, n) ** 2)
    for i in range(n):
        quad = QM.Quadrotor()
        quad.initDyn(Jx=0.0023, Jy=0.0023, Jz=0.004, mass=0.5, l=0.35, c=0.0245)
        quad.initCost(wrt=5, wqt=80, wthrust=0.1, wrf=5, wvf=5, wqf=0, wwf=3, goal_pos=goals[i])  # quad_policy.py:38
        tra_atti = QP.Rd2Rp(atra[i])
        quad.init_TraCost(ptra[i], tra_atti)
        X, U = sym_vec(quad.X), sym_vec(quad.U)
        subs_x = dict(zip(X, xs[i])); subs_u = dict(zip(U, us[i]))
        path = float(quad.goal_cost.scalar.subs(subs_x))
        final = float(quad.final_cost.scalar.subs(subs_x))
        thrust = float(quad.thrust_cost.scalar.subs(subs_u))
        tra_e = quad.tra_cost.scalar
        tra = float(tra_e.subs(subs_x))
        stage = wks[i] * tra_e + quad.goal_cost.scalar
        g = [float(sp.diff(stage, v).subs(subs_x)) for v in X]
        H = sp.hessian(stage, X)
        Hn = np.array(H.subs(subs_x).evalf(), dtype=np.float64)
        for k, v in (("path", path), ("final", final), ("thrust", thrust), ("tra", tra), ("grad", g), ("hess", Hn),
                     ("qtra", np.array(quad.tra_q, dtype=np.float64))):
            res[k].append(v)
    res = {k: np.array(v) for k, v in res.items()}
    np.savez_compressed(os.path.join(HERE, "costs.npz"), x=xs, u=us, goal=goals, ptra=ptra, atra=atra, wk=wks, **res)
    print("costs.npz", {k: v.shape for k, v in res.items()})


def gen_rd2quat(QM, QP, rng, n=64):
    a64 = rng.uniform(-0.8, 0.8, (n, 3))
    a32 = rng.uniform(-0.8, 0.8, (n, 3)).astype(np.float32)
    q64, q32, th32 = [], [], []
    for i in range(n):
        th, vec = QP.Rd2Rp(a64[i])
        q64.append(QM.toQuaternion(th, vec))
        th, vec = QP.Rd2Rp(a32[i])
        q32.append(QM.toQuaternion(th, vec))
        th32.append(th)
    np.savez_compressed(os.path.join(HERE, "rd2quat.npz"), a64=a64, q64=np.array(q64), a32=a32, q32=np.array(q32),
                        theta32=np.array(th32))
    print("rd2quat.npz")


def _tracks_through_gate(rng, gate12, n_steps=51):
    """Straight-ish rotor tracks that cross the gate plane near the centre, the frame and far away."""
    g = gate12.reshape(4, 3)
    cen = g.mean(0)
    nrm = np.cross(g[1] - cen, g[0] - cen)  # plane1 normal direction (solid_geometry.py:23: cross(vec2, vec1))
    nrm /= np.linalg.norm(nrm)
    u1 = g[1] - g[0]; u1 /= np.linalg.norm(u1)
    u2 = np.cross(nrm, u1)
    mode = rng.integers(0, 4)
    if mode == 0:      # near centre
        off = rng.normal(0, 0.15, 2)
    elif mode == 1:    # near an edge / outside
        off = rng.normal(0, 0.8, 2)
    elif mode == 2:    # far outside
        off = rng.normal(0, 3.0, 2)
    else:              # starts behind the plane
        off = rng.normal(0, 0.3, 2)
    hit = cen + off[0] * u1 + off[1] * u2
    start = hit + nrm * rng.uniform(2, 9) + rng.normal(0, 0.5, 3)
    if mode == 3:
        start = hit - nrm * rng.uniform(0.5, 3)
    end = hit - nrm * rng.uniform(1, 6) + rng.normal(0, 0.5, 3)
    s = np.linspace(0, 1, n_steps)[:, None] ** rng.uniform(0.7, 1.4)
    tr = start + s * (end - start) + rng.normal(0, 0.02, (n_steps, 3))
    return tr


def gen_geometry(SG, QM, rng, n=256):
    gates, tracks, col, co = [], [], [], []
    for i in range(n):
        w = np.clip(rng.normal(0.9, 0.3), 0.5, 1.25)
        pitch = rng.uniform(-np.pi / 2, np.pi / 2)
        gp = np.array([[-w / 2, 0, 1], [w / 2, 0, 1], [w / 2, 0, -1], [-w / 2, 0, -1]])
        gt = QM.gate(gp)
        g12 = gt.rotate_y_out(pitch).reshape(12) + rng.normal(0, 0.5, 3).repeat(4).reshape(3, 4).T.reshape(12) * 0
        tr = _tracks_through_gate(rng, g12)
        ob = SG.obstacle(g12[0:3], g12[3:6], g12[6:9], g12[9:12])
        c = ob.collis_det(tr, 50)
        gates.append(g12); tracks.append(tr); col.append(c); co.append(ob.co)
    # rotor tips on random state trajectories (quad_model.py:239-276)
    quad = QM.Quadrotor()
    states = np.zeros((8, 51, 13))
    states[:, :, 0:3] = rng.uniform(-5, 5, (8, 51, 3))
    states[:, :, 6:10] = rng.normal(0, 0.6, (8, 51, 4))
    tips = np.stack([quad.get_quadrotor_position(wing_len=1.5, state_traj=states[i]) for i in range(8)])
    np.savez_compressed(os.path.join(HERE, "geometry.npz"), gate12=np.array(gates), tracks=np.array(tracks),
                        collision=np.array(col), co=np.array(co), states=states, tips=tips)
    print("geometry.npz", len(gates), "branches nonzero:", int(np.sum(np.array(col) != 0)), "co:", int(np.sum(co)))


def gen_scenario(QM, QP, n=16):
    import quad_nn as QN
    ins, gates, inis = [], [], []
    for s in range(n):
        np.random.seed(s)
        x = QN.nn_sample()
        gp = np.array([[-x[7] / 2, 0, 1], [x[7] / 2, 0, 1], [x[7] / 2, 0, -1], [-x[7] / 2, 0, -1]])  # deep_learning.py:25
        g12 = QM.gate(gp).rotate_y_out(x[8]).reshape(12)
        ini = np.array(x[0:3].tolist() + [0.0, 0.0, 0.0] + QM.toQuaternion(x[6], [0, 0, 1]) + [0.0, 0.0, 0.0])
        ins.append(x); gates.append(g12); inis.append(ini)
    np.savez_compressed(os.path.join(HERE, "scenario.npz"), inputs=np.array(ins), gate12=np.array(gates), ini=np.array(inis))
    print("scenario.npz")


def gen_policy(QM, QP, n=8, seed=7):
    """run_quad.objective / sol_gradient with the C oracle substituted for ocSolver (captured params)."""
    import quad_nn as QN
    params = O.default_params(t_probe_f32=1)  # this container runs NumPy >= 2 (NEP 50), see SURVEY A10
    rng = np.random.default_rng(seed)
    rec = {k: [] for k in ("ini", "goal", "gate12", "dnn", "out8", "calls_p", "calls_q", "calls_t", "calls_ulast",
                           "rewards", "x_calls", "x_opt", "u_opt", "lam_opt", "cost_opt", "status")}
    for s in range(n):
        np.random.seed(100 + s)
        x = QN.nn_sample()
        gp = np.array([[-x[7] / 2, 0, 1], [x[7] / 2, 0, 1], [x[7] / 2, 0, -1], [-x[7] / 2, 0, -1]])
        g12 = QM.gate(gp).rotate_y_out(x[8]).reshape(12)
        quad = QP.run_quad(goal_pos=x[3:6], ini_r=x[0:3].tolist(), ini_q=QM.toQuaternion(x[6], [0, 0, 1]))
        quad.init_obstacle(g12)
        out = np.zeros(7, dtype=np.float32)
        out[0:3] = rng.uniform(-0.3, 0.3, 3)
        out[3:6] = rng.uniform(-0.5, 0.5, 3)
        out[6] = np.float32(rng.uniform(1.9, 4.1))
        calls = []

        def fake_ocsolver(ini_state, Ulast=None, horizon=None, auxvar_value=1, print_level=0, dt=0.1,
                          costate_option=0, _q=quad, _calls=calls):
            p = np.array(_q.uav1.tra_r_I, dtype=np.float64).reshape(3)
            qt = np.array(_q.uav1.tra_q, dtype=np.float64).reshape(4)
            t = float(_q.uavoc1.t)
            ul = np.zeros(4) if Ulast is None else np.array(Ulast, dtype=np.float64)
            r = O.solve(np.array(ini_state, dtype=np.float64), np.array(_q.goal_pos, dtype=np.float64), p, qt, t, ul,
                        params=params)
            _calls.append((p, qt, t, ul, r))
            return {"state_traj_opt": r["x"][0], "control_traj_opt": r["u"][0], "costate_traj_opt": r["lam"][0],
                    "cost": r["cost"][0].reshape(1, 1)}

        quad.uavoc1.ocSolver = fake_ocsolver
        rewards = []
        orig_obj = quad.objective

        def obj_wrap(*a, **k):
            v = orig_obj(*a, **k)
            rewards.append(float(v))
            return v

        quad.objective = obj_wrap
        g = quad.sol_gradient(quad.ini_state, out[0:3], out[3:6], out[6])
        assert len(calls) == 9
        rec["ini"].append(np.array(quad.ini_state, dtype=np.float64)); rec["goal"].append(np.array(x[3:6]))
        rec["gate12"].append(g12); rec["dnn"].append(out); rec["out8"].append(np.array(g, dtype=np.float64))
        rec["calls_p"].append(np.stack([c[0] for c in calls])); rec["calls_q"].append(np.stack([c[1] for c in calls]))
        rec["calls_t"].append(np.array([c[2] for c in calls])); rec["calls_ulast"].append(np.stack([c[3] for c in calls]))
        rec["rewards"].append(np.array(rewards))
        rec["x_calls"].append(np.stack([c[4]["x"][0] for c in calls]))
        r0 = calls[0][4]
        rec["x_opt"].append(r0["x"][0]); rec["u_opt"].append(r0["u"][0]); rec["lam_opt"].append(r0["lam"][0])
        rec["cost_opt"].append(r0["cost"][0]); rec["status"].append(np.array([c[4]["status"][0] for c in calls]))
    rec = {k: np.array(v) for k, v in rec.items()}
    np.savez_compressed(os.path.join(HERE, "policy.npz"), **rec)
    print("policy.npz", rec["out8"].shape, "status", np.unique(rec["status"]))


def gen_last_inputs():
    path = os.path.join(REF, "gym_pybullet_drone", "last_inputs.npy")
    with open(path, "rb") as fh:
        recs = []
        while True:
            try:
                recs.append(np.load(fh, allow_pickle=False))
            except Exception:
                break
    vec = [r for r in recs if r.size == 9]
    np.savez_compressed(os.path.join(HERE, "last_inputs.npz"), inputs=np.array(vec[0], dtype=np.float64),
                        n_records=len(recs))
    print("last_inputs.npz", vec[0])


NN3_1 = os.path.join(REF, "gym_pybullet_drone", "nn3_1.pth")
# archive/data/<key> of nn3_1.pth: the six parameter storages in the order its data.pkl names them (l1 weight
# '0', bias '1'; l2 '2', '3'; l3 '4', '5'), each a contiguous little-endian float32 buffer
NN3_1_LAYOUT = (("l1.weight", (128, 18)), ("l1.bias", (128,)), ("l2.weight", (128, 128)), ("l2.bias", (128,)),
                ("l3.weight", (7, 128)), ("l3.bias", (7,)))


def load_nn3_1():
    """DNN2's trained weights (main.py:41-42 torch.load("nn3_1.pth")) read as raw float32 from the checkpoint's
    zip archive; the pickled module description (data.pkl) is not unpickled -- only its storage keys were read
    as text to fix NN3_1_LAYOUT, and every storage's byte size is checked against it here."""
    import zipfile
    z = zipfile.ZipFile(NN3_1)
    names = {n.split("/")[-1]: n for n in z.namelist() if "/data/" in n}
    out = {}
    for key, (name, shape) in enumerate(NN3_1_LAYOUT):
        raw = z.read(names[str(key)])
        assert len(raw) == 4 * int(np.prod(shape)), (name, len(raw))
        out[name] = np.frombuffer(raw, dtype="<f4").reshape(shape).copy()
    return out


def gen_dnn2():
    w = load_nn3_1()
    np.savez_compressed(os.path.join(HERE, "dnn2_nn3_1.npz"), **{k.replace(".", "_"): v for k, v in w.items()})
    print("dnn2_nn3_1.npz", {k: v.shape for k, v in w.items()})
    return w


def gen_moving(QM, QP, n_ep=2, steps=120, name="moving.npz"):
    """main.py:18-116 restated around the reference's own functions (see the module docstring), driven by the
    trained DNN2 (nn3_1.pth, load_nn3_1).  Episode 0 is last_inputs.npy's scenario (the 9-vector the reference
    ships), episode s >= 1 is nn_sample() under np.random.seed(500 + s); every episode draws its gate.move noise
    after np.random.seed(500 + s) and one nn_sample() call (discarded for episode 0), so the draw order is the
    same for both kinds."""
    import torch
    import quad_moving as QMV
    import quad_nn as QN
    model = QN.network(18, 128, 128, 7)            # nn3_1.pth architecture (nn_train_2.py:11-23)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in load_nn3_1().items()})
    weights = {k.replace(".", "_"): v.detach().numpy().copy() for k, v in model.state_dict().items()}
    last = np.load(os.path.join(HERE, "last_inputs.npz"))["inputs"]   # gen_last_inputs: the npy's 9-vector
    quad = QM.Quadrotor()
    quad.initDyn(Jx=0.0023, Jy=0.0023, Jz=0.004, mass=0.5, l=0.35, c=0.0245)
    X, U = sym_vec(quad.X), sym_vec(quad.U)
    f_np = sp.lambdify(X + U, list(quad.f.m), "numpy")

    def dyn_fn(x, u):                               # quad1.uav1.setDyn(0.01); dyn_fn (quad_model.py:215-219)
        return np.asarray(x, dtype=np.float64) + 0.01 * np.array(f_np(*x, *u), dtype=np.float64)

    v, w = np.array([1, 0.3, 0.4]), math.pi / 2     # main.py:45-46
    rec = {k: [] for k in ("inputs", "gate_move", "V", "t", "states", "controls", "ins18", "outs", "source")}
    for s in range(n_ep):
        np.random.seed(500 + s)
        inputs = QN.nn_sample()
        if s == 0:
            inputs = np.array(last, dtype=np.float64)
        rec["source"].append(0 if s == 0 else 1)   # 0: last_inputs.npy, 1: nn_sample
        final_point = inputs[3:6]
        gp0 = np.array([[-inputs[7] / 2, 0, 1], [inputs[7] / 2, 0, 1], [inputs[7] / 2, 0, -1], [-inputs[7] / 2, 0, -1]])
        gate1 = QM.gate(gp0)
        gate1.rotate_y(inputs[8])
        gate1 = QM.gate(gate1.gate_point)
        quad1 = QP.run_quad(goal_pos=inputs[3:6], ini_r=inputs[0:3].tolist(), ini_q=QM.toQuaternion(inputs[6], [0, 0, 1]))
        state = np.array(quad1.ini_state)
        gate_move, V = gate1.move(v=v, w=w)
        u = [0, 0, 0, 0]
        ts, states, controls, ins18, outs = [], [state], [], [], []
        for i in range(steps):
            gate_n = QM.gate(gate_move[i])
            t = QMV.solver(model, state, final_point, gate_n, V[i], w)
            ts.append(t)
            if i % 10 == 0:
                gate_n.translate(t * V[i])
                gate_n.rotate_y(t * w)
                inp = np.zeros(18)
                inp[16] = QMV.magni(gate_n.gate_point[0, :] - gate_n.gate_point[1, :])   # solid_geometry.magni
                inp[17] = math.atan((gate_n.gate_point[0, 2] - gate_n.gate_point[1, 2]) /
                                    (gate_n.gate_point[0, 0] - gate_n.gate_point[1, 0]))
                inp[0:13] = gate_n.transform(state)
                inp[13:16] = gate_n.t_final(final_point)
                out = model(inp).data.numpy()
                quad2 = QP.run_quad(goal_pos=inp[13:16], horizon=50)

                def fake_ocsolver(ini_state, Ulast=None, horizon=None, auxvar_value=1, print_level=0, dt=0.1,
                                  costate_option=0, _q=quad2):
                    p = np.array(_q.uav1.tra_r_I, dtype=np.float64).reshape(3)
                    qt = np.array(_q.uav1.tra_q, dtype=np.float64).reshape(4)
                    ul = np.zeros(4) if Ulast is None else np.array(Ulast, dtype=np.float64)
                    r = O.solve(np.array(ini_state, dtype=np.float64), np.array(_q.goal_pos, dtype=np.float64), p, qt,
                                float(_q.uavoc1.t), ul)
                    return {"state_traj_opt": r["x"][0], "control_traj_opt": r["u"][0], "costate_traj_opt": r["lam"][0],
                            "cost": r["cost"][0].reshape(1, 1)}

                quad2.uavoc1.ocSolver = fake_ocsolver
                u = quad2.get_input(inp[0:13], u, out[0:3], out[3:6], out[6])
                ins18.append(inp)
                outs.append(out)
            state = dyn_fn(state, u).reshape(13)
            states.append(state)
            controls.append(np.array(u, dtype=np.float64))
        rec["inputs"].append(inputs); rec["gate_move"].append(gate_move); rec["V"].append(V)
        rec["t"].append(np.array(ts)); rec["states"].append(np.stack(states)); rec["controls"].append(np.stack(controls))
        rec["ins18"].append(np.stack(ins18)); rec["outs"].append(np.stack(outs))
    rec = {k: np.array(v) for k, v in rec.items()}
    np.savez_compressed(os.path.join(HERE, name), **rec, **weights)
    print(name, {k: v.shape for k, v in rec.items()})


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    SG, QM, QP = import_reference()
    rng = np.random.default_rng(20250124)
    gen_model(QM, rng)
    gen_costs(QM, QP, rng)
    gen_rd2quat(QM, QP, rng)
    gen_geometry(SG, QM, rng)
    gen_scenario(QM, QP)
    gen_last_inputs()
    gen_policy(QM, QP)
    gen_dnn2()
    gen_moving(QM, QP)
    gen_moving(QM, QP, n_ep=1, steps=500, name="moving500.npz")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "moving":
        os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
        _, _QM, _QP = import_reference()
        gen_dnn2()
        gen_moving(_QM, _QP)
    elif len(sys.argv) > 1 and sys.argv[1] == "moving500":
        # configs[4] at main.py's full length (main.py:65: 500 plant steps, 50 MPC solves), episode 0 only
        os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
        _, _QM, _QP = import_reference()
        gen_moving(_QM, _QP, n_ep=1, steps=500, name="moving500.npz")
    else:
        main()
