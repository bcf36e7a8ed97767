"""Moving-gate receding-horizon flight, batched over episodes: SURVEY.md §8(f) row 1, BASELINE configs[4].

main.py:18-116 for B independent episodes at once:
  gate kinematics   quad_model.py:670-815   gate.__init__ / rotate_y / translate / translate_out / move /
                                            transform / t_final, vectorised over the batch (numpy; the
                                            attitude transform uses scipy's Rotation, as the reference does)
  traversal time    quad_moving.py:29-57    solver(): fixed-point iteration t1 += (t2 - t1)/2 on DNN2's time
                                            output until |t2 - t1| <= 0.001, every plant step, per episode
  control (10 Hz)   main.py:76-107          gate advanced by the traversal time, DNN2 on the gate-frame state,
                                            run_quad(goal=gate-frame final point).get_input(..., Ulast=u)
                                            -> ONE lafse3_get_input launch for all B episodes (GPU)
  plant (100 Hz)    main.py:35, 108         Quadrotor.dyn_fn after setDyn(0.01) (quad_model.py:215-219):
                                            explicit Euler of the quadrotor f (quad_model.py:35-119) at dt 0.01

The gate frame I_G used by transform/t_final is the one rotate_y/translate leave behind (rows [ax, ay, az],
quad_model.py:700, 729): every path of main.py and quad_moving.solver rotates the gate before transforming.
DNN2 is any callable mapping (B, 18) float64 inputs to (B, 7) float32 outputs (the reference evaluates
``network.forward`` in float32, quad_nn.py:131-139); ``torch_dnn`` wraps an nn.Module.
"""
from __future__ import annotations

import math

import numpy as np
import torch
from scipy.spatial.transform import Rotation

from . import scenario

DT_PLANT = 0.01      # quad1.uav1.setDyn(0.01), main.py:35
CTRL_EVERY = 10      # main.py:76
T_TOL = 0.001        # quad_moving.py:45


# ---- gate kinematics (quad_model.py:670-815) -----------------------------------------------------------
def centroid(gp):
    """np.mean over the 4 corners per axis (quad_model.py:676): (B, 4, 3) -> (B, 3)."""
    return ((gp[:, 0] + gp[:, 1]) + gp[:, 2] + gp[:, 3]) / 4.0


def gate_frame(gp):
    """I_G = [ax; ay; az] (rows) with ay = norm((p1 - p0) x (p2 - p1)), az = e_z, ax = ay x az
    (quad_model.py:696-700, after rotate_y / translate)."""
    ay = np.cross(gp[:, 1] - gp[:, 0], gp[:, 2] - gp[:, 1])
    ay = ay / np.sqrt(np.einsum("bi,bi->b", ay, ay))[:, None]
    az = np.broadcast_to(np.array([0.0, 0.0, 1.0]), ay.shape)
    ax = np.cross(ay, az)
    return np.stack([ax, ay, az], axis=1)


def rotate_y(gp, angle):
    """Rotation about the gate's y axis through its centroid, in the x-z plane (quad_model.py:686-692)."""
    c = centroid(gp)
    rel = gp - c[:, None, :]
    ca, sa = np.cos(angle)[:, None], np.sin(angle)[:, None]
    out = rel.copy()
    out[:, :, 0] = ca * rel[:, :, 0] + (-sa) * rel[:, :, 2]
    out[:, :, 2] = sa * rel[:, :, 0] + ca * rel[:, :, 2]
    return out + c[:, None, :]


def translate(gp, d):
    """gate.translate / translate_out (quad_model.py:720-733)."""
    return gp + d[:, None, :]


def move(gp0, v, w, noise, dt=0.01):
    """gate.move(T, dt, v, w) (quad_model.py:769-790) with its per-step velocity noise given:
    noise (B, S, 3) = clip(normal(0, 0.1, 3), -0.1, 0.1) per step.  Returns (B, S+1, 4, 3), (B, S+1, 3)."""
    B, S = noise.shape[0], noise.shape[1]
    v = np.broadcast_to(np.asarray(v, dtype=np.float64), (B, 3))
    c, s = math.cos(dt * w), math.sin(dt * w)
    out = np.zeros((B, S + 1, 4, 3))
    V = np.zeros((B, S + 1, 3))
    gp = np.array(gp0, dtype=np.float64)
    out[:, 0], V[:, 0] = gp, v
    for i in range(S):
        cen = centroid(gp)
        rel = gp - cen[:, None, :]
        x0, z0 = rel[:, :, 0].copy(), rel[:, :, 2].copy()
        rel[:, :, 0] = c * x0 + (-s) * z0
        rel[:, :, 2] = s * x0 + c * z0
        vel = v + noise[:, i]
        gp = rel + cen[:, None, :] + dt * vel[:, None, :]
        out[:, i + 1], V[:, i + 1] = gp, vel
    return out, V


def move_noise(seed_or_rs, steps=500):
    """The reference's noise draws of gate.move for one episode from a legacy RandomState (main.py draws
    them after nn_sample from the global numpy stream)."""
    rs = seed_or_rs if isinstance(seed_or_rs, np.random.RandomState) else np.random.RandomState(seed_or_rs)
    return np.stack([np.clip(rs.normal(0, 0.1, 3), -0.1, 0.1) for _ in range(steps)])


def transform(IG, cen, state):
    """World-frame state -> gate frame (quad_model.py:793-811)."""
    out = np.zeros_like(state)
    out[:, 0:3] = np.einsum("bij,bj->bi", IG, state[:, 0:3] - cen)
    out[:, 3:6] = np.einsum("bij,bj->bi", IG, state[:, 3:6])
    out[:, 10:13] = state[:, 10:13]
    quat = np.concatenate([state[:, 7:10], state[:, 6:7]], axis=1)          # scipy order x, y, z, w
    r2 = Rotation.from_matrix(np.matmul(IG, Rotation.from_quat(quat).as_matrix()))
    qo = r2.as_quat()
    out[:, 6] = qo[:, 3]
    out[:, 7:10] = qo[:, 0:3]
    return out


def t_final(IG, cen, final_point):
    """quad_model.py:814-815."""
    return np.einsum("bij,bj->bi", IG, final_point - cen)


def dnn2_inputs(gp, state, final_point):
    """The 18 DNN2 inputs of main.py:90-94 / quad_moving.py:38-42 for gates gp (already advanced)."""
    IG, cen = gate_frame(gp), centroid(gp)
    inp = np.zeros((gp.shape[0], 18))
    d01 = gp[:, 0] - gp[:, 1]
    inp[:, 16] = np.sqrt(np.einsum("bi,bi->b", d01, d01))
    inp[:, 17] = np.arctan(d01[:, 2] / d01[:, 0])
    inp[:, 0:13] = transform(IG, cen, state)
    inp[:, 13:16] = t_final(IG, cen, final_point)
    return inp


def torch_dnn(net, device=None):
    """DNN2 callable from an nn.Module: float64 (B, 18) -> float32 (B, 7) numpy (batched forward)."""
    dev = device if device is not None else next(net.parameters()).device

    def f(inputs):
        with torch.no_grad():
            return net(torch.as_tensor(inputs, dtype=torch.float32, device=dev)).cpu().numpy()

    return f


def solve_t(dnn2, state, final_point, gp, velo, w, max_iter=200):
    """quad_moving.solver for B episodes: t1 = |centroid - r| / 3, then t1 += (t2 - t1)/2 until
    |t2 - t1| <= 0.001, t2 = DNN2(gate advanced by velo t1, w t1)[6].  Returns (t (B,), iterations (B,))."""
    cen = centroid(gp)
    d = cen - state[:, 0:3]
    t1 = np.sqrt(np.einsum("bi,bi->b", d, d)) / 3
    it = np.zeros(len(t1), dtype=np.int64)
    active = np.ones(len(t1), dtype=bool)

    def t_of(t):
        gx = rotate_y(translate(gp, velo * t[:, None]), w * t)
        return dnn2(dnn2_inputs(gx, state, final_point))[:, 6].astype(np.float64)

    t2 = t_of(t1)
    for _ in range(max_iter):
        active &= np.abs(t2 - t1) > T_TOL
        if not active.any():
            break
        t1 = np.where(active, t1 + (t2 - t1) / 2, t1)
        it += active
        t2 = np.where(active, t_of(t1), t2)
    return t1, it


def plant_step(state, u, params=None, dt=DT_PLANT):
    """x + dt f(x, u) with the quadrotor f of quad_model.py:79-119 (constants quad_policy.py:37, g 9.78)."""
    m, Jx, Jy, Jz, l, c, g = 0.5, 0.0023, 0.0023, 0.004, 0.35, 0.0245, 9.78
    if params is not None:
        m, Jx, Jy, Jz, l, c, g = (params.mass, params.Jx, params.Jy, params.Jz, params.arm_l, params.c_tau,
                                  params.grav)
    x = np.asarray(state, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    v, q, w = x[:, 3:6], x[:, 6:10], x[:, 10:13]
    T = u.sum(1)
    hl = l / 2
    f = np.zeros_like(x)
    f[:, 0:3] = v
    f[:, 3] = T / m * (2 * (q[:, 1] * q[:, 3] + q[:, 0] * q[:, 2]))
    f[:, 4] = T / m * (2 * (q[:, 2] * q[:, 3] - q[:, 0] * q[:, 1]))
    f[:, 5] = T / m * (1 - 2 * (q[:, 1] ** 2 + q[:, 2] ** 2)) - g
    f[:, 6] = 0.5 * (-w[:, 0] * q[:, 1] - w[:, 1] * q[:, 2] - w[:, 2] * q[:, 3])
    f[:, 7] = 0.5 * (w[:, 0] * q[:, 0] + w[:, 2] * q[:, 2] - w[:, 1] * q[:, 3])
    f[:, 8] = 0.5 * (w[:, 1] * q[:, 0] - w[:, 2] * q[:, 1] + w[:, 0] * q[:, 3])
    f[:, 9] = 0.5 * (w[:, 2] * q[:, 0] + w[:, 1] * q[:, 1] - w[:, 0] * q[:, 2])
    Mx = hl * (u[:, 3] - u[:, 1])
    My = hl * (u[:, 2] - u[:, 0])
    Mz = c * (u[:, 0] - u[:, 1] + u[:, 2] - u[:, 3])
    f[:, 10] = (Mx - (Jz - Jy) * w[:, 1] * w[:, 2]) / Jx
    f[:, 11] = (My - (Jx - Jz) * w[:, 0] * w[:, 2]) / Jy
    f[:, 12] = (Mz - (Jy - Jx) * w[:, 0] * w[:, 1]) / Jz
    return x + dt * f


def initial_episodes(samples):
    """main.py:18-37: gate corners (width, pitch) and the quadrotor's initial state for (B, 9) samples."""
    samples = np.asarray(samples, dtype=np.float64).reshape(-1, 9)
    gp = scenario.gate_corners(samples[:, 7], samples[:, 8]).reshape(-1, 4, 3)
    return gp, scenario.initial_state(samples[:, 0:3], samples[:, 6])


def run_episodes(engine, dnn2, samples, noise, v=(1.0, 0.3, 0.4), w=math.pi / 2, steps=500):
    """main.py:44-116 for B episodes.  Returns dict of (B, steps+1, 13) states, (B, steps, 4) controls,
    (B, steps) traversal times, (B, steps//10, 18) DNN2 inputs and (B, steps//10, 7) outputs at the control
    steps, (B, steps//10) solver statuses, and the number of MPC solves."""
    gp0, state = initial_episodes(samples)
    final_point = np.asarray(samples, dtype=np.float64).reshape(-1, 9)[:, 3:6]
    B = state.shape[0]
    gate_move, V = move(gp0, v, w, noise)
    u = np.zeros((B, 4))
    states, controls, ts, ins, outs, stats = [state], [], [], [], [], []
    for i in range(steps):
        gp = gate_move[:, i]
        t, _ = solve_t(dnn2, state, final_point, gp, V[:, i], w)
        ts.append(t)
        if i % CTRL_EVERY == 0:
            gn = rotate_y(translate(gp, V[:, i] * t[:, None]), w * t)
            inp = dnn2_inputs(gn, state, final_point)
            out = np.asarray(dnn2(inp), dtype=np.float32)
            u0, st = engine.get_input(inp[:, 0:13], inp[:, 13:16], out, u)
            u = u0.cpu().numpy()
            ins.append(inp)
            outs.append(out)
            stats.append(st.cpu().numpy())
        state = plant_step(state, u)
        states.append(state)
        controls.append(u)
    return {"states": np.stack(states, 1), "controls": np.stack(controls, 1), "t": np.stack(ts, 1),
            "ins18": np.stack(ins, 1), "outs": np.stack(outs, 1), "status": np.stack(stats, 1),
            "solves": B * len(ins), "gate_move": gate_move, "V": V}
