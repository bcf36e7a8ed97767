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


# ---- the same loop with the episode state on the device (torch, float64) --------------------------------
# Gate kinematics, the attitude transform (scipy's Rotation conventions restated: from_quat normalises,
# as_matrix of the unit quaternion, from_matrix by the largest of trace / diagonal, as_quat unnormalised
# sign), DNN2 and the plant run as batched torch ops on the GPU; the fixed-point loop checks convergence
# on the host every `check` iterations (converged episodes are masked, so the check interval does not
# change results).
def _quat_to_matrix_t(q):
    """scipy Rotation.from_quat(q).as_matrix() for (B, 4) [x, y, z, w]."""
    q = q / torch.linalg.vector_norm(q, dim=1, keepdim=True)
    x, y, z, w = q.unbind(1)
    x2, y2, z2, w2 = x * x, y * y, z * z, w * w
    xy, zw, xz, yw, yz, xw = x * y, z * w, x * z, y * w, y * z, x * w
    m = torch.stack([x2 - y2 - z2 + w2, 2 * (xy - zw), 2 * (xz + yw),
                     2 * (xy + zw), -x2 + y2 - z2 + w2, 2 * (yz - xw),
                     2 * (xz - yw), 2 * (yz + xw), -x2 - y2 + z2 + w2], dim=1)
    return m.reshape(-1, 3, 3)


def _matrix_to_quat_t(m):
    """scipy Rotation.from_matrix(m).as_quat() for (B, 3, 3) rotation matrices: [x, y, z, w]."""
    d = torch.stack([m[:, 0, 0], m[:, 1, 1], m[:, 2, 2]], dim=1)
    tr = d.sum(1)
    choice = torch.argmax(torch.cat([d, tr[:, None]], dim=1), dim=1)
    q = torch.zeros(m.shape[0], 4, dtype=m.dtype, device=m.device)
    # trace branch
    qt = torch.stack([m[:, 2, 1] - m[:, 1, 2], m[:, 0, 2] - m[:, 2, 0], m[:, 1, 0] - m[:, 0, 1], 1 + tr], dim=1)
    q = torch.where((choice == 3)[:, None], qt, q)
    for i in range(3):
        j, k = (i + 1) % 3, (i + 2) % 3
        qi = torch.zeros_like(q)
        qi[:, i] = 1 - tr + 2 * m[:, i, i]
        qi[:, j] = m[:, j, i] + m[:, i, j]
        qi[:, k] = m[:, k, i] + m[:, i, k]
        qi[:, 3] = m[:, k, j] - m[:, j, k]
        q = torch.where((choice == i)[:, None], qi, q)
    return q / torch.linalg.vector_norm(q, dim=1, keepdim=True)


def centroid_t(gp):
    return ((gp[:, 0] + gp[:, 1]) + gp[:, 2] + gp[:, 3]) / 4.0


def gate_frame_t(gp):
    ay = torch.cross(gp[:, 1] - gp[:, 0], gp[:, 2] - gp[:, 1], dim=1)
    ay = ay / torch.sqrt((ay * ay).sum(1, keepdim=True))
    az = torch.zeros_like(ay)
    az[:, 2] = 1.0
    ax = torch.cross(ay, az, dim=1)
    return torch.stack([ax, ay, az], dim=1)


def rotate_y_t(gp, angle):
    c = centroid_t(gp)
    rel = gp - c[:, None, :]
    ca, sa = torch.cos(angle)[:, None], torch.sin(angle)[:, None]
    x0, z0 = rel[:, :, 0], rel[:, :, 2]
    out = torch.stack([ca * x0 + (-sa) * z0, rel[:, :, 1], sa * x0 + ca * z0], dim=2)
    return out + c[:, None, :]


def dnn2_inputs_t(gp, state, final_point):
    IG, cen = gate_frame_t(gp), centroid_t(gp)
    d01 = gp[:, 0] - gp[:, 1]
    quat = torch.cat([state[:, 7:10], state[:, 6:7]], dim=1)
    qo = _matrix_to_quat_t(torch.matmul(IG, _quat_to_matrix_t(quat)))
    return torch.cat([torch.einsum("bij,bj->bi", IG, state[:, 0:3] - cen),
                      torch.einsum("bij,bj->bi", IG, state[:, 3:6]),
                      qo[:, 3:4], qo[:, 0:3], state[:, 10:13],
                      torch.einsum("bij,bj->bi", IG, final_point - cen),
                      torch.sqrt((d01 * d01).sum(1, keepdim=True)),
                      torch.atan(d01[:, 2:3] / d01[:, 0:1])], dim=1)


def solve_t_t(net, state, final_point, gp, velo, w, max_iter=200, check=4):
    """quad_moving.solver on the device (see solve_t); net: DNN2 nn.Module on the same device."""
    d = centroid_t(gp) - state[:, 0:3]
    t1 = torch.sqrt((d * d).sum(1)) / 3
    active = torch.ones_like(t1, dtype=torch.bool)

    def t_of(t):
        gx = rotate_y_t(gp + (velo * t[:, None])[:, None, :], w * t)
        with torch.no_grad():
            return net(dnn2_inputs_t(gx, state, final_point).float())[:, 6].double()

    t2 = t_of(t1)
    for n in range(max_iter):
        active = active & (torch.abs(t2 - t1) > T_TOL)
        if n % check == 0 and not bool(active.any()):
            break
        t1 = torch.where(active, t1 + (t2 - t1) / 2, t1)
        t2 = torch.where(active, t_of(t1), t2)
    return t1


class FixedPointGraph:
    """solve_t_t with its iterations captured in HIP graphs (the loop is launch-bound: ~80 tiny kernels per
    iteration).  One graph computes t1, t2 from the staged inputs, one graph runs `check` masked iterations;
    the host replays the second until no episode is active (converged episodes are masked, so the result is
    that of solve_t_t)."""

    def __init__(self, net, B, w, device, check=4):
        self.net, self.w, self.check = net, w, check
        f64 = dict(dtype=torch.float64, device=device)
        self.state, self.final = torch.zeros(B, 13, **f64), torch.zeros(B, 3, **f64)
        self.gp, self.velo = torch.zeros(B, 4, 3, **f64), torch.zeros(B, 3, **f64)
        self.t1, self.t2 = torch.zeros(B, **f64), torch.zeros(B, **f64)
        self.active = torch.ones(B, dtype=torch.bool, device=device)
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):          # warm-up outside capture (allocator, BLAS handles)
            self._init()
            self._iters()
        torch.cuda.current_stream(device).wait_stream(s)
        self.g_init, self.g_iter = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_init):
            self._init()
        with torch.cuda.graph(self.g_iter):
            self._iters()

    def _t_of(self, t):
        gx = rotate_y_t(self.gp + (self.velo * t[:, None])[:, None, :], self.w * t)
        with torch.no_grad():
            return self.net(dnn2_inputs_t(gx, self.state, self.final).float())[:, 6].double()

    def _init(self):
        d = centroid_t(self.gp) - self.state[:, 0:3]
        self.t1.copy_(torch.sqrt((d * d).sum(1)) / 3)
        self.t2.copy_(self._t_of(self.t1))
        self.active.fill_(True)

    def _iters(self):
        for _ in range(self.check):
            self.active.copy_(self.active & (torch.abs(self.t2 - self.t1) > T_TOL))
            self.t1.copy_(torch.where(self.active, self.t1 + (self.t2 - self.t1) / 2, self.t1))
            self.t2.copy_(torch.where(self.active, self._t_of(self.t1), self.t2))

    def solve(self, state, final_point, gp, velo, max_iter=200):
        self.state.copy_(state)
        self.final.copy_(final_point)
        self.gp.copy_(gp)
        self.velo.copy_(velo)
        self.g_init.replay()
        for _ in range(0, max_iter, self.check):
            self.g_iter.replay()
            if not bool((self.active & (torch.abs(self.t2 - self.t1) > T_TOL)).any()):
                break
        return self.t1.clone()


def plant_step_t(state, u, dt=DT_PLANT):
    """plant_step on the device (same constants and operation order)."""
    m, Jx, Jy, Jz, l, c, g = 0.5, 0.0023, 0.0023, 0.004, 0.35, 0.0245, 9.78
    v, q, w = state[:, 3:6], state[:, 6:10], state[:, 10:13]
    T = u.sum(1)
    hl = l / 2
    Mx, My, Mz = hl * (u[:, 3] - u[:, 1]), hl * (u[:, 2] - u[:, 0]), c * (u[:, 0] - u[:, 1] + u[:, 2] - u[:, 3])
    f = torch.stack([
        v[:, 0], v[:, 1], v[:, 2],
        T / m * (2 * (q[:, 1] * q[:, 3] + q[:, 0] * q[:, 2])),
        T / m * (2 * (q[:, 2] * q[:, 3] - q[:, 0] * q[:, 1])),
        T / m * (1 - 2 * (q[:, 1] ** 2 + q[:, 2] ** 2)) - g,
        0.5 * (-w[:, 0] * q[:, 1] - w[:, 1] * q[:, 2] - w[:, 2] * q[:, 3]),
        0.5 * (w[:, 0] * q[:, 0] + w[:, 2] * q[:, 2] - w[:, 1] * q[:, 3]),
        0.5 * (w[:, 1] * q[:, 0] - w[:, 2] * q[:, 1] + w[:, 0] * q[:, 3]),
        0.5 * (w[:, 2] * q[:, 0] + w[:, 1] * q[:, 1] - w[:, 0] * q[:, 2]),
        (Mx - (Jz - Jy) * w[:, 1] * w[:, 2]) / Jx,
        (My - (Jx - Jz) * w[:, 0] * w[:, 2]) / Jy,
        (Mz - (Jy - Jx) * w[:, 0] * w[:, 1]) / Jz], dim=1)
    return state + dt * f


def run_episodes_device(engine, net, samples, noise, v=(1.0, 0.3, 0.4), w=math.pi / 2, steps=500, check=4,
                        graphs=True, fixed_point="kernel", counters=None, capture=None):
    """run_episodes with the episode state on the GPU (gate motion precomputed by ``move`` on the host).
    fixed_point: "kernel" = one lafse3_traversal_time launch per plant step (HIP, the whole fixed point of
    quad_moving.solver with DNN2 inside); "torch" = solve_t_t as batched torch ops, through FixedPointGraph
    when graphs=True.  counters: a list that receives engine.last_counters() + kernel_ms after every get_input (diagnostics;
    each read waits for the launch).  capture: a list that receives, per get_input, the MPC instance inputs
    (gate-frame state, gate-frame goal, DNN2 output, u_last) and the statuses (diagnostics / fixtures)."""
    dev = engine.device
    gp0, state0 = initial_episodes(samples)
    gate_move, V = move(gp0, v, w, noise[:, :max(steps, 1)])
    gm = torch.as_tensor(gate_move, device=dev)
    Vt = torch.as_tensor(V, device=dev)
    final_point = torch.as_tensor(np.asarray(samples, dtype=np.float64).reshape(-1, 9)[:, 3:6], device=dev)
    state = torch.as_tensor(state0, device=dev)
    B = state.shape[0]
    u = torch.zeros(B, 4, dtype=torch.float64, device=dev)
    states, ts, solves = [state], [], 0
    stats = []
    if fixed_point not in ("kernel", "torch"):
        raise ValueError("fixed_point is 'kernel' or 'torch'")
    fp = FixedPointGraph(net, B, w, dev, check) if (graphs and fixed_point == "torch") else None
    for i in range(steps):
        gp = gm[:, i]
        if fixed_point == "kernel":
            t = engine.traversal_time(state, final_point, gp, Vt[:, i], w, net)
        elif fp is not None:
            t = fp.solve(state, final_point, gp, Vt[:, i])
        else:
            t = solve_t_t(net, state, final_point, gp, Vt[:, i], w, check=check)
        ts.append(t)
        if i % CTRL_EVERY == 0:
            gn = rotate_y_t(gp + (Vt[:, i] * t[:, None])[:, None, :], w * t)
            inp = dnn2_inputs_t(gn, state, final_point)
            with torch.no_grad():
                out = net(inp.float())
            u_prev = u
            u, st = engine.get_input(inp[:, 0:13].contiguous(), inp[:, 13:16].contiguous(), out.contiguous(), u)
            stats.append(st)
            if capture is not None:
                capture.append({"ini": inp[:, 0:13].clone(), "goal": inp[:, 13:16].clone(), "dnn_out": out.clone(),
                                "u_last": u_prev.clone(), "status": st.clone(), "step": i})
            solves += B
            if counters is not None:
                counters.append(dict(engine.last_counters(), **engine.last_resto_counters(),
                                     kernel_ms=engine.last_kernel_ms()))
        state = plant_step_t(state, u)
        states.append(state)
    return {"states": torch.stack(states, 1), "t": torch.stack(ts, 1), "status": torch.stack(stats, 1),
            "solves": solves}
