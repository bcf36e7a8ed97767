"""Independent KKT certificate for solutions of the quad_OC NLP (quad_OC.py:124-174).

The NLP is rebuilt here from scratch in torch fp64 (objective + multiple-shooting defects) and
differentiated by autograd — no code shared with the oracle or the HIP kernels — so a small residual
certifies that a returned (x*, u*, lam*) is a first-order KKT point of the reference's NLP:

    min  sum_k [w_k tra(x_k) + path(x_k) + 0.1||u_k||^2 + ||u_k - u_{k-1}||^2] + path(x_N)
    s.t. x_{k+1} = x_k + dt f(x_k, u_k),  0 <= u <= 2.44,  |omega_k| <= pi/2 (k >= 1)
"""
from __future__ import annotations

import math

import numpy as np
import torch

DT = 0.1
MASS, JX, JY, JZ, ARM, CT, G = 0.5, 0.0023, 0.0023, 0.004, 0.35, 0.0245, 9.78
U_UB, W_UB = 2.44, math.pi / 2


def _dcm(q):
    q0, q1, q2, q3 = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    return torch.stack([
        torch.stack([1 - 2 * (q2 ** 2 + q3 ** 2), 2 * (q1 * q2 + q0 * q3), 2 * (q1 * q3 - q0 * q2)], -1),
        torch.stack([2 * (q1 * q2 - q0 * q3), 1 - 2 * (q1 ** 2 + q3 ** 2), 2 * (q2 * q3 + q0 * q1)], -1),
        torch.stack([2 * (q1 * q3 + q0 * q2), 2 * (q2 * q3 - q0 * q1), 1 - 2 * (q1 ** 2 + q2 ** 2)], -1)], -2)


def _f(x, u):
    v, q, w = x[..., 3:6], x[..., 6:10], x[..., 10:13]
    T = u.sum(-1, keepdim=True)
    C = _dcm(q)
    acc = T / MASS * C[..., 2, :] + torch.tensor([0.0, 0.0, -G], dtype=x.dtype)
    wx, wy, wz = w[..., 0], w[..., 1], w[..., 2]
    q0, q1, q2, q3 = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    dq = 0.5 * torch.stack([-wx * q1 - wy * q2 - wz * q3, wx * q0 + wz * q2 - wy * q3,
                            wy * q0 - wz * q1 + wx * q3, wz * q0 + wy * q1 - wx * q2], -1)
    f1, f2, f3, f4 = u[..., 0], u[..., 1], u[..., 2], u[..., 3]
    M = torch.stack([ARM / 2 * (f4 - f2), ARM / 2 * (f3 - f1), CT * (f1 - f2 + f3 - f4)], -1)
    Jv = torch.tensor([JX, JY, JZ], dtype=x.dtype)
    dw = (M - torch.cross(w, Jv * w, dim=-1)) / Jv
    return torch.cat([v, acc, dq, dw], -1)


def objective_and_defects(x, u, ini, goal, ptra, qtra, t, ulast):
    """x: (N+1,13) with x[0] = ini, u: (N,4). Returns J (scalar), c (N,13)."""
    N = u.shape[0]
    Rt = _dcm(qtra)
    k = torch.arange(N + 1, dtype=x.dtype)
    wk = 60 * torch.exp(-10 * (DT * k - t) ** 2)
    r, v, w = x[:, 0:3], x[:, 3:6], x[:, 10:13]
    path = 5 * ((r - goal) ** 2).sum(-1) + 5 * (v ** 2).sum(-1) + 3 * (w ** 2).sum(-1)
    tau = 3 - (Rt * _dcm(x[:, 6:10])).sum((-1, -2))
    tra = 5 * ((r - ptra) ** 2).sum(-1) + 80 * tau ** 2
    uprev = torch.cat([ulast[None], u[:-1]], 0)
    J = (wk[:N] * tra[:N] + path[:N]).sum() + 0.1 * (u ** 2).sum() + ((u - uprev) ** 2).sum() + path[N]
    c = x[:-1] + DT * _f(x[:-1], u) - x[1:]
    return J, c


def dual_scale(lam):
    """IPOPT's dual-infeasibility scaling s_d = max(s_max, mean |multiplier|) / s_max, s_max = 100
    (Waechter & Biegler 2006, eq. 6): the solver stops on dual / s_d, so a certificate on the unscaled
    dual residual carries the same factor (equality multipliers only; the bound duals are implied here)."""
    return max(100.0, float(np.mean(np.abs(np.asarray(lam, dtype=np.float64))))) / 100.0


def kkt_residual(x, u, lam, ini, goal, ptra, qtra, t, ulast=None):
    """Projected first-order residuals at one solution.

    Returns dict(primal=max|c|, dual=max |grad L| over unbounded variables, compl=max complementarity
    of the implied bound multipliers, bound_viol, J).
    lam follows CasADi's lam_g convention (L = J + lam^T g, g_k = f_d(x_k,u_k) - x_{k+1}).
    """
    dt = torch.float64
    X = torch.tensor(x, dtype=dt, requires_grad=True)
    U = torch.tensor(u, dtype=dt, requires_grad=True)
    L = torch.tensor(lam, dtype=dt)
    args = [torch.tensor(np.asarray(a, dtype=np.float64), dtype=dt) for a in (ini, goal, ptra, qtra)]
    tt = torch.tensor(float(t), dtype=dt)
    ul = torch.zeros(4, dtype=dt) if ulast is None else torch.tensor(np.asarray(ulast, np.float64), dtype=dt)
    J, c = objective_and_defects(X, U, args[0], args[1], args[2], args[3], tt, ul)
    Lag = J + (L * c).sum()
    gX, gU = torch.autograd.grad(Lag, [X, U])
    gX, gU = gX.numpy()[1:], gU.numpy()           # x_0 is fixed
    xs, us = np.asarray(x)[1:], np.asarray(u)
    # bounded variables: implied bound multipliers z_L = max(r, 0), z_U = max(-r, 0); certify
    # complementarity z_L (v - lb) and z_U (ub - v).  Unbounded variables: |r|.
    def box(r, v, lb, ub):
        zl, zu = np.maximum(r, 0.0), np.maximum(-r, 0.0)
        return float(np.max(np.maximum(zl * (v - lb), zu * (ub - v)), initial=0.0))
    compl = max(box(gU, us, 0.0, U_UB), box(gX[:, 10:13], xs[:, 10:13], -W_UB, W_UB))
    dual = float(np.max(np.abs(gX[:, :10])))
    bound_viol = float(max(np.max(-us, initial=0), np.max(us - U_UB, initial=0),
                           np.max(np.abs(xs[:, 10:13]) - W_UB, initial=0)))
    return {"primal": float(np.max(np.abs(c.detach().numpy()))), "dual": dual, "compl": compl,
            "s_d": dual_scale(lam),
            "bound_viol": bound_viol, "J": float(J.detach())}
