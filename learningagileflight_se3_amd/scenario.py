"""Host-side scenario preparation for the batched MPC hot path.

Restates the reference's per-sample input prep (12 numbers per instance, host side):
  * ``nn_sample``           quad_nn.py:18-48    (random start / goal / yaw / gate width / pitch)
  * ``gate_corners``        deep_learning.py:25-27 + quad_model.py:672-683 (gate.__init__)
                            + quad_model.py:735-741 (gate.rotate_y_out)
  * ``initial_state``       quad_policy.py:26-30 + quad_model.py:818-825 (toQuaternion(yaw, [0,0,1]))
  * ``synthetic_batch``     SURVEY.md §8(d): seeded batch of (ini_state, goal, gate12, dnn_out)

Everything here is vectorised numpy over the batch; none of it is on the device hot path.
"""
from __future__ import annotations

import math

import numpy as np


def to_quaternion(angle: float, direction) -> np.ndarray:
    """toQuaternion(angle, dir)  quad_model.py:818-825."""
    d = np.asarray(direction, dtype=np.float64)
    d = d / np.linalg.norm(d)
    q = np.zeros(4)
    q[0] = math.cos(angle / 2)
    q[1:] = math.sin(angle / 2) * d
    return q


def nn_sample(rng: np.random.Generator) -> np.ndarray:
    """One 9-vector [p0(3), goal(3), yaw, width, pitch] with quad_nn.py:18-48's distributions."""
    x = np.zeros(9)
    x[0:3] = rng.uniform(-5, 5, size=3) + np.array([0, -9, 0])
    x[3:6] = rng.uniform(-2, 2, size=3) + np.array([0, 6, 0])
    x[6] = rng.uniform(-0.1, 0.1)
    x[7] = np.clip(rng.normal(0.9, 0.3), 0.5, 1.25)
    angle = np.clip(1.3 * (1.2 - x[7]), 0, math.pi / 3)
    angle1 = (math.pi / 2 - angle) / 3
    judge = rng.normal(0, 1)
    if judge > 0:
        x[8] = np.clip(rng.normal(angle + angle1, 2 * angle1 / 3), angle, math.pi / 2)
    else:
        x[8] = np.clip(rng.normal(-angle - angle1, 2 * angle1 / 3), -math.pi / 2, -angle)
    return x


def gate_corners(width, pitch) -> np.ndarray:
    """Gate of width ``width`` pitched by ``pitch`` about its centroid (x-z plane).

    deep_learning.py:25-27: corners [[-w/2,0,1],[w/2,0,1],[w/2,0,-1],[-w/2,0,-1]] then
    gate.rotate_y_out(pitch) (quad_model.py:735-741).  Vectorised: width/pitch arrays of shape (B,).
    Returns (B, 12).
    """
    w = np.atleast_1d(np.asarray(width, dtype=np.float64))
    a = np.atleast_1d(np.asarray(pitch, dtype=np.float64))
    B = w.shape[0]
    pts = np.zeros((B, 4, 3))
    pts[:, 0] = np.stack([-w / 2, np.zeros(B), np.ones(B)], -1)
    pts[:, 1] = np.stack([w / 2, np.zeros(B), np.ones(B)], -1)
    pts[:, 2] = np.stack([w / 2, np.zeros(B), -np.ones(B)], -1)
    pts[:, 3] = np.stack([-w / 2, np.zeros(B), -np.ones(B)], -1)
    cen = pts.mean(axis=1, keepdims=True)
    rel = pts - cen
    c, s = np.cos(a)[:, None], np.sin(a)[:, None]
    x0, z0 = rel[..., 0].copy(), rel[..., 2].copy()
    rel[..., 0] = c * x0 - s * z0
    rel[..., 2] = s * x0 + c * z0
    return (rel + cen).reshape(B, 12)


def initial_state(p0, yaw) -> np.ndarray:
    """ini_state = [p0, 0,0,0, toQuaternion(yaw,[0,0,1]), 0,0,0]  (quad_policy.py:26-30)."""
    p0 = np.atleast_2d(np.asarray(p0, dtype=np.float64))
    yaw = np.atleast_1d(np.asarray(yaw, dtype=np.float64))
    B = p0.shape[0]
    x = np.zeros((B, 13))
    x[:, 0:3] = p0
    x[:, 6] = np.cos(yaw / 2)
    x[:, 9] = np.sin(yaw / 2)
    return x


def synthetic_batch(B: int, seed: int = 0):
    """Seeded synthetic workload of SURVEY.md §8(d).

    Returns dict with ini (B,13) f64, goal (B,3) f64, gate12 (B,12) f64, dnn_out (B,7) float32
    (p_tra ~ U(-0.3,0.3)^3, a_tra ~ U(-0.5,0.5)^3, t in {2.0,...,4.0}), samples (B,9).
    """
    rng = np.random.default_rng(seed)
    samples = np.stack([nn_sample(rng) for _ in range(B)]) if B > 0 else np.zeros((0, 9))
    ini = initial_state(samples[:, 0:3], samples[:, 6])
    goal = samples[:, 3:6].copy()
    gate12 = gate_corners(samples[:, 7], samples[:, 8])
    dnn = np.zeros((B, 7), dtype=np.float32)
    dnn[:, 0:3] = rng.uniform(-0.3, 0.3, size=(B, 3))
    dnn[:, 3:6] = rng.uniform(-0.5, 0.5, size=(B, 3))
    dnn[:, 6] = 2.0 + 0.1 * rng.integers(0, 21, size=B)
    return {"ini": ini, "goal": goal, "gate12": gate12, "dnn_out": dnn, "samples": samples}
