"""Imitation data for DNN2 from optimal trajectories: SURVEY.md §8(f) row 3, nn_train_2.py:29-96 batched.

Reference, per sample (one process each, nn_train_2.py:49-69):
  traj()    nn_train_2.py:29-40   gate corners from the sample (deep_learning.py:25-27), run_quad(goal, ini)
                                  and ``get_input(ini_state, tra_pos, tra_ang, t, Ulast=[0,0,0,0])`` on DNN1's
                                  float32 output; the state trajectory sol1['state_traj_opt'] (51 x 13).
  pairs     nn_train_2.py:72-84   50 (input 18, target 7) pairs per trajectory: input = [x_i (world frame),
                                  final position, gate width, gate pitch], target = [out[0:6], out[6] - 0.1 i].

Here all B trajectories come from ONE lafse3_get_input launch (the 51 x 13 trajectory is returned by the
kernel next to the first control), and the pairs are formed with array operations.
"""
from __future__ import annotations

import numpy as np
import torch

from . import scenario


def trajectories(engine, samples, dnn_out):
    """Optimal state trajectories (B, N+1, 13) for samples (B, 9) under DNN1 outputs (B, 7) float32.

    nn_train_2.py:30-39: ini_state from the sample (quad_policy.py:26-30), goal = sample[3:6],
    Ulast = [0,0,0,0] (passed explicitly by the reference; zero), t = out[6] unrounded (get_input).
    """
    samples = np.asarray(samples, dtype=np.float64).reshape(-1, 9)
    B = samples.shape[0]
    ini = scenario.initial_state(samples[:, 0:3], samples[:, 6])
    goal = samples[:, 3:6].copy()
    dnn = dnn_out if isinstance(dnn_out, torch.Tensor) else np.asarray(dnn_out, dtype=np.float32).reshape(B, 7)
    _, x, status = engine.get_input(ini, goal, dnn, np.zeros((B, 4)), want_x=True)
    return x, status


def imitation_pairs(samples, dnn_out, x, n_pairs: int | None = None):
    """(inputs (B*n, 18) float64, targets (B*n, 7) float32) of nn_train_2.py:72-84.

    The target's time entry follows the reference environment's NumPy 1.x scalar promotion: the float32
    DNN output minus the Python float 0.1*i is formed in float64, stored in a float64 array and cast to
    float32 by ``torch.tensor(out, dtype=torch.float)`` (SURVEY A10 for the same NumPy 2 caveat).
    """
    samples = np.asarray(samples, dtype=np.float64).reshape(-1, 9)
    out = np.asarray(dnn_out.detach().cpu().numpy() if isinstance(dnn_out, torch.Tensor) else dnn_out,
                     dtype=np.float32).reshape(-1, 7)
    xs = np.asarray(x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else x, dtype=np.float64)
    B = samples.shape[0]
    n = xs.shape[1] - 1 if n_pairs is None else n_pairs          # batch_size = 50 = horizon in the reference
    inputs = np.zeros((B, n, 18))
    inputs[:, :, 0:13] = xs[:, :n, :]
    inputs[:, :, 13:16] = samples[:, None, 3:6]
    inputs[:, :, 16:18] = samples[:, None, 7:9]
    targets = np.zeros((B, n, 7))
    targets[:, :, 0:6] = out[:, None, 0:6].astype(np.float64)
    targets[:, :, 6] = out[:, None, 6].astype(np.float64) - np.arange(n)[None, :] * 0.10
    return inputs.reshape(B * n, 18), targets.reshape(B * n, 7).astype(np.float32)
