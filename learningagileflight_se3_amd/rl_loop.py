"""The reference's RL training loop on the engine: SURVEY.md §8(f) row 2, deep_learning.py:34-94.

Reference, per epoch (deep_learning.py:41-93): batch_size samples in groups of num_cores.  For a group the
DNN1 outputs are taken at the current parameters (deep_learning.py:51-63), every sample's
``run_quad.sol_gradient`` runs in its own process (deep_learning.py:24-32, 66-72), then one Adam step per
sample, in sample order, on ``myloss(model(inputs_j), grad_j[0:7])`` (deep_learning.py:75-81).  The reward
grad_j[7] goes to Every_reward[epoch, j] and its batch mean to Mean_Reward (deep_learning.py:82-93).

Here a group's sol_gradient calls are ONE lafse3_sol_gradient launch (9 NLP solves per sample on the GPU).
``update="reference"`` replays the per-sample Adam steps of a group in the reference's order;
``update="batched"`` takes one step per group on the summed loss (rl_step.train_step, the data-parallel
form bench.py measures).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import scenario
from .rl_step import train_step


def engine_gradient(engine, grad_mode: int | None = None):
    """grad_fn for run_rl: the reference's per-sample ``grad`` (deep_learning.py:24-32), batched on the GPU.
    ``grad_mode`` 1 uses the IFT gradient (3 solves + 6 sensitivity sweeps per sample, lafse3.h) instead of
    the reference's 9-solve FD; None keeps the engine's setting (FD by default)."""

    def grad_fn(samples, dnn_out):
        samples = np.asarray(samples, dtype=np.float64)
        ini = scenario.initial_state(samples[:, 0:3], samples[:, 6])
        gate12 = scenario.gate_corners(samples[:, 7], samples[:, 8])
        out8 = engine.sol_gradient(ini, samples[:, 3:6], gate12, np.asarray(dnn_out, dtype=np.float32),
                                   grad_mode=grad_mode)
        return out8.cpu().numpy()

    return grad_fn


def run_rl(net, opt, grad_fn, epochs: int, batch_size: int = 100, num_cores: int = 10,
           update: str = "reference", rng: np.random.Generator | None = None, out_dir: str | None = None,
           run: int = 0):
    """deep_learning.py:41-93 for `epochs` epochs.  grad_fn(samples (G,9), dnn_out (G,7) float32) -> (G,8).

    Returns {"every_reward": (epochs, batch_size), "mean_reward": (epochs,)} (the arrays the reference
    saves as Every_reward / Mean_Reward).  With ``out_dir`` the run's outputs are written as the reference
    writes them (deep_learning.py:91-94) for run index ``run`` (the reference's k): after every epoch
    Iteration.npy, Mean_Reward{run}.npy (the epochs so far) and Every_reward{run}.npy; at the end the
    network as nn_deep2_{run}.pt -- its state_dict (torch.save of the whole module, as the reference does,
    would pickle the class)."""
    if update not in ("reference", "batched"):
        raise ValueError("update is 'reference' or 'batched'")
    rng = np.random.default_rng(0) if rng is None else rng
    dev = next(net.parameters()).device
    every = np.zeros((epochs, batch_size))
    mean = np.zeros(epochs)
    groups = batch_size // num_cores
    for ep in range(epochs):
        evalue = 0.0
        for i in range(groups):
            samples = np.stack([scenario.nn_sample(rng) for _ in range(num_cores)])
            x = torch.as_tensor(samples, dtype=torch.float32, device=dev)     # torch.tensor(input, dtype=float)
            with torch.no_grad():                                             # deep_learning.py:55-56 (float32)
                if update == "reference":   # one forward per sample, as the reference (bitwise-identical outputs)
                    out = torch.stack([net(x[j]) for j in range(num_cores)]).cpu().numpy()
                else:
                    out = net(x).cpu().numpy()
            g8 = np.asarray(grad_fn(samples, out), dtype=np.float64)
            if update == "reference":
                for j in range(num_cores):                                    # deep_learning.py:75-81
                    outputs = net(x[j])
                    loss = net.myloss(outputs, torch.as_tensor(g8[j, 0:7], dtype=torch.float32, device=dev))
                    opt.zero_grad()
                    loss.backward()
                    opt.step()
            else:
                train_step(net, opt, x, torch.as_tensor(g8, device=dev), 1)
            evalue += float(g8[:, 7].sum())
            every[ep, i * num_cores:(i + 1) * num_cores] = g8[:, 7]
        mean[ep] = evalue / batch_size
        if out_dir is not None:
            os.makedirs(out_dir, exist_ok=True)
            np.save(os.path.join(out_dir, "Iteration.npy"), np.arange(1, ep + 2))
            np.save(os.path.join(out_dir, f"Mean_Reward{run}.npy"), mean[:ep + 1])
            np.save(os.path.join(out_dir, f"Every_reward{run}.npy"), every)
    if out_dir is not None:
        torch.save(net.state_dict(), os.path.join(out_dir, f"nn_deep2_{run}.pt"))
    return {"every_reward": every, "mean_reward": mean}
