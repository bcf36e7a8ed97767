"""Multi-rank path on CPU (gloo, world size 2): sharding + the single gradient all-reduce.

The data-parallel RL step (learningagileflight_se3_amd/rl_step.py) must give every rank the same
parameters after a step, equal to a single-process step over the whole batch (the sum of shard losses
is the full-batch loss).  The MPC gradients out8 are synthetic here (no GPU): the collective path is
what is under test.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from learningagileflight_se3_amd.policy_net import Network
from learningagileflight_se3_amd.rl_step import shard_range, train_step


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(B):
    g = torch.Generator().manual_seed(11)
    return torch.randn(B, 9, generator=g), torch.randn(B, 8, generator=g, dtype=torch.float64)


def _worker(rank, world, port, B, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = Network(9, 64, 64, 7).double()
    opt = torch.optim.Adam(net.parameters(), lr=1e-2)
    x, o8 = _data(B)
    lo, hi = shard_range(B, rank, world)
    for _ in range(3):
        train_step(net, opt, x[lo:hi].double(), o8[lo:hi], world)
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
    np.save(os.path.join(out_dir, f"r{rank}.npy"), flat.numpy())
    dist.destroy_process_group()


def test_shard_range_covers_batch():
    for n in (0, 1, 7, 64, 4097):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_step_matches_single_process(tmp_path):
    B, world = 10, 2
    mp.spawn(_worker, args=(world, _free_port(), B, str(tmp_path)), nprocs=world, join=True)
    r0, r1 = np.load(tmp_path / "r0.npy"), np.load(tmp_path / "r1.npy")
    assert np.array_equal(r0, r1)                  # replicas stay identical
    torch.manual_seed(0)
    net = Network(9, 64, 64, 7).double()
    opt = torch.optim.Adam(net.parameters(), lr=1e-2)
    x, o8 = _data(B)
    for _ in range(3):
        train_step(net, opt, x.double(), o8, 1)
    ref = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).numpy()
    assert np.max(np.abs(r0 - ref)) < 1e-12
