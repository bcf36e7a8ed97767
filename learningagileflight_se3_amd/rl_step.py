"""Batched, data-parallel form of the reference's RL step (deep_learning.py:45-83).

Reference (per sample, one process each through multiprocessing, deep_learning.py:66-72):
  out = DNN1(inputs);  grad = run_quad.sol_gradient(out)  (9 MPC solves);
  loss = myloss(out, grad[:7]);  loss.backward();  optimizer.step()      (deep_learning.py:75-81)

Here: every rank owns a contiguous shard of the batch (weak scaling), solves its shard's
sol_gradient on its own GPU, forms the batched myloss, and the only collective is one SUM all-reduce
of the DNN1 parameter gradients (RCCL over xGMI on GPUs, gloo on CPU in the tests) before one Adam
step per batch (documented semantics change — one optimizer step per batch).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) slice of a batch of n_total for `rank` (sizes differ by at most one)."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def allreduce_grads(params, world: int, group=None):
    """SUM all-reduce of the parameter gradients, bucketed into one flat buffer (one collective)."""
    if world <= 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


def train_step(net, opt, inputs, out8, world: int = 1, group=None):
    """One batched RL step given this shard's MPC gradients out8 (B, 8): returns the local loss."""
    outputs = net(inputs)
    loss = net.myloss(outputs, out8[:, :7].to(outputs.dtype))
    opt.zero_grad(set_to_none=False)
    loss.backward()
    allreduce_grads(list(net.parameters()), world, group)
    opt.step()
    return loss.detach()
