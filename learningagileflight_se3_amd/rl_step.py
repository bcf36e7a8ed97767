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


class GraphedTrainStep:
    """train_step with its device work replayed from two HIP graphs (GPU only): [DNN1 forward, myloss, backward]
    and [Adam step], the gradient all-reduce between them left eager so that the same code serves every world
    size.  The step's ~40 small kernels cost ~0.6 ms of Python / autograd / launch time per call when issued one
    by one (more right after the host wakes from the solver's wait); a replay costs ~0.03 ms.  The arithmetic is
    the eager step's, with Adam in its capturable form (bias corrections from the on-device step count).

    Capturing needs warm-up steps on the real parameters; the parameters, the Adam moments and step counts are
    restored afterwards, so that the first call starts from the untouched network as the eager path does."""

    def __init__(self, net, opt, inputs, out8_shape, world: int = 1, group=None):
        if not all(g.get("capturable", False) for g in opt.param_groups):
            raise ValueError("GraphedTrainStep: the optimizer must be created with capturable=True")
        self.net, self.opt, self.world, self.group = net, opt, world, group
        self.inputs = inputs
        self.params = list(net.parameters())
        self.o8 = torch.zeros(out8_shape, dtype=torch.float64, device=inputs.device)
        saved = [p.detach().clone() for p in self.params]
        side = torch.cuda.Stream(device=inputs.device)
        side.wait_stream(torch.cuda.current_stream(inputs.device))
        with torch.cuda.stream(side):
            for _ in range(3):
                self.opt.zero_grad(set_to_none=True)
                self._forward_backward()
                allreduce_grads(self.params, world, group)
                self.opt.step()
        torch.cuda.current_stream(inputs.device).wait_stream(side)
        # the warm-up's collectives complete before the capture starts, and the capture checks only this thread's
        # HIP calls (a communicator's helper threads keep running beside it)
        torch.cuda.synchronize(inputs.device)
        self.opt.zero_grad(set_to_none=True)   # backward inside the capture writes (not accumulates) the grads
        self.g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fb, capture_error_mode="thread_local"):
            self.loss = self._forward_backward()
        self.g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_opt, capture_error_mode="thread_local"):
            self.opt.step()
        with torch.no_grad():
            for p, v in zip(self.params, saved):
                p.copy_(v)
            for st in self.opt.state.values():
                for v in st.values():
                    if torch.is_tensor(v):
                        v.zero_()
        torch.cuda.synchronize(inputs.device)

    def _forward_backward(self):
        outputs = self.net(self.inputs)
        loss = self.net.myloss(outputs, self.o8[:, :7].to(outputs.dtype))
        loss.backward()
        return loss.detach()

    def __call__(self, out8):
        self.o8.copy_(out8)
        self.g_fb.replay()
        allreduce_grads(self.params, self.world, self.group)
        self.g_opt.replay()
        return self.loss
