"""Policy MLP of the reference (quad_nn.py:119-145), kept in PyTorch (ROCm) as the north star asks.

``Network(D_in, D_h1, D_h2, D_out)`` = Linear-ReLU-Linear-ReLU-Linear; ``myloss(para, dp)`` = Dp . para,
the "loss" through which the MPC gradient is injected (deep_learning.py:76-81).  Batched: para (B, 7),
dp (B, 7) -> scalar sum_i dp_i . para_i (one optimizer step per batch instead of the reference's one
per sample — the documented semantics change of SURVEY.md §8(e)).
"""
from __future__ import annotations

import torch
import torch.nn as nn


class Network(nn.Module):
    def __init__(self, D_in: int, D_h1: int, D_h2: int, D_out: int):
        super().__init__()
        self.l1 = nn.Linear(D_in, D_h1)
        self.F1 = nn.ReLU()
        self.l2 = nn.Linear(D_h1, D_h2)
        self.F2 = nn.ReLU()
        self.l3 = nn.Linear(D_h2, D_out)

    def forward(self, x):
        if not isinstance(x, torch.Tensor):
            x = torch.tensor(x, dtype=torch.float)
        return self.l3(self.F2(self.l2(self.F1(self.l1(x)))))

    @staticmethod
    def myloss(para, dp):
        dp = dp if isinstance(dp, torch.Tensor) else torch.tensor(dp, dtype=torch.float, device=para.device)
        if para.dim() == 1:
            return torch.matmul(dp, para)
        return (dp * para).sum()
