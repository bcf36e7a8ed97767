"""Where bench.py's per-step host time outside the solver kernel goes: the bench_rl step with synchronised
timers around sol_gradient, the counter read-back and each part of train_step."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402
from learningagileflight_se3_amd.policy_net import Network  # noqa: E402

dev = torch.device("cuda")
B = int(os.environ.get("B", "4096"))
sb = S.synthetic_batch(B, seed=1000)
ini, goal, gate, dnn = (torch.as_tensor(sb[k], device=dev) for k in ("ini", "goal", "gate12", "dnn_out"))
inputs = torch.as_tensor(sb["samples"], dtype=torch.float32, device=dev)
torch.manual_seed(0)
net = Network(9, 64, 64, 7).to(dev)
opt = torch.optim.Adam(net.parameters(), lr=1e-4)
eng = Engine(device=dev)
eng.reserve(9 * B)


def t():
    torch.cuda.synchronize()
    return time.perf_counter()


for rep in range(4):
    a = t()
    out8, _, st9 = eng.sol_gradient(ini, goal, gate, dnn, want_rewards=True)
    b = t()
    eng.last_kernel_ms()
    eng.last_counters()
    c = t()
    outputs = net(inputs)
    d = t()
    loss = net.myloss(outputs, out8[:, :7].to(outputs.dtype))
    e = t()
    opt.zero_grad(set_to_none=False)
    loss.backward()
    f = t()
    opt.step()
    g = t()
    print(f"rep {rep}: solve {1e3*(b-a):.1f} counters {1e3*(c-b):.2f} fwd {1e3*(d-c):.2f} loss {1e3*(e-d):.2f} "
          f"bwd {1e3*(f-e):.2f} adam {1e3*(g-f):.2f} ms", flush=True)
