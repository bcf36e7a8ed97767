"""Host and device time of bench.py's train_step (DNN1 forward, batched myloss backward, Adam) at B = 4096, for
Adam variants: default (foreach), fused, and the whole step captured in a CUDA/HIP graph."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learningagileflight_se3_amd.policy_net import Network  # noqa: E402
from learningagileflight_se3_amd.rl_step import train_step  # noqa: E402

dev = torch.device("cuda")
B = 4096
torch.manual_seed(0)
inputs = torch.randn(B, 9, device=dev)
out8 = torch.randn(B, 8, dtype=torch.float64, device=dev)


def run(tag, opt_kw, n=20):
    torch.manual_seed(0)
    net = Network(9, 64, 64, 7).to(dev)
    opt = torch.optim.Adam(net.parameters(), lr=1e-4, **opt_kw)
    for _ in range(3):
        train_step(net, opt, inputs, out8)
    torch.cuda.synchronize()
    hs, ds = [], []
    for _ in range(n):
        t0 = time.perf_counter()
        train_step(net, opt, inputs, out8)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        hs.append(t1 - t0)
        ds.append(t2 - t0)
    hs.sort(); ds.sort()
    print(f"{tag:10s} host {1e3 * hs[n // 2]:.3f} ms  host+device {1e3 * ds[n // 2]:.3f} ms  (max {1e3 * ds[-1]:.3f})",
          flush=True)


run("default", {})
run("foreach", {"foreach": True})
run("fused", {"fused": True})


def run_graph(n=20):
    """the whole train_step captured once in a HIP graph (Adam capturable=True), replayed per step"""
    torch.manual_seed(0)
    net = Network(9, 64, 64, 7).to(dev)
    opt = torch.optim.Adam(net.parameters(), lr=1e-4, capturable=True)
    so8 = out8.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            train_step(net, opt, inputs, so8)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        train_step(net, opt, inputs, so8)
    torch.cuda.synchronize()
    hs, ds = [], []
    for _ in range(n):
        t0 = time.perf_counter()
        so8.copy_(out8)
        g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        hs.append(t1 - t0)
        ds.append(t2 - t0)
    hs.sort(); ds.sort()
    print(f"{'graph':10s} host {1e3 * hs[n // 2]:.3f} ms  host+device {1e3 * ds[n // 2]:.3f} ms  (max {1e3 * ds[-1]:.3f})",
          flush=True)


run("capturable", {"capturable": True})
run_graph()
