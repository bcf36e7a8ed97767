"""Concurrency probe: one NLP instance replicated B times; kernel time vs B shows how many instance
waves the GPU actually runs at once (flat region) and the single-wave latency (B=1)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine

eng = Engine()
sb = S.synthetic_batch(8, seed=3)
i = int(os.environ.get("INST", "0"))
p = sb["dnn_out"][i:i + 1, :3].astype(np.float64); a = sb["dnn_out"][i:i + 1, 3:6].astype(np.float64)
t = sb["dnn_out"][i:i + 1, 6].astype(np.float64)
ini, goal = sb["ini"][i:i + 1], sb["goal"][i:i + 1]
for B in (1, 64, 256, 512, 768, 1024, 1280, 1536, 2048, 3072, 4096):
    rep = lambda z: np.repeat(z, B, axis=0)
    out = eng.ocp_solve(rep(ini), rep(goal), rep(p), rep(a), rep(t))
    torch.cuda.synchronize()
    ms = eng.last_kernel_ms(); cnt = eng.last_counters()
    print(f"B={B:5d} kernel {ms:8.2f} ms  iters/inst {cnt['iterations'] / B:.1f}  per-instance {ms / B * 1e3:.1f} us", flush=True)
