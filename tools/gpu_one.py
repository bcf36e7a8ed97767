"""One launch of a single NLP instance replicated B times (clean per-wave PMC numbers)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine

B = int(os.environ.get("B", "2048"))
eng = Engine()
sb = S.synthetic_batch(8, seed=3)
i = 0
rep = lambda z: np.repeat(z[i:i + 1], B, axis=0)
p = sb["dnn_out"][:, :3].astype(np.float64); a = sb["dnn_out"][:, 3:6].astype(np.float64)
t = sb["dnn_out"][:, 6].astype(np.float64)
out = eng.ocp_solve(rep(sb["ini"]), rep(sb["goal"]), rep(p), rep(a), rep(t))
torch.cuda.synchronize()
print(f"B={B} kernel {eng.last_kernel_ms():.2f} ms counters {eng.last_counters()}", flush=True)
