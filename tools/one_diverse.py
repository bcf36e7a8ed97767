"""One ocp_solve launch of B distinct instances (synthetic_batch seed 5) -- the diverse counterpart of gpu_one.py."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402

B = int(os.environ.get("B", "1024"))
eng = Engine()
sb = S.synthetic_batch(B, seed=5)
p = sb["dnn_out"][:, :3].astype(np.float64)
a = sb["dnn_out"][:, 3:6].astype(np.float64)
t = sb["dnn_out"][:, 6].astype(np.float64)
eng.ocp_solve(sb["ini"], sb["goal"], p, a, t)
torch.cuda.synchronize()
print(f"B={B} kernel {eng.last_kernel_ms():.2f} ms counters {eng.last_counters()}", flush=True)
