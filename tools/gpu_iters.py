"""Per-instance IPM iteration counts of the bench batch (B samples x 9 solves, seed 1000) -> gpurun_out/iters.npz,
for dispatch-order studies (tail of the launch)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine

B = int(os.environ.get("B", "4096"))
sb = S.synthetic_batch(B, seed=1000)
eng = Engine()
it = torch.full((B, 9), -1, dtype=torch.int32, device="cuda")
eng.record_iters(it)
out8, R9, S9 = eng.sol_gradient(sb["ini"], sb["goal"], sb["gate12"], sb["dnn_out"], want_rewards=True)
torch.cuda.synchronize()
print("kernel ms", eng.last_kernel_ms(), eng.last_counters(), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/iters.npz", it=it.cpu().numpy(), st=S9.cpu().numpy(), ini=sb["ini"], goal=sb["goal"],
         dnn=sb["dnn_out"], kernel_ms=eng.last_kernel_ms())
