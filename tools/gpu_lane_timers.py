"""Per-phase cycle breakdown of the lane kernel (one accumulator set per wave)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine

B = int(os.environ.get("B", "256"))
names = ["init+revert", "errors+mu", "solve call ovh", "backward", "forward", "adjoint", "residual", "refine_bwd",
         "linesearch", "accept", "reward", "newton misc"]
from learningagileflight_se3_amd import _lib
eng = Engine(variant=_lib.VARIANT_LANE, max_soc=0)
sb = S.synthetic_batch(B, seed=5)
p = sb["dnn_out"][:, :3].astype(np.float64); a = sb["dnn_out"][:, 3:6].astype(np.float64)
t = sb["dnn_out"][:, 6].astype(np.float64)
nb = (B + 63) // 64
buf = torch.zeros((max(nb, 1), 16), dtype=torch.int64, device="cuda")
eng.debug_timers(buf)
out = eng.ocp_solve(sb["ini"], sb["goal"], p, a, t)
torch.cuda.synchronize()
ms = eng.last_kernel_ms(); cnt = eng.last_counters()
eng.debug_timers(None)
R = buf.cpu().numpy().astype(np.float64)
T = R[:, :12].copy()
C = R[:, 12:16].mean(0)
print("wave-level executions per wave: newton_solve %.0f, refine %.0f, merit %.0f, ipm iterations %.0f" % tuple(C))
print("per-lane averages: sweeps %.1f, trials %.1f, iterations %.1f" % (cnt["sweeps"] / B, cnt["trials"] / B, cnt["iterations"] / B))
T[:, 2] -= T[:, 3:6].sum(1)   # slot 2 = lk_newton_solve incl. its phases 3-5
tot = T.sum(1)
it = cnt["iterations"] / B
print(f"B={B} waves={nb} kernel {ms:.1f} ms, counters {cnt}, iters/instance {it:.1f}")
print("  cycles/wave %.3e ; per iteration %.3e ; clock est %.2f GHz" % (tot.mean(), tot.mean() / it, tot.mean() / (ms * 1e6)))
sw = cnt["sweeps"] / B
for n, v in zip(names, T.mean(0)):
    print(f"   {n:12s} {100*v/tot.mean():6.2f}%   cycles/iter {v / it:.3e}  cycles/sweep {v / sw:.3e}")
