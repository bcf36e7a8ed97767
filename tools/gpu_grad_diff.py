"""Per-sample sol_gradient differences GPU vs oracle (diagnostic for the parity tolerances)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine
from oracle import oracle as O

eng = Engine()
for seed, B in ((2025, 24), (7, 64)):
    sb = S.synthetic_batch(B, seed=seed)
    args = (sb["ini"], sb["goal"], sb["gate12"], sb["dnn_out"])
    out8, R9, S9 = eng.sol_gradient(*args, want_rewards=True)
    torch.cuda.synchronize()
    out8, R9 = out8.cpu().numpy(), R9.cpu().numpy()
    r8, rR, rS = O.sol_gradient(*args)
    d8 = np.abs(out8 - r8)[:, :7] / (1 + np.abs(r8[:, :7]))
    dR = np.abs(R9 - rR).max(1)
    print(f"seed {seed} B {B}: reward-close(1e-8) {np.mean(dR < 1e-8):.3f}  d8rel max {d8.max():.3e} "
          f"frac<1e-6 {np.mean(d8.max(1) < 1e-6):.3f} frac<1e-5 {np.mean(d8.max(1) < 1e-5):.3f}  d8[:,7] max {np.abs(out8-r8)[:,7].max():.3e}")
    print("  per-sample d8rel:", np.array2string(d8.max(1), precision=1))
    print("  per-sample dR   :", np.array2string(dR, precision=1))
