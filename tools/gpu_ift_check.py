"""IFT vs FD gradient modes of lafse3_sol_gradient on the same samples (diagnostic: agreement per
component, timing of both modes)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine

eng = Engine()
for B in (256, 4096):
    sb = S.synthetic_batch(B, seed=2025)
    args = (sb["ini"], sb["goal"], sb["gate12"], sb["dnn_out"])
    res = {}
    for m in (0, 1):
        eng.sol_gradient(*[a[:8] for a in args], grad_mode=m)   # warm
        torch.cuda.synchronize()
        t0 = time.time()
        o, R9, S9 = eng.sol_gradient(*args, want_rewards=True, grad_mode=m)
        torch.cuda.synchronize()
        res[m] = (o.cpu().numpy(), R9.cpu().numpy(), S9.cpu().numpy(), time.time() - t0)
    fd, ift = res[0][0], res[1][0]
    print(f"B={B}: FD {B / res[0][3]:.1f} grads/s, IFT {B / res[1][3]:.1f} grads/s")
    print("  status ok FD %.3f IFT %.3f" % (np.mean(res[0][2] <= 1), np.mean(res[1][2] <= 1)))
    print("  j, t-rule identical:", np.array_equal(fd[:, 6:], ift[:, 6:]))
    d = np.abs(fd[:, :6] - ift[:, :6])
    rel = d / (np.abs(fd[:, :6]) + 1e-4)
    for c in range(6):
        print("  comp %d: max abs %.3e  median abs %.3e  p90 rel %.3e  max rel %.3e  |fd| median %.3e" %
              (c, d[:, c].max(), np.median(d[:, c]), np.quantile(rel[:, c], 0.9), rel[:, c].max(),
               np.median(np.abs(fd[:, c]))))
    dR = np.abs(res[0][1][:, 1:7] - res[1][1][:, 1:7])
    print("  probe reward diff: median %.3e p90 %.3e p99 %.3e max %.3e" %
          (np.median(dR), np.quantile(dR, 0.9), np.quantile(dR, 0.99), dR.max()))
