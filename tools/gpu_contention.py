"""Per-wave speed of the solver vs. how many waves share the chip / a CU: ocp_solve launches of B instances
(persistent grid = min(B, slots)) with the placement record; prints ms per IPM iteration per wave and the number of
waves per CU, to separate per-CU sharing (LDS, vector memory) from chip-wide contention."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402

eng = Engine()
sb = S.synthetic_batch(2048, seed=5)
p = sb["dnn_out"][:, :3].astype(np.float64)
a = sb["dnn_out"][:, 3:6].astype(np.float64)
t = sb["dnn_out"][:, 6].astype(np.float64)
eng.ocp_solve(sb["ini"][:64], sb["goal"][:64], p[:64], a[:64], t[:64])
for B in (64, 128, 256, 512, 768, 1024, 2048):
    buf = torch.zeros((B, 32), dtype=torch.int64, device="cuda")
    eng.debug_timers(buf)
    eng.ocp_solve(sb["ini"][:B], sb["goal"][:B], p[:B], a[:B], t[:B])
    torch.cuda.synchronize()
    ms = eng.last_kernel_ms()
    eng.debug_timers(None)
    R = buf.cpu().numpy()
    dur = (R[:, 17] - R[:, 16]) / 1e5   # ms (100 MHz)
    its = np.maximum(R[:, 20], 1)
    hw = R[:, 18].astype(np.int64)
    xcc = R[:, 19].astype(np.int64) & 0xF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 7
    sh = (hw >> 12) & 1
    cuid = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    # waves per CU over the instances' lifetimes: the count of instances started on the same CU in the first round
    first = R[:, 16] <= np.sort(R[:, 16])[min(len(R), 1024) - 1]
    per_cu = np.bincount(cuid[first])
    per_cu = per_cu[per_cu > 0]
    print(f"B {B:5d}: kernel {ms:7.1f} ms; ms/iteration per wave median {np.median(dur / its):.4f} "
          f"mean {np.mean(dur / its):.4f}; CUs used {len(per_cu)}, waves/CU mean {per_cu.mean():.2f} "
          f"max {per_cu.max()}", flush=True)
