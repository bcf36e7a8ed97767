"""Per-iteration trace comparison GPU vs oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine
from oracle import oracle as O

B, IT = 4, 6
sb = S.synthetic_batch(B, seed=3)
p = sb["dnn_out"][:, :3].astype(np.float64)
a = sb["dnn_out"][:, 3:6].astype(np.float64)
t = sb["dnn_out"][:, 6].astype(np.float64)
q = np.stack([O.rd2quat(ai) for ai in a])
eng = Engine(max_iter=IT)
buf = torch.zeros((B, IT, 16), dtype=torch.float64, device="cuda")
eng.debug_trace(buf, IT)
out = eng.ocp_solve(sb["ini"], sb["goal"], p, a, t)
torch.cuda.synchronize()
tg = buf.cpu().numpy()
to = np.zeros((B, IT, 16))
O.debug_trace(to, IT)
ref = O.solve(sb["ini"], sb["goal"], p, q, t, params=O.default_params(max_iter=IT))
names = ["mu", "E0", "th", "ph", "gBD", "amax", "az", "alpha", "dw", "acc", "nf", "sw", "r0", "r1", "r2", "nref"]
np.set_printoptions(linewidth=200, precision=6)
for b in range(2):
    print("instance", b)
    for it in range(IT):
        g, o = tg[b, it], to[b, it]
        print(f" it {it:2d} GPU " + " ".join(f"{n}={v:.6e}" for n, v in zip(names, g)))
        print(f"       ORC " + " ".join(f"{n}={v:.6e}" for n, v in zip(names, o)))
