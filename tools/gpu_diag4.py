"""Dump the Newton step at iteration IT (before refinement) from GPU and oracle, locate differences."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine
from oracle import oracle as O

B = 2
sb = S.synthetic_batch(4, seed=3)
p = sb["dnn_out"][:B, :3].astype(np.float64)
a = sb["dnn_out"][:B, 3:6].astype(np.float64)
t = sb["dnn_out"][:B, 6].astype(np.float64)
q = np.stack([O.rd2quat(ai) for ai in a])
ini, goal = sb["ini"][:B], sb["goal"][:B]
np.set_printoptions(linewidth=220, precision=3)
for IT in (1, 2):
    for after in (0, 1):
        eng = Engine(max_iter=IT + 1)
        buf = torch.zeros((B, 1513), dtype=torch.float64, device="cuda")
        eng.debug_dump(buf, IT, bool(after))
        eng.ocp_solve(ini, goal, p, a, t)
        torch.cuda.synchronize()
        g = buf.cpu().numpy()
        o = np.zeros((B, 1513))
        O.debug_dump(o, IT, bool(after))
        O.solve(ini, goal, p, q, t, params=O.default_params(max_iter=IT + 1))
        O.debug_dump(None, -1)
        dx = np.abs(g[:, :663] - o[:, :663]).reshape(B, 51, 13)
        du = np.abs(g[:, 663:863] - o[:, 663:863]).reshape(B, 50, 4)
        dl = np.abs(g[:, 863:] - o[:, 863:]).reshape(B, 50, 13)
        sx = np.abs(o[:, :663]).reshape(B, 51, 13).max()
        print(f"IT={IT} after_refine={after} |dx|max={sx:.3e}  err dx {dx.max():.3e} du {du.max():.3e} lam {dl.max():.3e}")
        print("  dx err by stage", dx[0].max(1)[::5])
        print("  dx err by comp ", dx[0].max(0))
        print("  du err by stage", du[0].max(1)[::5])
        print("  lam err by comp", dl[0].max(0))
