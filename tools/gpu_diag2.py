"""Bisect GPU vs oracle: compare iterates after max_iter = 0,1,2,3,5,10."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S, _lib
from learningagileflight_se3_amd.engine import Engine
from oracle import oracle as O

B = 8
sb = S.synthetic_batch(B, seed=3)
p = sb["dnn_out"][:, :3].astype(np.float64)
a = sb["dnn_out"][:, 3:6].astype(np.float64)
t = sb["dnn_out"][:, 6].astype(np.float64)
q = np.stack([O.rd2quat(ai) for ai in a])
for lsq in (0, 1):
    for mi in (0, 1, 2, 3, 5, 10):
        eng = Engine(max_iter=mi, lsq_mult_init=lsq)
        out = eng.ocp_solve(sb["ini"], sb["goal"], p, a, t)
        ref = O.solve(sb["ini"], sb["goal"], p, q, t, params=O.default_params(max_iter=mi, lsq_mult_init=lsq))
        msg = [f"lsq={lsq} max_iter={mi}"]
        for k in ("x", "u", "lam", "cost"):
            d = np.abs(out[k].cpu().numpy() - ref[k])
            msg.append(f"{k}:{d.max():.3e}")
        msg.append("it gpu " + str(out["iters"].cpu().numpy().tolist()) + " orc " + str(ref["iters"].tolist()))
        print("  ".join(msg), flush=True)
        if mi == 1:
            d = np.abs(out["x"].cpu().numpy() - ref["x"])[0]
            print("   x err per stage (inst 0):", np.round(d.max(axis=1)[:12], 8))
            print("   x err per comp (inst 0):", np.round(d.max(axis=0), 8))
            d = np.abs(out["u"].cpu().numpy() - ref["u"])[0]
            print("   u err per stage (inst 0):", np.round(d.max(axis=1)[:12], 8))
            d = np.abs(out["lam"].cpu().numpy() - ref["lam"])[0]
            print("   lam err per stage:", np.round(d.max(axis=1)[:12], 6), np.round(d.max(axis=0), 6))
