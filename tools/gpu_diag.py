"""First-light diagnostics: GPU engine vs CPU oracle on a small seeded batch (prints, no asserts)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine
from oracle import oracle as O

B = int(os.environ.get("B", "32"))
sb = S.synthetic_batch(B, seed=3)
eng = Engine()
p = sb["dnn_out"][:, :3].astype(np.float64)
a = sb["dnn_out"][:, 3:6].astype(np.float64)
t = sb["dnn_out"][:, 6].astype(np.float64)
g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "policy.npz"))
xr = g["x_calls"].reshape(-1, 51, 13)
R = eng.reward(xr, np.repeat(g["goal"], 9, 0), np.repeat(g["gate12"], 9, 0)).cpu().numpy()
print("reward vs reference max err", np.max(np.abs(R - g["rewards"].reshape(-1))), flush=True)

torch.cuda.synchronize()
t0 = time.time()
out = eng.ocp_solve(sb["ini"], sb["goal"], p, a, t)
torch.cuda.synchronize()
print("gpu solve wall", time.time() - t0, "kernel ms", eng.last_kernel_ms(), eng.last_counters(), flush=True)
q = np.stack([O.rd2quat(ai) for ai in a])
ref = O.solve(sb["ini"], sb["goal"], p, q, t)
st = out["status"].cpu().numpy()
print("status gpu", np.unique(st, return_counts=True), "oracle", np.unique(ref["status"], return_counts=True))
it = out["iters"].cpu().numpy()
print("iters gpu", it[:16], "\niters orc", ref["iters"][:16])
for k in ("x", "u", "lam", "cost"):
    d = np.abs(out[k].cpu().numpy() - ref[k])
    print(k, "max abs err", d.max(), "median", np.median(d))
t0 = time.time()
o8, R9, S9 = eng.sol_gradient(sb["ini"], sb["goal"], sb["gate12"], sb["dnn_out"], want_rewards=True)
torch.cuda.synchronize()
print("gpu grad wall", time.time() - t0, "kernel ms", eng.last_kernel_ms(), eng.last_counters(), flush=True)
ro8, rR, rS = O.sol_gradient(sb["ini"], sb["goal"], sb["gate12"], sb["dnn_out"])
print("grad status", np.unique(S9.cpu().numpy(), return_counts=True))
dR = np.abs(R9.cpu().numpy() - rR)
print("rewards max err", dR.max(), "median", np.median(dR))
d8 = np.abs(o8.cpu().numpy() - ro8)
print("out8 max err", d8.max(axis=0))
