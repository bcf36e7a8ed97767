"""Time both kernel variants (lane / wave) on the same batch and compare their results."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S, _lib
from learningagileflight_se3_amd.engine import Engine

B = int(os.environ.get("B", "2048"))
sb = S.synthetic_batch(B, seed=5)
p = sb["dnn_out"][:, :3].astype(np.float64); a = sb["dnn_out"][:, 3:6].astype(np.float64)
t = sb["dnn_out"][:, 6].astype(np.float64)
res = {}
for name, var in (("lane", _lib.VARIANT_LANE), ("wave", _lib.VARIANT_WAVE)):
    if name == "wave" and os.environ.get("SKIP_WAVE"):
        continue
    eng = Engine(variant=var, max_soc=0)
    out = eng.ocp_solve(sb["ini"][:64], sb["goal"][:64], p[:64], a[:64], t[:64])   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = eng.ocp_solve(sb["ini"], sb["goal"], p, a, t)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms = eng.last_kernel_ms(); cnt = eng.last_counters()
    res[name] = {k: v.cpu().numpy() for k, v in out.items()}
    print(f"[{name}] ocp_solve B={B}: kernel {ms:.1f} ms (wall {1e3*dt:.1f}), {B/(ms*1e-3):.0f} solves/s, "
          f"counters {cnt}, status hist {np.bincount(res[name]['status'], minlength=7).tolist()}", flush=True)
    if os.environ.get("GRAD"):
        G = int(os.environ.get("GRAD"))
        out8 = eng.sol_gradient(sb["ini"][:G], sb["goal"][:G], sb["gate12"][:G], sb["dnn_out"][:G])
        torch.cuda.synchronize()
        ms = eng.last_kernel_ms()
        print(f"[{name}] sol_gradient B={G}: kernel {ms:.1f} ms -> {G/(ms*1e-3):.0f} grads/s", flush=True)
if "wave" in res:
    L, Wv = res["lane"], res["wave"]
    same = L["iters"] == Wv["iters"]
    print("same iteration count:", same.mean())
    for k in ("x", "u", "cost"):
        d = np.abs(L[k][same] - Wv[k][same]) / (1 + np.abs(Wv[k][same]))
        print(k, "max rel diff (same iters):", d.max())
    print("cost rel diff all:", np.max(np.abs(L["cost"] - Wv["cost"]) / np.abs(Wv["cost"])))
