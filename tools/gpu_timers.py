"""Per-phase cycle breakdown of the IPM kernel (debug timers)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the phase timers exist only in the diagnostic build (python -m learningagileflight_se3_amd.build --timers)
os.environ.setdefault("LAFSE3_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                 "learningagileflight_se3_amd", "liblafse3_timers.so"))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine

B = int(os.environ.get("B", "64"))
sb = S.synthetic_batch(B, seed=3)
eng = Engine()
p = sb["dnn_out"][:, :3].astype(np.float64); a = sb["dnn_out"][:, 3:6].astype(np.float64)
t = sb["dnn_out"][:, 6].astype(np.float64)
names = ["init", "errors", "table", "backward", "forward", "adjoint", "residual", "refine_bwd", "linesearch",
         "accept", "reward", "other"]   # slot 11 also takes the refinement backups / adds
for label, batch in (("small", 64), ("full", int(os.environ.get("BIG", "2048")))):
    sbb = S.synthetic_batch(batch, seed=5)
    pp = sbb["dnn_out"][:, :3].astype(np.float64); aa = sbb["dnn_out"][:, 3:6].astype(np.float64)
    tt = sbb["dnn_out"][:, 6].astype(np.float64)
    buf = torch.zeros((batch, 32), dtype=torch.int64, device="cuda")
    eng.debug_timers(buf)
    out = eng.ocp_solve(sbb["ini"], sbb["goal"], pp, aa, tt)
    torch.cuda.synchronize()
    ms = eng.last_kernel_ms(); cnt = eng.last_counters()
    eng.debug_timers(None)
    T = buf.cpu().numpy().astype(np.float64)[:, :12]
    tot = T.sum(1)
    print(f"[{label}] B={batch} kernel {ms:.1f} ms, counters {cnt}")
    print("  mean cycles/instance %.3e ; per iteration %.3e ; per sweep %.3e" %
          (tot.mean(), tot.sum() / cnt["iterations"], tot.sum() / cnt["sweeps"]))
    for n, v in zip(names, T.sum(0) / T.sum()):
        print(f"   {n:12s} {100*v:6.2f}%   cycles/sweep {T.sum(0)[names.index(n)] / cnt['sweeps']:.3e}")
    X = buf.cpu().numpy().astype(np.float64)[:, 12:16].sum(0) / (cnt["iterations"] + batch) / 50
    W = buf.cpu().numpy().astype(np.float64)[:, 24:32].sum(0)
    nst = (cnt["iterations"] + batch) * 50
    print("   factorisation vector-memory waits: probe0 %.0f  probe1 %.0f ticks per stage (probe cost %.0f per probe);"
          " %.2f %% of all instance cycles (probe cost removed)" %
          (W[0] / nst, W[1] / nst, W[7] / max(1.0, nst * ((W[0] > 0) + (W[1] > 0))),
           100.0 * max(0.0, W[0] + W[1] - W[7]) / T.sum()))
    print("   backward_full per stage (ticks): [A] %.0f  [C+D] %.0f  [E] %.0f  [F] %.0f" % tuple(X)); print("   slot5 %.0f  slot10 %.0f per stage (diagnostic splits)" % tuple(T.sum(0)[[5, 10]] / (cnt["iterations"] + batch) / 50))
