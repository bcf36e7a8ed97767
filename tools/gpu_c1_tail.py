"""configs[1] tail study: one B = 1024 ocp_solve launch of bench.py's configs[1] batch (seed 77) with the per-instance
debug record (start / end s_memrealtime at 100 MHz, iterations, sweeps, status): what sets the launch time."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine

B = int(os.environ.get("B", "1024"))
eng = Engine()
if "RESTO" in os.environ:
    eng.params.restoration = int(os.environ["RESTO"])
    eng.set_params(eng.params)
sb = S.synthetic_batch(B, seed=int(os.environ.get("SEED", "77")))
args = [torch.as_tensor(sb["ini"], device="cuda"), torch.as_tensor(sb["goal"], device="cuda"),
        torch.as_tensor(sb["dnn_out"][:, :3].astype(np.float64), device="cuda"),
        torch.as_tensor(sb["dnn_out"][:, 3:6].astype(np.float64), device="cuda"),
        torch.as_tensor(sb["dnn_out"][:, 6].astype(np.float64), device="cuda")]
eng.ocp_solve(*args); torch.cuda.synchronize()
plain = []
for _ in range(3):
    eng.ocp_solve(*args); torch.cuda.synchronize(); plain.append(eng.last_kernel_ms())
buf = torch.zeros((B, 32), dtype=torch.int64, device="cuda")
eng.debug_timers(buf)
eng.ocp_solve(*args); torch.cuda.synchronize()
ms = eng.last_kernel_ms(); cnt = eng.last_counters(); cnt.update(eng.last_resto_counters())
eng.debug_timers(None)
R = buf.cpu().numpy()
t0 = R[:, 16].min()
st = (R[:, 16] - t0) / 1e5; en = (R[:, 17] - t0) / 1e5
dur = en - st
its = R[:, 20]; sw = R[:, 21]; stt = R[:, 22]
print(f"B={B} kernel ms plain {np.round(plain, 2)}  with record {ms:.2f}; counters {cnt}")
print("instance ms pcts 50/90/99/max:", np.round(np.percentile(dur, [50, 90, 99, 100]), 2))
print("iterations pcts 50/90/99/max:", np.percentile(its, [50, 90, 99, 100]), " status counts", np.bincount(stt))
top = np.argsort(dur)[-12:][::-1]
print("longest (inst, ms, iters, sweeps, sweeps/iter, ms/iter, status):")
for i in top:
    print(f"  {int(i):5d} {dur[i]:7.2f} {int(its[i]):5d} {int(sw[i]):6d} {sw[i] / max(its[i], 1):5.2f} "
          f"{dur[i] / max(its[i], 1):.4f} {int(stt[i])}")
print("ms per iteration: median %.4f" % np.median(dur / np.maximum(its, 1)))
grid = np.linspace(0, en.max(), 21)
print("concurrency over time (20 bins):", [int(np.sum((st <= g) & (en > g))) for g in grid[:-1]])
