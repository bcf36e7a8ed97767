"""Launch schedule of one sol_gradient launch (bench batch, B samples x 9 solves) from the timers build's
placement record (start/end s_memrealtime at 100 MHz, HW_ID, XCC_ID per instance) -> gpurun_out/sched.npz.
Slot occupancy = sum of instance durations / (slots x launch span); tail = time from the first idle slot
that never refills to the launch end."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LAFSE3_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                 "learningagileflight_se3_amd", "liblafse3_timers.so"))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine

B = int(os.environ.get("B", "4096"))
sb = S.synthetic_batch(B, seed=1000)
eng = Engine()
buf = torch.zeros((B * 9, 32), dtype=torch.int64, device="cuda")
eng.debug_timers(buf)
eng.sol_gradient(sb["ini"], sb["goal"], sb["gate12"], sb["dnn_out"])
torch.cuda.synchronize()
ms = eng.last_kernel_ms()
eng.debug_timers(None)
T = buf.cpu().numpy()
st, en = T[:, 16].astype(np.float64), T[:, 17].astype(np.float64)
span = (en.max() - st.min()) / 1e5
busy = (en - st).sum() / 1e5
slot = T[:, 18] * 16 + T[:, 19]                    # HW_ID x XCC (unique enough per slot)
nslot = len(np.unique(slot))
print(f"kernel {ms:.1f} ms, span {span:.1f} ms, slots {nslot}, occupancy {busy / (nslot * span):.3f}", flush=True)
t = np.linspace(st.min(), en.max(), 200)
active = np.array([((st <= x) & (en > x)).sum() for x in t])
print("active instances over the launch (20 points):", active[::10].tolist(), flush=True)
dur = (en - st) / 1e5
print("instance duration ms p50/p99/max:", np.percentile(dur, [50, 99, 100]).round(2).tolist(),
      "iters corr", np.corrcoef(dur, T[:, 20])[0, 1])
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/sched.npz", T=T, ms=ms)
