"""Where does a bench-sized sol_gradient launch lose time?  Per-instance start/end (s_memrealtime,
100 MHz) and HW_ID/XCC_ID from the debug record: slot utilisation, instance-duration tail, concurrency."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from learningagileflight_se3_amd import scenario as S
from learningagileflight_se3_amd.engine import Engine

B = int(os.environ.get("B", "4096"))
eng = Engine(**({"grad_mode": int(os.environ["GRAD_MODE"])} if "GRAD_MODE" in os.environ else {}))
if "RESTO" in os.environ:   # restoration phase on / off (lafse3_params.restoration; builds before 0.5 ignore it)
    eng.params.restoration = int(os.environ["RESTO"])
    eng.set_params(eng.params)
sb = S.synthetic_batch(B, seed=1000)
args = [torch.as_tensor(sb[k], device="cuda") for k in ("ini", "goal", "gate12", "dnn_out")]
eng.sol_gradient(*args); torch.cuda.synchronize()              # warm
NS = 3 if os.environ.get("GRAD_MODE") == "1" else 9   # NLP instances per sample (IFT: nominal + 2 t-probes)
buf = torch.zeros((NS * B, 32), dtype=torch.int64, device="cuda")
eng.debug_timers(buf)
eng.sol_gradient(*args); torch.cuda.synchronize()
ms = eng.last_kernel_ms(); cnt = eng.last_counters()
try:
    cnt.update(eng.last_resto_counters())
except Exception:   # a build without lafse3_last_resto_counters
    pass
eng.debug_timers(None)
R = buf.cpu().numpy()
t0 = R[:, 16].min()
st = (R[:, 16] - t0) / 1e5; en = (R[:, 17] - t0) / 1e5        # ms
dur = en - st
hw = R[:, 18].astype(np.int64); xcc = R[:, 19].astype(np.int64) & 0xF
simd = (hw >> 4) & 3; cu = (hw >> 8) & 0xF; sh = (hw >> 12) & 1; se = (hw >> 13) & 7
slot = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
span = en.max()
print(f"kernel {ms:.1f} ms (events), span {span:.1f} ms (realtime); instances {len(R)}; iters {cnt}")
print("distinct xcc %d se %d cu %d simd %d slots %d" % (len(set(xcc)), len(set(se)), len(set(cu)), len(set(simd)), len(set(slot))))
busy = np.bincount(slot, weights=dur)
nz = busy[busy > 0]
print(f"slot busy ms: mean {nz.mean():.1f} min {nz.min():.1f} max {nz.max():.1f}; utilisation {nz.sum() / (len(nz) * span):.3f}")
print("instance ms pcts 50/90/99/99.9/max:", np.round(np.percentile(dur, [50, 90, 99, 99.9, 100]), 2), " mean", round(dur.mean(), 3))
srt = np.sort(dur)[::-1]
cs = np.cumsum(srt) / dur.sum()
for f in (0.001, 0.01, 0.05):
    k = max(1, int(f * len(dur))); print(f"  top {f*100:.1f}% instances = {cs[k-1]*100:.1f}% of instance time")
# concurrency over time
grid = np.linspace(0, span, 41)
conc = [(np.sum((st <= g) & (en > g))) for g in grid[:-1]]
print("concurrency over time (40 bins):", conc)
last = np.argsort(en)[-10:]
its = R[:, 20]; sw = R[:, 21]; stt = R[:, 22]
print("iterations pcts 50/90/99/99.9/max:", np.percentile(its, [50, 90, 99, 99.9, 100]), " status counts", np.bincount(stt))
top = np.argsort(dur)[-12:]
print("longest instances: (inst, ms, iters, sweeps, status)", [(int(i), round(dur[i], 1), int(its[i]), int(sw[i]), int(stt[i])) for i in top])
print("longest instances' start ms and kind (instance id // B: 0 nominal, >= 1 probe):",
      [(round(st[i], 1), int(i) // B) for i in top])
print("ms per iteration: median %.3f  for longest %.3f" % (np.median(dur / np.maximum(its, 1)), np.median(dur[top] / np.maximum(its[top], 1))))
print("last 10 finishers: start/end/dur ms", [(round(st[i], 1), round(en[i], 1), round(dur[i], 1)) for i in last])
if os.environ.get("OUT"):
    np.savez(os.environ["OUT"], timers=R, kernel_ms=ms)
