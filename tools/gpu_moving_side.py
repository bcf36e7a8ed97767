"""The default bench line's configs[4] side figure (bench.moving_side_figure) twice in a fresh process, then once
after a sol_gradient launch of the bench batch: separates first-run effects from the in-process state of the FD
bench that precedes it in bench.py."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

dev = torch.device("cuda", 0)
for i in range(2):
    t0 = time.perf_counter()
    r = bench.moving_side_figure(torch, dev, episodes=8192, plant_steps=500, groups=2)
    print(f"run {i}: {r['moving_mpc_solves_per_s']} MPC solves/s ({time.perf_counter() - t0:.1f} s incl. setup)", flush=True)
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402
eng = Engine(device=dev)
sb = S.synthetic_batch(4096, seed=1000)
g = [torch.as_tensor(sb[k], device=dev) for k in ("ini", "goal", "gate12", "dnn_out")]
eng.sol_gradient(*g)
torch.cuda.synchronize()
r = bench.moving_side_figure(torch, dev, episodes=8192, plant_steps=500, groups=2)
print(f"after an FD launch (engine alive): {r['moving_mpc_solves_per_s']}", flush=True)
