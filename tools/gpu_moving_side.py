"""The default bench line's configs[4] side figure (bench.moving_side_figure) repeated in one process: runs with fresh
solver contexts (created and closed per run, as bench.py does) and runs reusing one pair of contexts, to tell an
allocation effect (workspace freed and re-allocated) from in-process state (profiles/r04_moving_side_contexts.log; that
run's library also logged each context's workspace addresses)."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402

dev = torch.device("cuda", 0)


def run(tag, engines=None):
    t0 = time.perf_counter()
    r = bench.moving_side_figure(torch, dev, episodes=8192, plant_steps=500, groups=2, engines=engines)
    print(f"{tag}: {r['moving_mpc_solves_per_s']} MPC solves/s ({time.perf_counter() - t0:.1f} s incl. setup)",
          flush=True)


run("fresh 0")
run("fresh 1")
kept = [Engine(device=dev) for _ in range(2)]
run("kept 0", kept)
run("kept 1", kept)
run("fresh 2")
run("kept 2", kept)
for e in kept:
    e.close()
