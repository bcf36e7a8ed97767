"""configs[4] side figure (bench.moving_side_figure) run several times in ONE process, for a rocprofv3 kernel trace of
a fast and a slow run.  Runs are named on the command line ("fresh" = contexts created and closed by
the run, as bench.py does; "kept" = one pair of contexts reused); a marker kernel (a 7-element int64 cumsum, nothing else launches one) is enqueued between runs so
that tools/trace_moving.py can cut the trace into runs.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mtrace -o run -- \
        python3 tools/gpu_moving_trace.py fresh fresh
    python3 tools/trace_moving.py gpurun_out/mtrace/run_kernel_trace.csv
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402

dev = torch.device("cuda", 0)
EPISODES = int(os.environ.get("EPISODES", "8192"))


def marker(i):
    torch.cuda.synchronize()
    torch.arange(7, device=dev, dtype=torch.int64).add_(i).cumsum(0)
    torch.cuda.synchronize()


kept = None
for i, what in enumerate(sys.argv[1:] or ["fresh", "fresh"]):
    marker(i)
    t0 = time.perf_counter()
    if what == "kept" and kept is None:
        kept = [Engine(device=dev) for _ in range(2)]
    r = bench.moving_side_figure(torch, dev, episodes=EPISODES, plant_steps=500, groups=2,
                                 engines=kept if what == "kept" else None)
    print(f"run {i} {what}: {r['moving_mpc_solves_per_s']} MPC solves/s ({time.perf_counter() - t0:.1f} s incl. setup)",
          flush=True)
marker(99)
if kept:
    for e in kept:
        e.close()
