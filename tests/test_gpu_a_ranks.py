"""GPU test of bench.py's N-rank path on the one-GPU box.

bench.py --gpus 2 --backend gloo --share-gpu spawns two rank processes (RANK / WORLD_SIZE / MASTER_* before any GPU
use), each solving its contiguous shard of one seeded batch on the GPU through the C ABI and training DNN1 with the
HIP-graph step (rl_step.GraphedTrainStep: graph replay, eager gloo all-reduce of the gradients, graph replay of
Adam) -- the batched form of deep_learning.py:66-83, whose fan-out is deep_learning.py:66-72.  Checked: exit code 0,
stdout is the JSON line alone, the DNN1 replicas agree, and the two shards' out8 equal a one-rank run over the same
128 samples bit for bit (a solve does not depend on its batch position or on the other rank).

This module runs first among the GPU tests (file name order): the pytest process must not have initialised the GPU
before it starts processes (a GPU-initialised process must not exec another program on this pool).
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, timeout=600):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    p = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env, timeout=timeout,
                       cwd=REPO)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = p.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout[-2000:]
    return json.loads(lines[0])


def test_two_spawned_ranks_share_gpu_equal_one_rank():
    assert not torch.cuda.is_initialized(), "run this module before any test that initialises the GPU"
    common = ["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-extra"]
    with tempfile.TemporaryDirectory() as d:
        two = _run(["--gpus", "2", "--backend", "gloo", "--share-gpu", "--batch", "64",
                    "--dump-out8", os.path.join(d, "two")] + common)
        one = _run(["--gpus", "1", "--batch", "128", "--dump-out8", os.path.join(d, "one")] + common)
        o2 = np.concatenate([np.load(os.path.join(d, f"two.rank{r}.npy")) for r in range(2)])
        o1 = np.load(os.path.join(d, "one.rank0.npy"))
    assert two["n_gpus"] == 2 and two["config"]["parallelism"] == "dp2" and two["config"]["backend"] == "gloo"
    assert two["config"]["global_batch"] == 128 and two["data"].startswith("REHEARSAL")
    assert two["config"]["dnn1_step"].startswith("HIP graphs")
    assert two["dnn1_replicas_consistent"] is True
    hist = two["status_hist"]   # rank 0's shard: 64 samples x 9 solves, every one solved / acceptable
    assert set(hist) <= {"solved", "acceptable"} and sum(hist.values()) == 64 * 9, hist
    assert o2.shape == (128, 8) and np.all(np.isfinite(o2))
    assert np.array_equal(o2, o1)
    # the all-reduced gradient is the full-batch gradient: the trained replicas match the one-rank DNN1 up to the
    # fp32 summation order of the reduction
    a, b = two["dnn1_param_checksum"], one["dnn1_param_checksum"]
    assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), (a, b)
