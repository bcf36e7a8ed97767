"""bench.py's distributed harness on CPU: the --gpus N launcher, contiguous sharding of one seeded batch and the
DNN1 gradient all-reduce, with the solver replaced by bench.py's CPU stub (``--engine stub``, gloo backend).

The reference fans its samples out to processes (deep_learning.py:66-72) and applies the MPC gradients to one
DNN1; here the N-rank run must (i) launch N ranks itself when no launcher set WORLD_SIZE, (ii) keep the replicas
identical, and (iii) equal a one-rank run over the same global batch (the all-reduced gradient is the full-batch
gradient).  A WORLD_SIZE that disagrees with --gpus must be refused."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["OMP_NUM_THREADS"] = "1"
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env, timeout=timeout,
                          cwd=REPO)


def _line(p):
    assert p.returncode == 0, p.stderr[-3000:]
    # stdout carries the JSON line alone (library banners such as Gloo's go to stderr: bench.py RESULT_OUT)
    lines = p.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout
    return json.loads(lines[0])


def test_two_rank_launcher_matches_one_rank():
    two = _line(_run(["--gpus", "2", "--engine", "stub", "--batch", "16", "--steps", "2", "--warmup", "1"]))
    assert two["n_gpus"] == 2
    assert two["config"]["global_batch"] == 32 and two["config"]["batch_per_gpu"] == 16
    assert two["config"]["parallelism"] == "dp2" and two["config"]["backend"] == "gloo"   # auto resolved
    assert two["dnn1_replicas_consistent"] is True
    assert two["data"].startswith("STUB ENGINE")
    one = _line(_run(["--gpus", "1", "--engine", "stub", "--batch", "32", "--steps", "2", "--warmup", "1"]))
    assert one["n_gpus"] == 1 and one["config"]["global_batch"] == 32
    # same seeded global batch, gradients summed across ranks = full-batch gradient (fp32 summation order aside)
    a, b = two["dnn1_param_checksum"], one["dnn1_param_checksum"]
    assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), (a, b)


def test_world_size_mismatch_is_refused():
    p = _run(["--gpus", "2", "--engine", "stub", "--batch", "4", "--steps", "1", "--warmup", "0"],
             env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE=1 but --gpus 2" in p.stderr


def test_share_gpu_needs_gloo():
    """--share-gpu (the N-rank rehearsal on fewer GPUs) is refused with RCCL, before any GPU is touched."""
    p = _run(["--gpus", "1", "--share-gpu", "--batch", "4", "--steps", "1", "--warmup", "0"])
    assert p.returncode == 2
    assert "--share-gpu needs --backend gloo" in p.stderr


def test_default_batch_per_config():
    sys.path.insert(0, REPO)
    import bench
    assert bench.parse(["--gpus", "1"]).batch == 4096          # configs[2]
    assert bench.parse(["--gpus", "8"]).batch == 8192          # configs[3]: 8 x 8192 = 65536
    assert bench.parse(["--gpus", "2", "--batch", "5"]).batch == 5
    # configs[4]: 8192 moving-gate episodes in all, over the GPUs
    assert bench.parse(["--gpus", "1", "--workload", "moving"]).batch == 8192
    assert bench.parse(["--gpus", "8", "--workload", "moving"]).batch == 1024


def test_moving_two_rank_launcher_matches_one_rank():
    """--workload moving on N ranks (VERDICT r3 missing #3): the launcher, the contiguous episode shards of one
    seeded set, the barrier-bracketed timed region and the MAX-over-ranks time, with the solver replaced by the CPU
    stub; the solve count of two ranks over 2 x 4 episodes equals one rank over 8."""
    args = ["--workload", "moving", "--engine", "stub", "--plant-steps", "20", "--steps", "1", "--warmup", "1"]
    two = _line(_run(["--gpus", "2", "--batch", "4"] + args))
    assert two["n_gpus"] == 2 and two["config"]["parallelism"] == "dp2" and two["config"]["backend"] == "gloo"
    assert two["config"]["global_episodes"] == 8 and two["data"].startswith("STUB ENGINE")
    one = _line(_run(["--gpus", "1", "--batch", "8"] + args))
    assert one["config"]["global_episodes"] == 8
    per_run = 8 * 2   # 8 episodes, get_input every 10 of 20 plant steps
    assert two["value"] * two["ms_per_step"] / 1e3 == pytest.approx(per_run, rel=1e-3)
    assert one["value"] * one["ms_per_step"] / 1e3 == pytest.approx(per_run, rel=1e-3)
    assert two["status_hist"] == {"solved": 4 * 2} and one["status_hist"] == {"solved": 8 * 2}   # rank 0's episodes
