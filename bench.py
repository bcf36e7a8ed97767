#!/usr/bin/env python3
"""Benchmark: MPC solves+gradients/sec (batch, 50-step horizon) on 1..8 MI355X.

One step = the deep_learning.py RL step (deep_learning.py:45-83) batched:
  1. run_quad.sol_gradient for B samples on the GPU (9 NLP solves each, quad_policy.py:94-112) —
     the hot path, inputs already resident in HBM;
  2. batched myloss (quad_nn.py:141-145): loss = sum_i Dp_i . DNN1(inputs_i), backward;
  3. all-reduce (SUM, RCCL over xGMI) of the DNN1 gradients across ranks, Adam step.
Per-GPU work is fixed (weak scaling): every rank solves its own B-sample shard (seed = 1000 + rank).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line (value = samples/s summed over ranks, samples = solve+gradient units).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "MPC solves+gradients/sec (batch, 50-step horizon) at 1/2/4/8 MI355X"
F_ITER = 740_000            # algorithmic flops per IPM iteration (N=50 Riccati sweep)
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector = FP64 matrix dense peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=4096, help="samples per GPU per step (configs[2]: 4096)")
    ap.add_argument("--cpu-sample", type=int, default=512, help="samples timed on the host oracle (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=1000, help="base seed of the synthetic batch (rank r uses seed+r)")
    ap.add_argument("--workload", choices=("rl", "moving"), default="rl",
                    help="rl: configs[2] sol_gradient RL step (default, the headline metric); "
                         "moving: configs[4] moving-gate receding horizon (main.py), --batch episodes per GPU")
    ap.add_argument("--plant-steps", type=int, default=500, help="moving: plant steps per episode (main.py:65)")
    ap.add_argument("--grad-mode", choices=("fd", "ift"), default="fd",
                    help="rl: fd = the reference's 9 solves per sample (default, the headline); ift = 3 solves + "
                         "6 KKT-sensitivity sweeps (lafse3_params.grad_mode = 1, SURVEY §8(d) 'report both')")
    return ap.parse_args()


def cpu_baseline(n_samples: int):
    """Host oracle (oracle/ C restatement, OpenMP) on a bounded sample of the same workload."""
    from oracle import oracle as O
    from learningagileflight_se3_amd import scenario as S
    sb = S.synthetic_batch(n_samples, seed=4242)
    O.lib()
    t0 = time.perf_counter()
    O.sol_gradient(sb["ini"], sb["goal"], sb["gate12"], sb["dnn_out"])
    dt = time.perf_counter() - t0
    return {"value": n_samples / dt, "unit": "solves+gradients/s", "cores": O.num_threads(), "kind": "port",
            "sample": f"{n_samples} sol_gradient samples ({9 * n_samples} NLP solves) of the same seeded "
                      f"workload on the CPU oracle (C fp64, OpenMP {O.num_threads()} threads), {dt:.1f} s"}


def bench_moving(args, torch, dist, world, rank, dev):
    """configs[4]: B moving-gate episodes per GPU (main.py:44-116), 500 plant steps = 50 receding-horizon MPC
    solves each (lafse3_get_input), DNN2 (18-128-128-7, random init), gate kinematics and the plant batched
    on the GPU (moving_gate.run_episodes_device).  value = MPC solves per second summed over ranks (weak
    scaling)."""
    from learningagileflight_se3_amd import moving_gate as MG
    from learningagileflight_se3_amd import scenario as S
    from learningagileflight_se3_amd.engine import Engine
    from learningagileflight_se3_amd.policy_net import Network
    B = args.batch
    rs = np.random.RandomState(args.seed + rank)
    samples = np.stack([S.nn_sample(rs) for _ in range(B)])
    noise = np.stack([MG.move_noise(rs, args.plant_steps) for _ in range(B)])
    torch.manual_seed(0)
    net = Network(18, 128, 128, 7)
    with torch.no_grad():   # untrained DNN2 with its time output centred on 2 s (trained: 2-4 s, quad_nn.py:56),
        net.l3.weight[6] *= 0.01   # so that quad_moving.solver's fixed point converges as with the real network
        net.l3.bias[6] = 2.0
    net = net.to(dev)
    eng = Engine(device=dev)
    eng.reserve(B)

    def episode(steps):   # episode state, gate kinematics, DNN2 and plant on the device
        return MG.run_episodes_device(eng, net, samples, noise[:, :max(steps, 1)], steps=steps)

    for _ in range(args.warmup):
        episode(MG.CTRL_EVERY)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    solves = 0
    for _ in range(args.steps):
        solves += episode(args.plant_steps)["solves"]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if rank == 0:
        print(json.dumps({
            "metric": "MPC solves/sec (moving-gate receding horizon, 50-step horizon, configs[4])",
            "value": round(world * solves / dt, 3), "unit": "MPC solves/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded nn_sample + gate.move noise); random-init DNN2, time output centred on 2 s",
            "config": {"workload": "main.py moving gate: per episode 500 plant steps (dt 0.01), traversal-time "
                                   "fixed point on DNN2 every step, get_input every 10 steps",
                       "episodes_per_gpu": B, "plant_steps": args.plant_steps, "horizon": 50,
                       "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    if args.workload == "moving":
        return bench_moving(args, torch, dist, world, rank, dev)
    from learningagileflight_se3_amd import scenario as S
    from learningagileflight_se3_amd.engine import Engine
    from learningagileflight_se3_amd.policy_net import Network
    from learningagileflight_se3_amd.rl_step import train_step

    B = args.batch
    sb = S.synthetic_batch(B, seed=args.seed + rank)
    ini = torch.as_tensor(sb["ini"], device=dev)
    goal = torch.as_tensor(sb["goal"], device=dev)
    gate = torch.as_tensor(sb["gate12"], device=dev)
    dnn = torch.as_tensor(sb["dnn_out"], device=dev)
    inputs = torch.as_tensor(sb["samples"], dtype=torch.float32, device=dev)

    torch.manual_seed(0)
    net = Network(9, 64, 64, 7).to(dev)          # DNN1 (deep_learning.py / nn_train.py architecture)
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    kw = {}
    ift = args.grad_mode == "ift"
    if ift:
        kw["grad_mode"] = 1
    solves = 3 if ift else 9                      # NLP solves per sample
    eng = Engine(device=dev, **kw)
    eng.reserve(9 * B)

    def step():
        out8 = eng.sol_gradient(ini, goal, gate, dnn)          # hot path (GPU)
        ms = eng.last_kernel_ms()
        cnt = eng.last_counters()
        train_step(net, opt, inputs, out8, world)              # myloss backward + RCCL all-reduce + Adam
        return out8, ms, cnt

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    kms, iters = [], []
    for _ in range(args.steps):
        out8, ms, cnt = step()
        kms.append(ms)
        iters.append(cnt["iterations"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    value = world * B * args.steps / dt
    kernel_ms = float(np.mean(kms))
    achieved = float(np.mean(iters)) * F_ITER / (kernel_ms * 1e-3) / 1e12
    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_current.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "solves+gradients/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded nn_sample restatement, SURVEY.md §8(d)); random-init DNN1",
            "config": {"workload": ("sol_gradient: B samples x 9 NLP solves (N=50, fp64, IPOPT-style IPM) "
                                    if not ift else
                                    "sol_gradient IFT mode: B samples x (3 NLP solves + 6 KKT-sensitivity sweeps) "
                                    "(N=50, fp64, IPOPT-style IPM) ") +
                                   "+ batched myloss backward + RCCL grad all-reduce + Adam (configs[2]/[3])",
                       "batch_per_gpu": B, "horizon": 50, "solves_per_sample": solves,
                       "grad_mode": args.grad_mode, "parallelism": f"dp{world}"},
            "solves_per_s": round(solves * value, 3),
            "kernel_ms": round(kernel_ms, 3),
            "ipm_iterations_per_solve": round(float(np.mean(iters)) / (solves * B), 2),
            "roofline": {"bound": "mfma", "achieved": round(achieved, 6), "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 8), "traffic": traffic,
                         "note": "FP64 compute roof (vector = matrix peak on gfx950); achieved = IPM iterations x "
                                 "740 kflop (SURVEY §8(d)) / ipm_kernel time from HIP events"},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_sample)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
