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
    ap.add_argument("--cpu-sample", type=int, default=1024, help="samples timed on the host oracle, all cores (rank 0, N=1)")
    ap.add_argument("--cpu-sample-1core", type=int, default=48, help="samples timed on the host oracle, one core")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the untimed side measurements (configs[1] ocp_solve rate, IFT rate)")
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


def cpu_baseline(n_samples: int, n_1core: int):
    """Host oracle (oracle/ C restatement) on a bounded sample of the same workload: the -O3 / FMA timing build
    (oracle/Makefile liblafse3_oracle_fast.so), all OpenMP threads and one thread."""
    from oracle import oracle as O
    from learningagileflight_se3_amd import scenario as S
    O.lib(fast=True)
    threads = O.num_threads(fast=True)
    sb = S.synthetic_batch(n_samples, seed=4242)
    t0 = time.perf_counter()
    O.sol_gradient(sb["ini"], sb["goal"], sb["gate12"], sb["dnn_out"], fast=True)
    dt = time.perf_counter() - t0
    s1 = S.synthetic_batch(n_1core, seed=4243)
    O.set_num_threads(1, fast=True)
    t1 = time.perf_counter()
    O.sol_gradient(s1["ini"], s1["goal"], s1["gate12"], s1["dnn_out"], fast=True)
    d1 = time.perf_counter() - t1
    O.set_num_threads(threads, fast=True)
    return {"value": n_samples / dt, "unit": "solves+gradients/s", "cores": threads, "kind": "port",
            "value_1core": n_1core / d1,
            "sample": f"{n_samples} sol_gradient samples ({9 * n_samples} NLP solves) of the same seeded workload "
                      f"on the CPU oracle (C fp64, -O3 FMA build, OpenMP {threads} threads), {dt:.1f} s; "
                      f"value_1core: {n_1core} samples on one thread, {d1:.1f} s"}


STATUS = {0: "solved", 1: "acceptable", 2: "max_iter", 3: "ls_fail", 4: "nonfinite", 5: "tiny_step", 6: "reg_fail"}


def side_measurements(eng_fd, torch, dev, B):
    """Untimed side figures (rank 0): configs[1] forward-solve rate (B = 1024 fp64, full x/u/lam/cost outputs)
    and the IFT gradient mode at the bench batch (configs[2] with grad_mode = 1)."""
    from learningagileflight_se3_amd import scenario as S
    from learningagileflight_se3_amd.engine import Engine
    out = {}
    sb = S.synthetic_batch(1024, seed=77)
    args = [torch.as_tensor(sb["ini"], device=dev), torch.as_tensor(sb["goal"], device=dev),
            torch.as_tensor(sb["dnn_out"][:, :3].astype(np.float64), device=dev),
            torch.as_tensor(sb["dnn_out"][:, 3:6].astype(np.float64), device=dev),
            torch.as_tensor(sb["dnn_out"][:, 6].astype(np.float64), device=dev)]
    eng_fd.ocp_solve(*args)
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        o = eng_fd.ocp_solve(*args)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = o["status"].cpu().numpy()
    out["ocp_solve_per_s"] = round(reps * 1024 / dt, 1)
    out["ocp_solve_config"] = ("configs[1]: B = 1024 random (start, goal, static gate) OCSys.ocSolver solves, fp64, "
                               "full outputs x (51x13) u (50x4) lam (50x13) cost, HIP-event kernel "
                               f"{eng_fd.last_kernel_ms():.1f} ms; {int((st <= 1).sum())}/1024 solved/acceptable")
    sb = S.synthetic_batch(B, seed=1000)
    g = [torch.as_tensor(sb[k], device=dev) for k in ("ini", "goal", "gate12", "dnn_out")]
    eng_ift = Engine(device=dev, grad_mode=1)
    eng_ift.reserve(3 * B)
    eng_ift.sol_gradient(*g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2):
        eng_ift.sol_gradient(*g)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out["ift_grads_per_s"] = round(2 * B / dt, 1)
    out["ift_config"] = (f"sol_gradient grad_mode = 1 (IFT: 3 NLP solves + 6 KKT-sensitivity sweeps per sample), "
                         f"B = {B}, fp64; an approximation of the reference's 9-solve FD semantics (DESIGN.md §3.2b)")
    eng_ift.close()
    return out


def bench_moving(args, torch, dist, world, rank, dev):
    """configs[4]: B moving-gate episodes per GPU (main.py:44-116), 500 plant steps = 50 receding-horizon MPC
    solves each (lafse3_get_input), the trained DNN2 (nn3_1.pth), gate kinematics and the plant batched
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
    # the reference's trained DNN2 (main.py:41-42 nn3_1.pth), read raw from the checkpoint into
    # tests/golden/dnn2_nn3_1.npz by tests/golden/make_golden.py (load_nn3_1; nothing unpickled)
    w = np.load(os.path.join(REPO, "tests", "golden", "dnn2_nn3_1.npz"))
    net = Network(18, 128, 128, 7)
    net.load_state_dict({k: torch.as_tensor(w[k.replace(".", "_")]) for k in net.state_dict()})
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
    # untimed diagnostics pass: IPM iterations, get_input kernel time and statuses per MPC solve
    cnts = []
    diag = MG.run_episodes_device(eng, net, samples, noise[:, :max(args.plant_steps, 1)], steps=args.plant_steps,
                                  counters=cnts)
    st_all = diag["status"].cpu().numpy().reshape(-1)
    n_diag = max(diag["solves"], 1)
    if rank == 0:
        print(json.dumps({
            "metric": "MPC solves/sec (moving-gate receding horizon, 50-step horizon, configs[4])",
            "value": round(world * solves / dt, 3), "unit": "MPC solves/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic episodes (seeded nn_sample + gate.move noise); the reference's trained DNN2 (nn3_1.pth)",
            "config": {"workload": f"main.py moving gate: per episode {args.plant_steps} plant steps (dt 0.01; "
                                   "main.py runs 500), traversal-time fixed point on DNN2 every step, get_input "
                                   "every 10 steps",
                       "episodes_per_gpu": B, "plant_steps": args.plant_steps, "horizon": 50,
                       "parallelism": f"dp{world}"},
            "ipm_iterations_per_solve": round(sum(c["iterations"] for c in cnts) / n_diag, 2),
            "get_input_kernel_ms": round(float(np.mean([c["kernel_ms"] for c in cnts])), 3) if cnts else None,
            "status_hist": {STATUS.get(int(k), str(int(k))): int(v)
                            for k, v in zip(*np.unique(st_all[st_all >= 0], return_counts=True))}}), flush=True)
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
    iters_rec = torch.full((B, 9), -1, dtype=torch.int32, device=dev)   # per-instance IPM iterations
    eng.record_iters(iters_rec)

    def step():
        out8, _, st9 = eng.sol_gradient(ini, goal, gate, dnn, want_rewards=True)   # hot path (GPU)
        step.status = st9
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
    eng.record_iters(None)
    it_all = iters_rec.cpu().numpy().reshape(-1)
    it_all = it_all[it_all >= 0]
    st_all = step.status.cpu().numpy().reshape(-1)
    # HBM bytes per launch come from the committed rocprofv3 PMC summary (FETCH_SIZE / WRITE_SIZE passes, gfx950
    # FETCH correction per MI355X_MICROARCH.md): a profile, not this run; traffic_source names file and build
    traffic, traffic_src = None, None
    pmc = os.path.join(REPO, "profiles", "pmc_current.json")
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            traffic = pj.get("hbm_bytes_per_launch")
            traffic_src = pj.get("source")
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
            "ipm_iterations": {"p50": int(np.percentile(it_all, 50)), "p99": int(np.percentile(it_all, 99)),
                               "max": int(it_all.max()), "instances": int(it_all.size)},
            "status_hist": {STATUS.get(int(k), str(int(k))): int(v)
                            for k, v in zip(*np.unique(st_all[st_all >= 0], return_counts=True))},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 6), "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 8), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "note": "FP64 compute roof (gfx950 FP64 vector = FP64 matrix dense peak); the kernel runs "
                                 "on the FP64 VALU (no MFMA: f64 MFMA has the VALU's rate and 17-wide stage "
                                 "matrices pad to 32), limited by one wave's issue/latency per SIMD; achieved = "
                                 "IPM iterations x 740 kflop (SURVEY §8(d)) / ipm_kernel time from HIP events"},
        }
        if world == 1 and not args.no_extra:
            res.update(side_measurements(eng, torch, dev, B))
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.cpu_sample_1core)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
