#!/usr/bin/env python3
"""Benchmark: MPC solves+gradients/sec (batch, 50-step horizon) on 1..8 MI355X.

One step = the deep_learning.py RL step (deep_learning.py:45-83) batched:
  1. run_quad.sol_gradient for this rank's samples on its GPU (9 NLP solves each, quad_policy.py:94-112) —
     the hot path, inputs already resident in HBM;
  2. batched myloss (quad_nn.py:141-145): loss = sum_i Dp_i . DNN1(inputs_i), backward;
  3. all-reduce (SUM, RCCL over xGMI) of the DNN1 gradients across ranks, Adam step.

Sharding (deep_learning.py:66-72's fan-out): ONE seeded batch of batch x N samples is drawn
and rank r solves its contiguous slice shard_range(batch x N, r, N).  Per-GPU work is fixed (weak scaling):
--batch defaults to 4096 at N = 1 (configs[2], the headline) and to 8192 per GPU at N > 1 (configs[3]: N = 8
is the 65 536-sample batch).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python bench.py --gpus N ...                        (spawns N rank processes itself when WORLD_SIZE is unset)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line (value = samples/s summed over ranks, samples = solve+gradient units).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "MPC solves+gradients/sec (batch, 50-step horizon) at 1/2/4/8 MI355X"
F_ITER = 740_000            # algorithmic flops per IPM iteration (N=50 Riccati sweep)
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector = FP64 matrix dense peak (spec)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=None,
                    help="samples (rl) / episodes (moving) per GPU per step; rl default 4096 at N = 1 (configs[2]), "
                         "8192 at N > 1 (configs[3]: 8 x 8192 = 65536); moving default 8192 / N (configs[4]: 8192 "
                         "episodes over the GPUs)")
    ap.add_argument("--cpu-sample", type=int, default=1024, help="samples timed on the host oracle, all cores (rank 0, N=1)")
    ap.add_argument("--cpu-sample-1core", type=int, default=48, help="samples timed on the host oracle, one core")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the untimed side measurements (configs[1] ocp_solve rate, IFT rate)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=1000, help="seed of the one synthetic batch all ranks slice")
    ap.add_argument("--workload", choices=("rl", "moving"), default="rl",
                    help="rl: configs[2]/[3] sol_gradient RL step (default, the headline metric); "
                         "moving: configs[4] moving-gate receding horizon (main.py), --batch episodes per GPU")
    ap.add_argument("--plant-steps", type=int, default=500, help="moving: plant steps per episode (main.py:65)")
    ap.add_argument("--moving-groups", type=int, default=2,
                    help="moving: episode groups per GPU, each on its own solver context / stream / host thread")
    ap.add_argument("--grad-mode", choices=("fd", "ift"), default="fd",
                    help="rl: fd = the reference's 9 solves per sample (default, the headline); ift = 3 solves + "
                         "6 KKT-sensitivity sweeps (lafse3_params.grad_mode = 1, SURVEY §8(d) 'report both')")
    ap.add_argument("--backend", choices=("auto", "nccl", "gloo"), default="auto",
                    help="torch.distributed backend for N > 1: auto = nccl (RCCL) on GPUs, gloo with --engine stub")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal of the N-rank harness on a box with fewer GPUs: rank r uses GPU r mod device "
                         "count (gloo only; the line is marked, its rate is not a scaling measurement)")
    ap.add_argument("--eager-train", action="store_true",
                    help="rl: issue the DNN1 step's kernels one by one instead of replaying its HIP graphs")
    ap.add_argument("--dump-out8", default=None, metavar="PREFIX",
                    help="test hook: every rank saves its shard's out8 of the last timed step to PREFIX.rank<r>.npy")
    ap.add_argument("--engine", choices=("hip", "stub"), default="hip",
                    help="hip: liblafse3 on the GPU (every reported number); stub: a CPU stand-in for the solver that "
                         "exercises the launcher, sharding and collective on hosts without a GPU (tests only)")
    a = ap.parse_args(argv)
    a.batch_default = a.batch is None
    if a.batch is None:
        if a.workload == "moving":   # configs[4]: 8192 episodes in all, split over the GPUs
            a.batch = max(1, 8192 // a.gpus)
        else:                         # configs[2] at N = 1, configs[3]'s 8192 per GPU at N > 1
            a.batch = 4096 if a.gpus == 1 else 8192
    return a


# ---------------------------------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv) -> int:
    """--gpus N > 1 without a launcher: start N rank processes of this script (one per GPU, before this process
    touches any GPU) with the torch.distributed env contract, wait for all, return the first failing exit code."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


# ---------------------------------------------------------------------------------------------- baselines
def cpu_baseline(n_samples: int, n_1core: int):
    """Host oracle (oracle/ C restatement) on bounded samples of the same workloads: the -O3 / FMA timing build
    (oracle/Makefile liblafse3_oracle_fast.so), all OpenMP threads and one thread.
      value / value_1core      configs[2] unit: sol_gradient samples (9 NLP solves each) per second
      configs1_solves_per_s*   configs[1] unit: OCSys.ocSolver forward solves per second (1 core / all cores)
      configs0                 configs[0]: the single seed-0 solve on one core (wall, iterations, final error)"""
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

    def fwd_args(sb):
        a = sb["dnn_out"][:, 3:6].astype(np.float64)
        q = np.stack([O.rd2quat(ai) for ai in a])
        return (sb["ini"], sb["goal"], sb["dnn_out"][:, :3].astype(np.float64), q,
                sb["dnn_out"][:, 6].astype(np.float64))

    # configs[1]: forward solves, same generator as the GPU side figure (seed 77), one core then all cores
    c1 = S.synthetic_batch(1024, seed=77)
    args1 = fwd_args(c1)
    n1 = 96
    t2 = time.perf_counter()
    O.solve(*(a[:n1] for a in args1), fast=True)
    d2 = time.perf_counter() - t2
    O.set_num_threads(threads, fast=True)
    t3 = time.perf_counter()
    O.solve(*args1, fast=True)
    d3 = time.perf_counter() - t3
    # configs[0]: one instance (seed 0), one core, with the final optimality error
    O.set_num_threads(1, fast=True)
    c0 = S.synthetic_batch(1, seed=0)
    fe = np.zeros((1, 4))
    O.debug_final_err(fe, fast=True)
    t4 = time.perf_counter()
    r0 = O.solve(*fwd_args(c0), fast=True)
    d4 = time.perf_counter() - t4
    O.debug_final_err(None, fast=True)
    O.set_num_threads(threads, fast=True)
    return {"value": n_samples / dt, "unit": "solves+gradients/s", "cores": threads, "kind": "port",
            "value_1core": n_1core / d1,
            "configs1_solves_per_s": 1024 / d3, "configs1_solves_per_s_1core": n1 / d2,
            "configs0": {"wall_s_1core": d4, "iterations": int(r0["iters"][0]), "status": int(r0["status"][0]),
                         "cost": float(r0["cost"][0]), "overall_nlp_error": float(fe[0, 0]),
                         "dual_inf": float(fe[0, 1]), "primal_inf": float(fe[0, 2]), "compl_inf": float(fe[0, 3])},
            "sample": f"{n_samples} sol_gradient samples ({9 * n_samples} NLP solves) of the same seeded workload "
                      f"on the CPU oracle (C fp64, -O3 FMA build, OpenMP {threads} threads), {dt:.1f} s; "
                      f"value_1core: {n_1core} samples on one thread, {d1:.1f} s; configs[1]: {n1} forward solves on "
                      f"one thread ({d2:.1f} s) and the 1024-solve batch on {threads} threads ({d3:.1f} s); "
                      f"configs[0]: the seed-0 single solve on one thread"}


STATUS = {0: "solved", 1: "acceptable", 2: "max_iter", 3: "ls_fail", 4: "nonfinite", 5: "tiny_step", 6: "reg_fail",
          7: "device_error", 8: "resto_fail", 9: "infeasible"}


def side_measurements(eng_fd, torch, dev, B, eng_b):
    """Untimed side figures (rank 0): configs[1] forward-solve rate (B = 1024 fp64, full x/u/lam/cost outputs)
    and the IFT gradient mode at the bench batch (configs[2] with grad_mode = 1).  ``eng_b``: the second
    default-parameter context (the caller's: it serves the moving-gate side figure next)."""
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
    # serving form of the same workload: consecutive B = 1024 batches on two contexts and two streams, so that a
    # launch's tail (its few longest instances) overlaps the next launch's start; results checked
    # bit-equal to the single-launch ones
    from learningagileflight_se3_amd.engine import QueueStream
    qs = [QueueStream(dev), QueueStream(dev)]   # two hardware queues: launches of the two contexts overlap
    streams = [q.stream for q in qs]
    pairs = [(eng_fd, streams[0]), (eng_b, streams[1])]
    for e, s in pairs:
        with torch.cuda.stream(s):
            e.ocp_solve(*args)
    torch.cuda.synchronize()
    K = 6
    t0 = time.perf_counter()
    outs = []
    for i in range(K):
        e, s = pairs[i % 2]
        with torch.cuda.stream(s):
            outs.append(e.ocp_solve(*args))
    torch.cuda.synchronize()
    dt2 = time.perf_counter() - t0
    same = all(torch.equal(q["cost"], o["cost"]) and torch.equal(q["x"], o["x"]) for q in outs)
    for q in qs:
        q.close()
    out["ocp_solve_per_s_2streams"] = round(K * 1024 / dt2, 1)
    out["ocp_solve_2streams_config"] = (f"{K} consecutive configs[1] batches (B = 1024 each) alternating over two "
                                        "solver contexts on two streams with hardware queues of their own (lafse3_stream_create; two launches in flight); outputs "
                                        f"bit-equal to the single launch: {same}")
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


def committed_profile():
    """The committed rocprofv3 PMC summary (profiles/pmc_current.json) when it was taken on this tree's kernel
    sources (its csrc_sha equals build.source_hash()); otherwise (None, reason)."""
    from learningagileflight_se3_amd.build import source_hash
    path = os.path.join(REPO, "profiles", "pmc_current.json")
    if not os.path.exists(path):
        return None, "no committed profile"
    pj = json.load(open(path))
    here = source_hash()
    if pj.get("csrc_sha") != here:
        return None, f"stale: profile of csrc {pj.get('csrc_sha')}, tree {here}"
    return pj, pj.get("source")


# ---------------------------------------------------------------------------------------------- engines
class StubEngine:
    """CPU stand-in for the solver (``--engine stub``): deterministic out8 from the inputs, no solve.  Lets the
    launcher / sharding / all-reduce harness run on hosts without a GPU (tests/test_bench_harness.py); every
    number it yields is meaningless and the JSON line says so."""

    def __init__(self, torch):
        self.torch = torch
        self.device = torch.device("cpu")

    def reserve(self, n):
        pass

    def record_iters(self, buf=None):
        pass

    def sol_gradient(self, ini, goal, gate, dnn, want_rewards=False, verify=True):
        t = self.torch
        out8 = t.zeros((ini.shape[0], 8), dtype=t.float64)
        out8[:, :7] = 1e-2 * t.tanh(dnn.double() + 0.1 * ini[:, :7] + 0.01 * gate[:, :7] + 0.1 * goal.sum(1, keepdim=True))
        out8[:, 7] = ini[:, 0] - goal[:, 0]
        R9 = out8[:, 7:8].expand(-1, 9).contiguous()
        S9 = t.zeros((ini.shape[0], 9), dtype=t.int32)
        return out8, R9, S9

    # moving workload (configs[4]): traversal time and the first MPC control, deterministic in their inputs
    def traversal_time(self, state, final_point, gp, velo, w, net):
        t = self.torch
        return 1.0 + 0.1 * t.tanh(state[:, 0] - final_point[:, 0] + 0.1 * gp[:, :, 0].mean(1) + 0.01 * velo[:, 0])

    def get_input(self, ini, goal, dnn_out, u_last=None):
        t = self.torch
        u = 1.22 + 0.1 * t.tanh(ini[:, :4] + goal.sum(1, keepdim=True) + dnn_out[:, :4].double())
        if u_last is not None:
            u = u + 0.01 * u_last
        return u, t.zeros((ini.shape[0],), dtype=t.int32)

    def last_kernel_ms(self):
        return 0.0

    def last_counters(self):
        return {"iterations": 0, "sweeps": 0, "trials": 0}

    def last_resto_counters(self):
        return {"resto_entries": 0, "resto_returns": 0}


def moving_episodes(torch, dev, samples, noise, plant_steps, groups, net, stub, steps=1, warmup=1, barrier=None,
                    engines=None):
    """Run the moving-gate episodes (main.py:44-116) `steps` times after `warmup` short runs: the episodes in `groups`
    contiguous groups, each with its own solver context, HIP stream and host thread (one group's get_input launch
    tail overlaps another group's work).  Returns (MPC solves per run, seconds of the timed runs, engine of group 0)."""
    from learningagileflight_se3_amd import moving_gate as MG
    from learningagileflight_se3_amd.rl_step import shard_range
    own = engines is None   # engines passed in stay open (the caller's)
    if stub:
        engs, G = [StubEngine(torch)], 1
    elif engines is not None:
        engs, G = list(engines), len(engines)
    else:
        from learningagileflight_se3_amd.engine import Engine
        G = max(1, int(groups))
        engs = [Engine(device=dev) for _ in range(G)]
    n_loc = len(samples)
    bounds = [shard_range(n_loc, g, G) for g in range(G)]
    for e, (a, b) in zip(engs, bounds):
        e.reserve(b - a)
    # one hardware queue per group (lafse3_stream_create): two ordinary torch streams may share one of HIP's
    # pooled queues, and the groups then run back to back (profiles/r05_moving_trace.log: 42.5 k instead of 62 k)
    if stub:
        qs, streams = [], [None] * G
    else:
        from learningagileflight_se3_amd.engine import QueueStream
        qs = [QueueStream(dev) for _ in range(G)]
        streams = [q.stream for q in qs]

    def sync():
        if not stub:
            torch.cuda.synchronize()

    def episode(st):   # episode state, gate kinematics, DNN2 and plant on the device
        if G == 1:
            return MG.run_episodes_device(engs[0], net, samples, noise[:, :max(st, 1)], steps=st)
        res, errs = [None] * G, []

        def run(g):
            a, b = bounds[g]
            try:
                with torch.cuda.stream(streams[g]):
                    res[g] = MG.run_episodes_device(engs[g], net, samples[a:b], noise[a:b, :max(st, 1)], steps=st)
            except BaseException as ex:   # re-raised on the main thread
                errs.append(ex)
        ths = [threading.Thread(target=run, args=(g,)) for g in range(G)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errs:
            raise errs[0]
        return {"solves": sum(r["solves"] for r in res)}

    for _ in range(warmup):
        episode(MG.CTRL_EVERY)
    sync()
    if barrier:
        barrier()
    t0 = time.perf_counter()
    solves = 0
    for _ in range(steps):
        solves += episode(plant_steps)["solves"]
    sync()
    if barrier:
        barrier()
    dt = time.perf_counter() - t0
    for q in qs:
        q.close()
    if own:
        for e in engs[1:]:
            e.close()
    return solves // max(steps, 1), dt, engs[0], G


def moving_inputs(torch, dev, n_total, lo, hi, plant_steps, seed):
    """The seeded episodes (nn_sample + gate.move noise) of rows [lo, hi) of n_total, and the reference's trained DNN2."""
    from learningagileflight_se3_amd import moving_gate as MG
    from learningagileflight_se3_amd import scenario as S
    from learningagileflight_se3_amd.policy_net import Network
    rs = np.random.RandomState(seed)
    samples = np.stack([S.nn_sample(rs) for _ in range(n_total)])[lo:hi]
    noise = np.stack([MG.move_noise(rs, plant_steps) for _ in range(n_total)])[lo:hi]
    # the reference's trained DNN2 (main.py:41-42 nn3_1.pth), read raw from the checkpoint into
    # tests/golden/dnn2_nn3_1.npz by tests/golden/make_golden.py (load_nn3_1; nothing unpickled)
    w = np.load(os.path.join(REPO, "tests", "golden", "dnn2_nn3_1.npz"))
    net = Network(18, 128, 128, 7)
    net.load_state_dict({k: torch.as_tensor(w[k.replace(".", "_")]) for k in net.state_dict()})
    return samples, noise, net.to(dev)


def moving_side_figure(torch, dev, episodes=8192, plant_steps=500, groups=2, seed=1000, engines=None):
    """Untimed side figure of the default bench line (rank 0, N = 1): configs[4] -- 8 192 moving-gate episodes x
    500 plant steps (50 MPC solves each) once, all of them on this GPU."""
    samples, noise, net = moving_inputs(torch, dev, episodes, 0, episodes, plant_steps, seed)
    solves, dt, eng, G = moving_episodes(torch, dev, samples, noise, plant_steps, groups, net, stub=False,
                                         engines=engines)
    if engines is None:
        eng.close()
    return {"moving_mpc_solves_per_s": round(solves / dt, 1),
            "moving_config": (f"configs[4]: {episodes} moving-gate episodes x {plant_steps} plant steps (main.py:44-116, "
                              f"trained DNN2), {solves} get_input MPC solves in {dt:.2f} s, one run, {G} episode groups "
                              "(bench.py --workload moving for the full line)")}


def bench_moving(args, torch, dist, world, rank, dev):
    """configs[4]: moving-gate episodes (main.py:44-116), 500 plant steps = 50 receding-horizon MPC solves each
    (lafse3_get_input), the trained DNN2 (nn3_1.pth), gate kinematics and the plant batched on the GPU
    (moving_gate.run_episodes_device).  --batch episodes per GPU (default 8192 / N: configs[4]'s 8192 over the GPUs,
    strong scaling); one seeded set of batch x N episodes, rank r takes its contiguous slice.  value = MPC solves per
    second summed over ranks (max-rank time).  ``--engine stub`` replaces the solver with bench.py's CPU stand-in
    (harness tests: the N-rank barrier / MAX-reduce path on gloo)."""
    from learningagileflight_se3_amd import moving_gate as MG
    from learningagileflight_se3_amd.rl_step import shard_range
    stub = args.engine == "stub"
    strong = bool(getattr(args, "batch_default", False))
    # default: configs[4]'s 8192 episodes in all, shard_range over the ranks (uneven when N does not divide 8192);
    # an explicit --batch is per GPU (weak scaling)
    n_total = 8192 if strong else args.batch * world
    lo, hi = shard_range(n_total, rank, world)
    B = hi - lo
    samples, noise, net = moving_inputs(torch, dev, n_total, lo, hi, args.plant_steps, args.seed)
    barrier = dist.barrier if world > 1 else None
    solves, dt, eng, G = moving_episodes(torch, dev, samples, noise, args.plant_steps, args.moving_groups, net, stub,
                                         steps=args.steps, warmup=args.warmup, barrier=barrier)
    solves *= args.steps
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        n = torch.tensor([float(solves)], dtype=torch.float64, device=dev)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        solves_all = int(n.item())
    else:
        solves_all = solves
    # untimed diagnostics pass: IPM iterations, get_input kernel time and statuses per MPC solve
    cnts = []
    diag = MG.run_episodes_device(eng, net, samples, noise[:, :max(args.plant_steps, 1)], steps=args.plant_steps,
                                  counters=cnts)
    st_all = diag["status"].cpu().numpy().reshape(-1)
    n_diag = max(diag["solves"], 1)
    if rank == 0:
        print(json.dumps({
            "metric": "MPC solves/sec (moving-gate receding horizon, 50-step horizon, configs[4])",
            "value": round(solves_all / dt, 3), "unit": "MPC solves/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f64",
            "data": ("STUB ENGINE (harness test, no solve: every rate here is meaningless)" if stub else
                     ("REHEARSAL: ranks share GPUs (--share-gpu), not a scaling measurement; "
                      if getattr(args, "share_gpu", False) else "") +
                     "synthetic episodes (seeded nn_sample + gate.move noise); the reference's trained DNN2 (nn3_1.pth)"),
            "config": {"workload": f"main.py moving gate: per episode {args.plant_steps} plant steps (dt 0.01; "
                                   "main.py runs 500), traversal-time fixed point on DNN2 every step, get_input "
                                   "every 10 steps",
                       "episodes_per_gpu": B, "global_episodes": n_total, "plant_steps": args.plant_steps,
                       "horizon": 50, "parallelism": f"dp{world}", "backend": args.backend if world > 1 else None,
                       "engine": "stub" if stub else "hip",
                       "groups_per_gpu": G, "grouping": "contiguous episode groups, one solver context + HIP stream + "
                                                        "host thread each (launch tails overlap)"},
            "ipm_iterations_per_solve": round(sum(c["iterations"] for c in cnts) / n_diag, 2),
            "get_input_kernel_ms": round(float(np.mean([c["kernel_ms"] for c in cnts])), 3) if cnts else None,
            "status_hist": {STATUS.get(int(k), str(int(k))): int(v)
                            for k, v in zip(*np.unique(st_all[st_all >= 0], return_counts=True))},
            "restoration": {"entries": int(sum(c["resto_entries"] for c in cnts)),
                            "returns": int(sum(c["resto_returns"] for c in cnts)),
                            "scope": "diagnostics pass (all MPC solves of the B x plant_steps episodes)"}}), file=RESULT_OUT, flush=True)


# the result line's stream: the process's stdout as it was at start.  A rank process points its fd 1 at stderr
# before torch.distributed starts, so that library banners written to stdout (Gloo's "[Gloo] Rank r is connected to
# ..." lines, from every rank) cannot precede or interleave with the JSON line: stdout carries that line alone
RESULT_OUT = sys.stdout


def _stdout_for_result_only():
    global RESULT_OUT
    sys.stdout.flush()
    RESULT_OUT = os.fdopen(os.dup(1), "w", buffering=1)
    os.dup2(2, 1)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, argv))          # before anything touches a GPU
    if int(env_world or 1) > 1:
        _stdout_for_result_only()
    world = int(env_world or 1)
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    stub = args.engine == "stub"
    if stub:
        dev = torch.device("cpu")
    else:
        if args.share_gpu:
            if args.backend != "gloo":
                print("bench.py: --share-gpu needs --backend gloo (RCCL takes one rank per GPU)", file=sys.stderr)
                sys.exit(2)
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    backend = args.backend if args.backend != "auto" else ("gloo" if stub else "nccl")
    args.backend = backend
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    try:
        if args.workload == "moving":
            bench_rl_or_moving = bench_moving
        else:
            bench_rl_or_moving = bench_rl
        bench_rl_or_moving(args, torch, dist, world, rank, dev)
    finally:
        if world > 1 and dist.is_initialized():
            dist.destroy_process_group()


def bench_rl(args, torch, dist, world, rank, dev):
    from learningagileflight_se3_amd import scenario as S
    from learningagileflight_se3_amd.policy_net import Network
    from learningagileflight_se3_amd.rl_step import GraphedTrainStep, shard_range, train_step

    stub = args.engine == "stub"
    B = args.batch
    lo, hi = shard_range(B * world, rank, world)
    sb = S.synthetic_batch(B * world, seed=args.seed)             # one seeded batch; this rank's contiguous slice
    ini = torch.as_tensor(sb["ini"][lo:hi], device=dev)
    goal = torch.as_tensor(sb["goal"][lo:hi], device=dev)
    gate = torch.as_tensor(sb["gate12"][lo:hi], device=dev)
    dnn = torch.as_tensor(sb["dnn_out"][lo:hi], device=dev)
    inputs = torch.as_tensor(sb["samples"][lo:hi], dtype=torch.float32, device=dev)
    Bl = hi - lo

    torch.manual_seed(0)
    net = Network(9, 64, 64, 7).to(dev)          # DNN1 (deep_learning.py / nn_train.py architecture)
    graphed = not stub and not args.eager_train
    # capturable Adam in both the graphed and the eager (--eager-train) step, so that the two modes train DNN1 with
    # the same optimiser arithmetic (the stub engine runs on the CPU, where capturable does not apply)
    opt = torch.optim.Adam(net.parameters(), lr=1e-4, **({"capturable": True} if not stub else {}))
    ift = args.grad_mode == "ift"
    solves = 3 if ift else 9                      # NLP solves per sample
    if stub:
        eng = StubEngine(torch)
    else:
        from learningagileflight_se3_amd.engine import Engine
        eng = Engine(device=dev, **({"grad_mode": 1} if ift else {}))
    eng.reserve(9 * Bl)
    iters_rec = None if stub else torch.full((Bl, 9), -1, dtype=torch.int32, device=dev)
    eng.record_iters(iters_rec)

    seg = {"launch": [], "wait_kernel": [], "train_step_host": []}

    def step():
        t0 = time.perf_counter()
        # hot path (GPU); last_counters below waits for it and raises on a lost probe task (device error word)
        out8, _, st9 = eng.sol_gradient(ini, goal, gate, dnn, want_rewards=True, verify=False)
        t1 = time.perf_counter()
        step.status = st9
        ms = eng.last_kernel_ms()
        cnt = eng.last_counters()
        step.resto = eng.last_resto_counters()
        t2 = time.perf_counter()
        if graphed:
            train_graph(out8)                                  # the same step replayed from its HIP graphs
        else:
            train_step(net, opt, inputs, out8, world)          # myloss backward + RCCL all-reduce + Adam
        t3 = time.perf_counter()
        seg["launch"].append(t1 - t0)
        seg["wait_kernel"].append(t2 - t1)
        seg["train_step_host"].append(t3 - t2)
        return out8, ms, cnt

    def sync():
        if not stub:
            torch.cuda.synchronize()

    # the DNN1 step's library kernels (GEMM, Adam) load and tune on their first calls (~380 ms, then ~15 ms, then
    # ~2 ms per step): warm them on a throwaway replica of the same shapes, so that the solver warmup steps below
    # leave the timed steps at steady state without touching the replica that is trained
    if not stub:
        torch.manual_seed(1)
        net_w = Network(9, 64, 64, 7).to(dev)
        opt_w = torch.optim.Adam(net_w.parameters(), lr=1e-4)
        for _ in range(4):
            train_step(net_w, opt_w, inputs, torch.zeros((Bl, 8), dtype=torch.float64, device=dev), 1)
        del net_w, opt_w
    train_graph = GraphedTrainStep(net, opt, inputs, (Bl, 8), world) if graphed else None
    for _ in range(args.warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    kms, iters = [], []
    for _ in range(args.steps):
        out8, ms, cnt = step()
        kms.append(ms)
        iters.append(cnt["iterations"])
    sync()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if args.dump_out8:
        np.save(f"{args.dump_out8}.rank{rank}.npy", out8.detach().cpu().numpy())
    # replicas must hold identical DNN1 parameters after the all-reduced steps
    csum = torch.cat([p.detach().reshape(-1).double() for p in net.parameters()]).sum()
    iters_t = torch.tensor([float(np.sum(iters)), float(Bl)], dtype=torch.float64, device=dev)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        allc = [torch.zeros_like(csum) for _ in range(world)]
        dist.all_gather(allc, csum)
        consistent = all(bool(c == allc[0]) for c in allc)
        dist.all_reduce(iters_t, op=dist.ReduceOp.SUM)
    else:
        consistent = True
    if rank != 0:
        return

    value = float(iters_t[1].item()) * args.steps / dt          # samples solved by all ranks / max-rank time
    kernel_ms = float(np.mean(kms))
    iters_mean = float(np.mean(iters))
    achieved = iters_mean * F_ITER / (kernel_ms * 1e-3) / 1e12 if kernel_ms > 0 else 0.0
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
        "data": ("STUB ENGINE (harness test, no solve: every rate here is meaningless)" if stub else
                 ("REHEARSAL: ranks share GPUs (--share-gpu), not a scaling measurement; " if args.share_gpu else "") +
                 "synthetic (seeded nn_sample restatement, SURVEY.md §8(d)); random-init DNN1"),
        "config": {"workload": ("sol_gradient: B samples x 9 NLP solves (N=50, fp64, IPOPT-style IPM) "
                                if not ift else
                                "sol_gradient IFT mode: B samples x (3 NLP solves + 6 KKT-sensitivity sweeps) "
                                "(N=50, fp64, IPOPT-style IPM) ") +
                               "+ batched myloss backward + RCCL grad all-reduce + Adam (" +
                               ("configs[2])" if world == 1 and B == 4096 else "configs[3] layout)"),
                   "batch_per_gpu": B, "global_batch": B * world, "seed": args.seed,
                   "sharding": "one seeded batch, rank r solves contiguous shard_range(global_batch, r, N)",
                   "horizon": 50, "solves_per_sample": solves, "grad_mode": args.grad_mode,
                   "parallelism": f"dp{world}", "backend": (args.backend if world > 1 else None),
                   "engine": args.engine, **({"shared_gpus": torch.cuda.device_count()} if args.share_gpu else {}),
                   "dnn1_step": ("HIP graphs: forward + myloss + backward, eager all-reduce, Adam (capturable)"
                                 if graphed else "eager, Adam (capturable)" if not stub else "eager"),
                   # the solver's decision variables: the same seeded dnn_out every step (open loop); DNN1 trains on
                   # the resulting gradients beside it but its output is not fed back (deep_learning.py:55-56, 67
                   # feeds model(inputs)); no warm start or cache: every step solves all 9 x B NLPs cold
                   "decision_vars": "fixed synthetic (SURVEY §8(d)): p_tra, a_tra, t drawn once per seed, not net(inputs)"},
        "dnn1_replicas_consistent": consistent,
        "host_ms_per_step": {k: round(1e3 * float(np.mean(v[-args.steps:])), 3) for k, v in seg.items()},
        "dnn1_param_checksum": float(csum.item()),
    }
    if not stub:
        eng.record_iters(None)
        it_all = iters_rec.cpu().numpy().reshape(-1)
        it_all = it_all[it_all >= 0]
        st_all = step.status.cpu().numpy().reshape(-1)
        pj, src = committed_profile()
        rf = {"bound": "fp64-valu-latency", "achieved": round(achieved, 6), "peak": FP64_PEAK_TFLOPS,
              "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 8),
              "traffic": pj.get("hbm_bytes_per_launch") if pj else None, "traffic_source": src,
              "valu_insts_per_alg_fma": pj.get("valu_insts_per_alg_fma") if pj else None,
              "note": "FP64 compute roof (gfx950 FP64 vector = FP64 matrix dense peak); the Riccati factorisation "
                      "stage runs on the f64 matrix cores (v_mfma_f64_16x16x4_f64, 7 per stage), the rest of the "
                      "IPM on the FP64 VALU; bound by one wave's dependent instruction chain per SIMD (issue + "
                      "LDS/VALU/MFMA latency); achieved "
                      "= IPM iterations x 740 kflop (SURVEY §8(d)) / ipm_kernel time from HIP events on the launch "
                      "stream; traffic = FETCH_SIZE x2 + WRITE_SIZE per launch from the committed PMC profile of "
                      "this tree's kernel sources (null when stale)"}
        res.update({
            "solves_per_s": round(solves * value, 3),
            "kernel_ms": round(kernel_ms, 3),
            "ipm_iterations_per_solve": round(float(iters_t[0].item()) / args.steps / (solves * B * world), 2),
            "ipm_iterations": {"p50": int(np.percentile(it_all, 50)), "p99": int(np.percentile(it_all, 99)),
                               "max": int(it_all.max()), "instances": int(it_all.size)},
            "status_hist": {STATUS.get(int(k), str(int(k))): int(v)
                            for k, v in zip(*np.unique(st_all[st_all >= 0], return_counts=True))},
            # IPOPT restoration phase (lafse3_last_resto_counters) in the last timed step's launch: entries, and
            # returns to the original problem (the rest ended their solve with status 2/4/6/8/9, see status_hist)
            "restoration": {"entries": step.resto["resto_entries"], "returns": step.resto["resto_returns"],
                            "scope": "last timed step's launch"},
            "roofline": rf,
        })
        if world == 1 and not args.no_extra:
            from learningagileflight_se3_amd.engine import Engine
            eng_b = Engine(device=dev)
            try:
                res.update(side_measurements(eng, torch, dev, B, eng_b))
            finally:
                eng_b.close()
            res.update(moving_side_figure(torch, dev))
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.cpu_sample_1core)
    print(json.dumps(res), file=RESULT_OUT, flush=True)


if __name__ == "__main__":
    main()
