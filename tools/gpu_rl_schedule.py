"""The reference's RL schedule end to end on the GPU: deep_learning.py:34-94 -- 100 epochs x 100
samples in groups of 10, sol_gradient on the engine (9 NLP solves per sample, one launch per group).

Two runs from the same DNN1 initialisation (random init, torch.manual_seed(0): the reference's pretrained nn_pre.pth
is not in the reference tree) and the same sample seeds:
  update="reference"  per-sample Adam steps in the reference's order (deep_learning.py:75-81)
  update="batched"    one Adam step per group on the summed loss (rl_step.train_step, bench.py's form)
Epoch 0 of the reference-order run is replayed with the CPU oracle (oracle/: TEST INFRASTRUCTURE, the checker) as
grad_fn on the same seeds and initialisation, and its rewards compared with the GPU run's at 1e-5 relative.

Writes gpurun_out/rl_schedule.json (wall time, Mean_Reward per epoch, per-epoch status histogram of the 900 solves,
the epoch-0 comparison) and gpurun_out/rl_schedule/ (Mean_Reward / Every_reward .npy, as deep_learning.py:91-93).
EPOCHS=<n> shortens the runs."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from learningagileflight_se3_amd import rl_loop, scenario  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402
from learningagileflight_se3_amd.policy_net import Network  # noqa: E402

EPOCHS = int(os.environ.get("EPOCHS", "100"))
BATCH, CORES = 100, 10
STATUS = {0: "solved", 1: "acceptable", 2: "max_iter", 3: "ls_fail", 4: "nonfinite", 5: "tiny_step", 6: "reg_fail",
          7: "device_error", 8: "resto_fail", 9: "infeasible"}
OUT = os.path.join(REPO, "gpurun_out", "rl_schedule")
os.makedirs(OUT, exist_ok=True)
dev = torch.device("cuda", 0)
eng = Engine(device=dev)


def gpu_grad(hist, rec=None):
    """rl_loop.engine_gradient with the 9 statuses of every sample counted per epoch (10 launches per epoch); rec
    (a list) collects epoch 0's launches: (samples, dnn_out, out8, rewards9)."""
    calls = [0]

    def grad_fn(samples, dnn_out):
        samples = np.asarray(samples, dtype=np.float64)
        ini = scenario.initial_state(samples[:, 0:3], samples[:, 6])
        gate12 = scenario.gate_corners(samples[:, 7], samples[:, 8])
        dn32 = np.asarray(dnn_out, dtype=np.float32)
        out8, R9, st9 = eng.sol_gradient(ini, samples[:, 3:6], gate12, dn32, want_rewards=True)
        ep = calls[0] // (BATCH // CORES)
        if rec is not None and ep == 0:
            rec.append((samples.copy(), dn32.copy(), out8.cpu().numpy(), R9.cpu().numpy()))
        calls[0] += 1
        for s in st9.cpu().numpy().reshape(-1):
            k = STATUS.get(int(s), str(int(s)))
            hist[ep][k] = hist[ep].get(k, 0) + 1
        return out8.cpu().numpy()

    return grad_fn


def oracle_grad(samples, dnn_out):
    from oracle import oracle as O   # the checker
    samples = np.asarray(samples, dtype=np.float64)
    ini = scenario.initial_state(samples[:, 0:3], samples[:, 6])
    gate12 = scenario.gate_corners(samples[:, 7], samples[:, 8])
    out8, _, _ = O.sol_gradient(ini, samples[:, 3:6], gate12, np.asarray(dnn_out, dtype=np.float32))
    return out8


def fresh(device):
    torch.manual_seed(0)
    net = Network(9, 64, 64, 7).to(device)
    return net, torch.optim.Adam(net.parameters(), lr=1e-4)   # deep_learning.py:15, 38


res = {"epochs": EPOCHS, "batch_size": BATCH, "num_cores": CORES,
       "dnn1": "random init (torch.manual_seed(0)); nn_pre.pth is not in the reference tree"}
for update in ("reference", "batched"):
    hist = [dict() for _ in range(EPOCHS)]
    net, opt = fresh(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rec0 = [] if update == "reference" else None
    r = rl_loop.run_rl(net, opt, gpu_grad(hist, rec0), epochs=EPOCHS, batch_size=BATCH, num_cores=CORES, update=update,
                       rng=np.random.default_rng(0), out_dir=os.path.join(OUT, update))
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    res[update] = {"wall_s": round(wall, 2), "samples_per_s": round(EPOCHS * BATCH / wall, 1),
                   "mean_reward": [round(float(v), 6) for v in r["mean_reward"]],
                   "status_hist_per_epoch": hist}
    if update == "reference":
        every0 = r["every_reward"][0].copy()
        launches0 = rec0
    print(update, "wall", round(wall, 1), "s; mean reward first/last", r["mean_reward"][0], r["mean_reward"][-1],
          flush=True)

# (1) the solver alone: epoch 0's 10 launches (the DNN1 outputs the GPU run fed them) through the oracle's sol_gradient
from oracle import oracle as O   # the checker
rr, ro8 = [], []
for samples, dn32, o8, R9 in launches0:
    ini = scenario.initial_state(samples[:, 0:3], samples[:, 6])
    gate12 = scenario.gate_corners(samples[:, 7], samples[:, 8])
    oo8, oR9, _ = O.sol_gradient(ini, samples[:, 3:6], gate12, dn32)
    rr.append(np.abs(R9 - oR9) / np.maximum(np.abs(oR9), 1e-12))
    # out8 on the north_star scale of the parity tests (tests/test_gpu_parity.py _grad_parity): |diff| / (1 + |ref|)
    # -- the clipped FD entries are often exactly 0 or near it, where a raw relative error means nothing
    ro8.append(np.abs(o8[:, :7] - oo8[:, :7]) / (1.0 + np.abs(oo8[:, :7])))
rr, ro8 = np.concatenate(rr), np.concatenate(ro8)
res["epoch0_solver_vs_oracle"] = {"rewards9_max_rel": float(rr.max()), "rewards9_n_over_1e-5": int((rr > 1e-5).sum()),
                                  "out8_max_diff_over_1_plus_ref": float(ro8.max()),
                                  "out8_n_over_1e-5": int((ro8 > 1e-5).sum()), "n_rewards": int(rr.size)}
print("epoch 0 solver vs oracle on the same inputs", res["epoch0_solver_vs_oracle"], flush=True)
# (2) epoch 0 of the reference-order run, replayed with the oracle as grad_fn (CPU network, same init and seeds): the
# networks differ by float32 rounding between the devices, so later samples of the epoch see slightly other inputs
net, opt = fresh(torch.device("cpu"))
t0 = time.perf_counter()
ro = rl_loop.run_rl(net, opt, oracle_grad, epochs=1, batch_size=BATCH, num_cores=CORES, update="reference",
                    rng=np.random.default_rng(0))
rel = np.abs(every0 - ro["every_reward"][0]) / np.maximum(np.abs(ro["every_reward"][0]), 1e-12)
res["epoch0_vs_oracle"] = {"max_rel_diff": float(rel.max()), "median_rel_diff": float(np.median(rel)),
                           "n_over_1e-5": int((rel > 1e-5).sum()), "n": int(rel.size),
                           "oracle_wall_s": round(time.perf_counter() - t0, 1),
                           "mean_reward_gpu": float(every0.mean()), "mean_reward_oracle": float(ro["every_reward"][0].mean())}
print("epoch 0 vs oracle", res["epoch0_vs_oracle"], flush=True)
json.dump(res, open(os.path.join(REPO, "gpurun_out", "rl_schedule.json"), "w"), indent=1)
eng.close()
