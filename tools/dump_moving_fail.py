"""MPC instances of the moving-gate loop whose solve ended in a line-search failure (status 3) with the build given
by LAFSE3_LIB: B episodes x 500 plant steps on the device loop (trained DNN2), the failing get_input instances'
inputs saved to gpurun_out/moving_fail_inputs.npz (tests/golden/resto.npz is made from it).

    LAFSE3_LIB=.../liblafse3_old.so python3 tools/dump_moving_fail.py [B] [n_keep]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from learningagileflight_se3_amd import moving_gate as MG  # noqa: E402
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402
from learningagileflight_se3_amd.policy_net import Network  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
keep = int(sys.argv[2]) if len(sys.argv) > 2 else 64
rs = np.random.RandomState(1000)
samples = np.stack([S.nn_sample(rs) for _ in range(B)])
noise = np.stack([MG.move_noise(rs, 500) for _ in range(B)])
w = np.load(os.path.join(REPO, "tests", "golden", "dnn2_nn3_1.npz"))
net = Network(18, 128, 128, 7)
net.load_state_dict({k: torch.as_tensor(w[k.replace(".", "_")]) for k in net.state_dict()})
net = net.cuda()
eng = Engine()
eng.reserve(B)
cap = []
MG.run_episodes_device(eng, net, samples, noise, steps=500, capture=cap)
rows = {k: [] for k in ("ini", "goal", "dnn_out", "u_last", "step", "episode")}
for c in cap:
    st = c["status"].cpu().numpy()
    for e in np.nonzero(st == 3)[0]:
        for k in ("ini", "goal", "dnn_out", "u_last"):
            rows[k].append(c[k][e].cpu().numpy())
        rows["step"].append(c["step"])
        rows["episode"].append(e)
n = len(rows["step"])
idx = np.sort(np.random.default_rng(0).choice(n, min(keep, n), replace=False))
out = {k: np.array(v)[idx] for k, v in rows.items()}
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "moving_fail_inputs.npz"), **out)
print(f"{n} failing MPC solves of {len(cap) * B}; kept {len(idx)}", flush=True)
