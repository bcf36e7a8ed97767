"""Device solves of the 64 configs[4] restoration-fixture instances (tests/golden/resto.npz) with their iteration
counts, statuses, trajectories and restoration counters -> gpurun_out/resto_moving_gpu.npz (compared with the oracle
on the host)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from learningagileflight_se3_amd.engine import Engine  # noqa: E402

g = dict(np.load(os.path.join(REPO, "tests", "golden", "resto.npz")))
eng = Engine()
B = len(g["moving_ini"])
it = torch.full((B,), -1, dtype=torch.int32, device="cuda")
eng.record_iters(it)
u0, x, st = eng.get_input(g["moving_ini"], g["moving_goal"], g["moving_dnn_out"], u_last=g["moving_u_last"], want_x=True)
rc = eng.last_resto_counters()
eng.record_iters(None)
tr = torch.zeros((B, 400, 16), dtype=torch.float64, device="cuda")
eng.debug_trace(tr, 400)
eng.get_input(g["moving_ini"], g["moving_goal"], g["moving_dnn_out"], u_last=g["moving_u_last"])
torch.cuda.synchronize()
eng.debug_trace(None)
np.savez(os.path.join(REPO, "gpurun_out", "resto_moving_gpu.npz"), x=x.cpu().numpy(), u0=u0.cpu().numpy(),
         status=st.cpu().numpy(), iters=it.cpu().numpy(), trace=tr.cpu().numpy())
print("moving fixture:", rc, np.unique(st.cpu().numpy(), return_counts=True), flush=True)
