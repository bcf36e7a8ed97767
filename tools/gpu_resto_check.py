"""sol_gradient on the bench batch's (synthetic_batch(4096, seed 1000)) samples that hold a line-search failure
in the pre-restoration solver (tests/golden/make_resto.py BENCH_SAMPLES): per-solve statuses, iterations and
rewards of the build in LAFSE3_LIB (default the in-tree one) -> gpurun_out/resto_check_<tag>.npz."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402
from make_resto import BENCH_SAMPLES  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "new"
sb = S.synthetic_batch(4096, seed=1000)
idx = np.array(BENCH_SAMPLES)
args = [sb[k][idx] for k in ("ini", "goal", "gate12", "dnn_out")]
eng = Engine()
it = torch.full((len(idx), 9), -1, dtype=torch.int32, device="cuda")
eng.record_iters(it)
o8, R9, S9 = eng.sol_gradient(*args, want_rewards=True)
torch.cuda.synchronize()
eng.record_iters(None)
np.savez(os.path.join(REPO, "gpurun_out", f"resto_check_{tag}.npz"), out8=o8.cpu().numpy(), R9=R9.cpu().numpy(),
         S9=S9.cpu().numpy(), iters=it.cpu().numpy())
print(tag, "statuses", np.unique(S9.cpu().numpy(), return_counts=True), flush=True)
