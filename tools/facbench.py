"""Hot-sweep throughput of a diagnostic build (-DLAFSE3_FACBENCH=R: R factorisation + refinement solves per instance
at the initial point, no IPM iterations) given by LAFSE3_LIB: kernel time and sweeps for B instances.

    LAFSE3_LIB=.../liblafse3_VF1.so python3 tools/facbench.py 4096
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
sb = S.synthetic_batch(B, seed=1000)
eng = Engine()
args = [torch.as_tensor(sb["ini"]).cuda(), torch.as_tensor(sb["goal"]).cuda(),
        torch.as_tensor(sb["dnn_out"][:, :3].astype(np.float64)).cuda(),
        torch.as_tensor(sb["dnn_out"][:, 3:6].astype(np.float64)).cuda(),
        torch.as_tensor(sb["dnn_out"][:, 6].astype(np.float64)).cuda()]
eng.reserve(B)
ms = []
for r in range(4):
    eng.ocp_solve(*args, want=())
    torch.cuda.synchronize()
    ms.append(eng.last_kernel_ms())
c = eng.last_counters()
print(f"{os.path.basename(os.environ.get('LAFSE3_LIB', 'liblafse3.so'))} B={B} kernel_ms {ms[1:]} counters {c} "
      f"us/sweep/instance {1e3 * min(ms[1:]) / max(c['sweeps'], 1) * 1:.3f}", flush=True)
