"""Line-search sub-phase cycles of the IPM (timer build with -DLAFSE3_PHASE_TIMERS -DLAFSE3_PT_LS, given by
LAFSE3_LIB): slots 16..21 of ipm_kernel.hip's PT_LS marks and phase 8, cycles per IPM iteration."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402

eng = Engine()
for batch in (64, int(os.environ.get("BIG", "2048"))):
    sb = S.synthetic_batch(batch, seed=5)
    buf = torch.zeros((batch, 32), dtype=torch.int64, device="cuda")
    eng.debug_timers(buf)
    eng.ocp_solve(sb["ini"], sb["goal"], sb["dnn_out"][:, :3].astype(np.float64),
                  sb["dnn_out"][:, 3:6].astype(np.float64), sb["dnn_out"][:, 6].astype(np.float64))
    torch.cuda.synchronize()
    cnt = eng.last_counters()
    eng.debug_timers(None)
    T = buf.cpu().numpy().astype(np.float64)
    it = cnt["iterations"]
    tot_inst = T[:, 0:16].sum() + T[:, 24:29].sum()
    parts = [("direction_stats (fraction to boundary, gBD)", T[:, 24].sum()),
             ("merit at the current point (when not cached)", T[:, 25].sum()),
             ("watchdog / alpha_min setup, SOC of the previous trial", T[:, 29].sum()),
             ("trial merit: the eval_merit call alone", T[:, 26].sum()),
             ("acceptance test ls_accept (filter read)", T[:, 27].sum()),
             ("SOC / soft restoration / loop exit", T[:, 28].sum()),
             ("filter update", T[:, 8].sum())]
    ls = sum(v for _, v in parts)
    print(f"B={batch} kernel {eng.last_kernel_ms():.1f} ms, iterations {it}, trials {cnt.get('trials')}; "
          f"line search {100 * ls / tot_inst:.2f} % of instance cycles, {ls / it:.0f} cycles per iteration")
    print("   " + "\n   ".join(f"{n:62s} {v / it:8.0f} per it  {100 * v / ls:5.1f} %" for n, v in parts))
