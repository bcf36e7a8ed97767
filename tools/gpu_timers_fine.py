"""Sub-phase cycles of the MFMA factorisation stage (timer build with -DLAFSE3_PT_FINE, given by LAFSE3_LIB):
slots 12..15 ([A] [C+D] [E] [F]) and the fine markers 16..23 of riccati_mfma.inc, ticks per stage."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402

eng = Engine()
for batch in (64, int(os.environ.get("BIG", "4096"))):
    sb = S.synthetic_batch(batch, seed=5)
    buf = torch.zeros((batch, 32), dtype=torch.int64, device="cuda")
    eng.debug_timers(buf)
    eng.ocp_solve(sb["ini"], sb["goal"], sb["dnn_out"][:, :3].astype(np.float64),
                  sb["dnn_out"][:, 3:6].astype(np.float64), sb["dnn_out"][:, 6].astype(np.float64))
    torch.cuda.synchronize()
    cnt = eng.last_counters()
    eng.debug_timers(None)
    T = buf.cpu().numpy().astype(np.float64)
    nst = (cnt["iterations"] + batch) * 50
    ph = T[:, 12:16].sum(0) / nst
    fine = T[:, 24:32].sum(0) / nst
    order = [("entry + row loads", ph[0]), ("W chain", fine[0]), ("M chain", fine[1]),
             ("Quu readlanes + Cholesky + vectors", ph[1]), ("LDS exchange", fine[4]), ("solve", fine[5]),
             ("F mfma", fine[6]), ("record to kbuf", ph[2]), ("flush + next row + gathers", fine[7]),
             ("border / gradient, stores, transpose", ph[3])]
    tot = sum(v for _, v in order)
    print(f"B={batch} kernel {eng.last_kernel_ms():.1f} ms; ticks per stage (normalised) {tot:.0f}")
    print("   " + "\n   ".join(f"{n:40s} {v:6.0f}  {100 * v / tot:5.1f} %" for n, v in order))
