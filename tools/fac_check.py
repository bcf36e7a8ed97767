"""Factorisation A/B inside one solve (diagnostic build liblafse3_FC.so, -DLAFSE3_FAC_CHECK): at every factorisation
of every IPM iteration both sweeps run on the same Newton system -- the VALU stage (riccati.inc backward_full) and
the MFMA stage (riccati_mfma.inc backward_mfma) -- and the MFMA sweep's factor record, P_k and p_k are compared
with the VALU sweep's; the solve continues on the VALU sweep's outputs.  Prints, over B instances, the worst
relative difference per array (max |MFMA - VALU| / max |VALU| over a sweep) and the inertia-test disagreements.

    NAME=FC tools/build_variant.sh -DLAFSE3_FAC_CHECK
    LAFSE3_LIB=.../liblafse3_FC.so python tools/fac_check.py [B]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LAFSE3_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                 "learningagileflight_se3_amd", "liblafse3_FC.so"))
from learningagileflight_se3_amd import scenario as S  # noqa: E402
from learningagileflight_se3_amd.engine import Engine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
sb = S.synthetic_batch(B, seed=1000)
eng = Engine()
buf = torch.zeros((B, 32), dtype=torch.int64, device="cuda")
eng.debug_timers(buf)
out = eng.ocp_solve(sb["ini"], sb["goal"], sb["dnn_out"][:, :3].astype(np.float64),
                    sb["dnn_out"][:, 3:6].astype(np.float64), sb["dnn_out"][:, 6].astype(np.float64))
torch.cuda.synchronize()
eng.debug_timers(None)
d = buf[:, :4].cpu().numpy().view(np.float64)
st = out["status"].cpu().numpy() if hasattr(out["status"], "cpu") else np.asarray(out["status"])
print(f"B={B} counters {eng.last_counters()} status {np.bincount(st.astype(np.int64), minlength=10).tolist()}")
for i, name in enumerate(["record K^T k L", "P_k packed", "p_k"]):
    v = d[:, i]
    print(f"  {name:16s} max {v.max():.3e}  p99 {np.quantile(v, 0.99):.3e}  p50 {np.median(v):.3e}  "
          f"worst instance {int(v.argmax())}")
print(f"  inertia-test disagreements: {int(d[:, 3].sum())} over {int((d[:, 3] > 0).sum())} instances")
