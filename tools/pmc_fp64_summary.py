"""Per-launch totals of tools/gpu_pmc_fp64.sh's counters for lafse3::ipm_kernel, and the FP64 flops they imply:
MFMA flops = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512; VALU flops = 64 lanes x (2 FMA + ADD + MUL) instructions (every lane
counted, active or not: an upper bound of the useful work).

    python3 tools/pmc_fp64_summary.py gpurun_out/pmc_fp64 [kernel_ms]
"""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1]
f = glob.glob(os.path.join(src, "p", "**", "*counter_collection.csv"), recursive=True)[0]
tot = collections.defaultdict(float)
disp = set()
for r in csv.DictReader(open(f)):
    if "ipm_kernel" not in r["Kernel_Name"]:
        continue
    disp.add(r["Dispatch_Id"])
    tot[r["Counter_Name"]] += float(r["Counter_Value"])
n = max(len(disp), 1)
per = {k: v / n for k, v in tot.items()}
mfma_flops = per.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0) * 512
valu_flops = 64 * (2 * per.get("SQ_INSTS_VALU_FMA_F64", 0) + per.get("SQ_INSTS_VALU_ADD_F64", 0)
                   + per.get("SQ_INSTS_VALU_MUL_F64", 0))
out = {"dispatches": n, "per_launch": per, "mfma_f64_flops": mfma_flops, "valu_f64_flops_upper": valu_flops}
if len(sys.argv) > 2:
    t = float(sys.argv[2]) / 1e3
    out["kernel_s"] = t
    out["executed_f64_TFLOPs"] = (mfma_flops + valu_flops) / t / 1e12
    out["mfma_share_of_f64_flops"] = mfma_flops / max(mfma_flops + valu_flops, 1)
print(json.dumps(out, indent=1))
