"""Summarise a tools/gpu_profile.sh run into profiles/<tag>_* and profiles/pmc_current.json.

    python3 tools/make_pmc_current.py gpurun_out/r02_prof r02_prof

Writes profiles/<tag>_bench.json (the bench line), profiles/<tag>_kernel_stats.csv (rocprofv3 --stats),
profiles/<tag>_pmc.json (per-launch counter totals of lafse3::ipm_kernel) and profiles/pmc_current.json
(what bench.py reads for roofline.traffic / traffic_source).  FETCH_SIZE is in KB and counts half the bytes
of wide reads on gfx950 (MI355X_MICROARCH.md HBM section): bytes = KB x 1024 x 2; WRITE_SIZE KB x 1024.
"""
import collections
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, tag = sys.argv[1], sys.argv[2]
prof = os.path.join(REPO, "profiles")
bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
json.dump(bench, open(os.path.join(prof, f"{tag}_bench.json"), "w"), indent=1)
stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
kstat = {}
for r in csv.DictReader(open(stats[0])):
    if "ipm_kernel" in r["Name"]:
        kstat = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}

agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for p in ("f", "w", "s", "l"):
    for f in glob.glob(os.path.join(src, p, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "ipm_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r.get("Dispatch_Id", "0"))
per = {k: v / max(1, len(disp[k])) for k, v in agg.items()}
sys.path.insert(0, REPO)
from learningagileflight_se3_amd.build import source_hash   # noqa: E402

commit = subprocess.run(["git", "-C", REPO, "rev-parse", "--short", "HEAD"], capture_output=True,
                        text=True).stdout.strip()
fetch = per["FETCH_SIZE"] * 1024 * 2
write = per["WRITE_SIZE"] * 1024
kns = kstat.get("avg_ns")
out = {
    "kernel": "lafse3::ipm_kernel",
    "command": "python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra (one sol_gradient launch, "
               "B=4096 samples = 36864 NLP instances)",
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE (KB) x1024 x2 "
              "(gfx950 half-count correction, MI355X_MICROARCH.md HBM section); WRITE_SIZE (KB) x1024",
    "source": f"profiles/{tag}_pmc.json (tools/gpu_profile.sh at commit {commit})",
    "fetch_bytes": fetch,
    "write_bytes": write,
    "hbm_bytes_per_launch": fetch + write,
    "kernel_ns_rocprof_stats": kns,
    "hbm_GBps": (fetch + write) / kns if kns else None,
    "counters": {k: v for k, v in sorted(per.items())},
    "wave_state_fraction": {
        "wait_any": per.get("SQ_WAIT_ANY", 0) / per["SQ_WAVE_CYCLES"],
        "active_inst": per.get("SQ_ACTIVE_INST_ANY", 0) / per["SQ_WAVE_CYCLES"],
        "wait_inst": per.get("SQ_WAIT_INST_ANY", 0) / per["SQ_WAVE_CYCLES"],
    } if "SQ_WAVE_CYCLES" in per else None,
    # the kernel sources the profile was taken on (bench.py uses traffic only when this equals the tree's hash)
    "csrc_sha": source_hash(),
    # VALU instructions per algorithmic 64-lane FMA instruction: SQ_INSTS_VALU / (IPM iterations x 740 kflop /
    # 128 flop), iterations from the bench line of the same build (ipm_iterations_per_solve x solves)
    "valu_insts_per_alg_fma": (per["SQ_INSTS_VALU"] / (bench["ipm_iterations_per_solve"] * 9 * 4096 * 740000 / 128)
                               if "SQ_INSTS_VALU" in per and bench.get("ipm_iterations_per_solve") else None),
    "bench_value": bench.get("value"),
    "bench_kernel_ms": bench.get("kernel_ms"),
}
json.dump(out, open(os.path.join(prof, f"{tag}_pmc.json"), "w"), indent=1)
json.dump(out, open(os.path.join(prof, "pmc_current.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
