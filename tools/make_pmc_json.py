"""Summarise a tools/gpu_prof.sh run (gpurun_out/prof) into profiles/<tag>_*.

    python tools/make_pmc_json.py <tag>          # e.g. r01_v3

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats), profiles/<tag>_bench.json (the bench line),
profiles/<tag>_pmc.json and profiles/pmc_current.json (HBM bytes per ipm_kernel launch, which bench.py
reports as roofline.traffic).  FETCH_SIZE is doubled (gfx950 half-count correction,
MI355X_MICROARCH.md HBM/rocprofv3 section); WRITE_SIZE is taken as is.  Both counters are in KB.
"""
import csv
import collections
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "gpurun_out", "prof")
KERNEL = "ipm_kernel"


def counters(path):
    agg, n = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]].add(r.get("Dispatch_Id", r.get("Correlation_Id", "0")))
    launches = max((len(v) for v in n.values()), default=1)
    return {k: v / launches for k, v in agg.items()}, launches


def main(tag):
    out = os.path.join(REPO, "profiles")
    shutil.copy(os.path.join(PROF, "kt", "run_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    shutil.copy(os.path.join(PROF, "bench.json"), os.path.join(out, f"{tag}_bench.json"))
    kns = None
    for r in csv.DictReader(open(os.path.join(PROF, "kt", "run_kernel_stats.csv"))):
        if KERNEL in r["Name"]:
            kns = float(r["AverageNs"])
    fetch, nl = counters(os.path.join(PROF, "pmc_fetch", "run_counter_collection.csv"))
    write, _ = counters(os.path.join(PROF, "pmc_write", "run_counter_collection.csv"))
    sq, _ = counters(os.path.join(PROF, "pmc_sq", "run_counter_collection.csv"))
    fb = fetch["FETCH_SIZE"] * 1024 * 2
    wb = write["WRITE_SIZE"] * 1024
    bench = json.loads(open(os.path.join(PROF, "bench.json")).read().strip().splitlines()[-1])
    rec = {
        "kernel": "lafse3::ipm_kernel",
        "command": f"python3 bench.py --steps 1 --warmup 0 --batch {bench['config']['batch_per_gpu']} --no-cpu-baseline "
                   f"(one sol_gradient launch = {9 * bench['config']['batch_per_gpu']} NLP instances)",
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE (KB) x1024 x2 "
                  "(gfx950 half-count correction, MI355X_MICROARCH.md HBM section); WRITE_SIZE (KB) x1024",
        "fetch_bytes": fb,
        "write_bytes": wb,
        "hbm_bytes_per_launch": fb + wb,
        "kernel_ns": kns,
        "hbm_GBps": (fb + wb) / kns if kns else None,
        "sq": sq,
        "wave_state_fraction": {
            "wait_any": sq.get("SQ_WAIT_ANY", 0) / sq["SQ_WAVE_CYCLES"],
            "active_inst": sq.get("SQ_ACTIVE_INST_ANY", 0) / sq["SQ_WAVE_CYCLES"],
            "wait_inst": sq.get("SQ_WAIT_INST_ANY", 0) / sq["SQ_WAVE_CYCLES"],
        } if sq.get("SQ_WAVE_CYCLES") else None,
        "bench_value": bench["value"],
    }
    for name in (f"{tag}_pmc.json", "pmc_current.json"):
        with open(os.path.join(out, name), "w") as f:
            json.dump(rec, f, indent=1)
    print(json.dumps({k: rec[k] for k in ("hbm_bytes_per_launch", "kernel_ns", "hbm_GBps", "bench_value")}))


if __name__ == "__main__":
    main(sys.argv[1])
