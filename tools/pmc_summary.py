"""Per-launch ipm_kernel counter totals of a tools/gpu_pmc_mem.sh run, normalised per IPM iteration.

    python tools/pmc_summary.py gpurun_out/pmcB
"""
import collections, csv, glob, os, re, sys

d = sys.argv[1]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "ipm_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r.get("Dispatch_Id", "0"))
it = None
for f in glob.glob(os.path.join(d, "*.log")):
    m = re.search(r"'iterations': (\d+), 'sweeps': (\d+)", open(f).read())
    if m:
        it, sw = int(m.group(1)), int(m.group(2))
print(f"iterations {it} sweeps {sw} (per launch)")
for k, v in sorted(agg.items()):
    v /= max(1, len(disp[k]))
    extra = ""
    if k in ("FETCH_SIZE", "WRITE_SIZE"):
        extra = f"  = {v * 1024 / it / 1e3:.1f} KB/iteration"
    elif k.startswith("SQ_INSTS"):
        extra = f"  = {v / it:.1f} wave-instr/iteration"
    print(f"{k:22s} {v:.4e}{extra}")
