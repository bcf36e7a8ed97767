#!/bin/bash
# L2 / memory-side counters of the bench launch (one sol_gradient step, B = 4096), one rocprofv3 --pmc pass each:
#   L2 hit rate (TCC_HIT / TCC_MISS), L2 -> fabric reads and their DRAM-bound part, and the average fabric read
#   latency by Little's law (TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_l2; mkdir -p $OUT
CMD="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra"
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/a -o run --output-format csv -- $CMD > $OUT/a.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $OUT/b -o run --output-format csv -- $CMD > $OUT/b.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum -d $OUT/c -o run --output-format csv -- $CMD > $OUT/c.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum -d $OUT/d -o run --output-format csv -- $CMD > $OUT/d.log 2>&1
rc=$?
python3 - <<'PY'
import csv, glob, collections, os
out = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out", "pmc_l2")
agg, disp = collections.defaultdict(float), collections.defaultdict(set)
for f in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
    p = os.path.relpath(f, out).split(os.sep)[0]
    for r in csv.DictReader(open(f)):
        if "ipm_kernel" in r["Kernel_Name"]:
            k = p + ":" + r["Counter_Name"]
            agg[k] += float(r["Counter_Value"]); disp[k].add(r.get("Dispatch_Id", "0"))
per = {k: v / max(1, len(disp[k])) for k, v in agg.items()}
for k in sorted(per):
    print(f"{k:40s} {per[k]:.6e}")
PY
exit $rc
