#!/bin/bash
# round 3: per-CU contention -- replicated vs distinct instances at 1 and 4 waves per CU, and the SQC instruction
# cache counters of each (one rocprofv3 --pmc pass per run)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/icache
O=gpurun_out/icache
for B in 256 1024; do
  B=$B timeout -k 10 120 python tools/gpu_one.py >> $O/times.log 2>&1 || exit 1
  B=$B timeout -k 10 120 python tools/one_diverse.py >> $O/times.log 2>&1 || exit 1
done
for B in 256 1024; do
  B=$B timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d $O/one_$B -o run --output-format csv -- python3 tools/gpu_one.py > $O/one_$B.log 2>&1 || exit 1
  B=$B timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d $O/div_$B -o run --output-format csv -- python3 tools/one_diverse.py > $O/div_$B.log 2>&1 || exit 1
done
