#!/bin/bash
# round 4 baseline on a fresh box: facbench of the factorisation-only build, quick bench, phase timers
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
VARIANTS="VF0" B=8192 bash tools/gpu_facbench.sh || exit $?
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit $?
timeout -k 10 200 python tools/gpu_timers.py > gpurun_out/timers.log 2>&1 || exit $?
