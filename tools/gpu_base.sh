#!/bin/bash
# Baseline probe on the GPU box: phase timers (diagnostic build) and a short bench line.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
BIG=2048 timeout -k 10 200 python -u tools/gpu_timers.py > gpurun_out/timers.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit $?
