#!/bin/bash
# Iteration check on the GPU box: parity tests, phase timers, short bench (no CPU baseline).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/gpu_timers.py > gpurun_out/timers.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit $?
