#!/bin/bash
# round 3: full GPU suite + bench placement record (restoration + watchdog, the defaults) + restoration/watchdog off
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/r03_place_wd.npz timeout -k 10 200 python -u tools/gpu_placement.py > gpurun_out/r03_place_wd.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
