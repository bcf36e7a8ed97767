#!/bin/bash
# round 3 final: full GPU suite, smoke, then the round profile (bench line + rocprofv3 stats + PMC passes)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
TAG=${TAG:-r03_final} bash tools/gpu_profile.sh
