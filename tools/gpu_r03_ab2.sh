#!/bin/bash
# round 3: GPU suite on the in-tree build, then an interleaved A/B against the liblafse3_V*.so builds
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab2.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_ab2.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} bash tools/gpu_variants.sh
