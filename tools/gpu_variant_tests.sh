#!/bin/bash
# one GPU test (TEST=...) against the in-tree build and every liblafse3_V*.so (LAFSE3_LIB), one line each
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/variant_tests.log
D=$GRAFT_REPO_ROOT/learningagileflight_se3_amd
for v in base $D/liblafse3_V*.so; do
  if [ "$v" = base ]; then n=base; unset LAFSE3_LIB; else n=$(basename $v .so); export LAFSE3_LIB=$v; fi
  timeout -k 10 300 python -u -m pytest "${TEST:-tests/test_gpu_launch.py::test_configs1_full_size_ocp_solve}" -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/vt_$n.log 2>&1; rc=$?
  echo "$n rc=$rc $(grep -E 'passed|failed' gpurun_out/vt_$n.log | tail -1) $(grep -m1 'AssertionError' gpurun_out/vt_$n.log)" >> gpurun_out/variant_tests.log
  [ $rc -le 1 ] || exit $rc
done
cat gpurun_out/variant_tests.log
