#!/bin/bash
# round 4: speculative-sweep check -- parity subset, facbench (sequential vs speculative), phase timers, quick benches
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/learningagileflight_se3_amd
VARIANTS="${VARIANTS:-VF0 VF1 VF3 VF4}" B=8192 bash tools/gpu_facbench.sh || exit $?
for v in ${TIMERS:-VT0 VT1 VT2}; do
  echo "== $v" >> gpurun_out/timers.log
  LAFSE3_LIB=$L/liblafse3_$v.so BIG=2048 timeout -k 10 200 python tools/gpu_timers.py >> gpurun_out/timers.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_spec.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_spec.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/bench_spec.log 2>&1 || exit $?
LAFSE3_LIB=$L/liblafse3_VS0.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/bench_seq.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/resto_diverge.py device > gpurun_out/resto_diverge_dev.log 2>&1 || exit $?
