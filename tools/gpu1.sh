cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu_timers.py > gpurun_out/timers.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/timers.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; exit $rc
