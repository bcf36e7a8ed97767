cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
D=$GRAFT_REPO_ROOT/learningagileflight_se3_amd
LAFSE3_LIB=$D/liblafse3_old.so timeout -k 10 300 python tools/dump_moving_fail.py 256 64 > gpurun_out/dump_moving_fail.log 2>&1 &&
LAFSE3_LIB=$D/liblafse3_old.so timeout -k 10 120 python tools/gpu_resto_check.py old > gpurun_out/resto_check.log 2>&1 &&
timeout -k 10 120 python tools/gpu_resto_check.py new >> gpurun_out/resto_check.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
