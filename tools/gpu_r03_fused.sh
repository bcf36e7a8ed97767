cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_fused.log
ROUNDS=2 bash tools/gpu_variants.sh
