cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 400 python tools/gpu_diag.py > gpurun_out/diag1.log 2>&1
echo "exit $?" >> gpurun_out/diag1.log
