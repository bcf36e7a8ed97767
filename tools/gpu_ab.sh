# A/B of an alternative build of the same ABI (LAFSE3_LIB): GPU parity tests (minus the in-tree-library
# name check) and a quick bench.  usage: gpurun -- bash tools/gpu_ab.sh  (edit LAFSE3_LIB below)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export LAFSE3_LIB=$GRAFT_REPO_ROOT/learningagileflight_se3_amd/liblafse3_hbm.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "not native_library" --timeout 200 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/ab_pytest.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_bench.log 2>&1
