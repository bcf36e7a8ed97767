cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py -m gpu -x -v -s --timeout 240 --timeout-method thread -k full_length > gpurun_out/pytest_moving500.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err &&
timeout -k 10 400 python bench.py --workload moving --batch 8192 --plant-steps 500 --steps 1 --warmup 1 > gpurun_out/bench_moving500.json 2> gpurun_out/bench_moving500.err  &&
for v in VF1 VF2 VF3; do LAFSE3_LIB=$GRAFT_REPO_ROOT/learningagileflight_se3_amd/liblafse3_$v.so timeout -k 10 120 python tools/facbench.py 8192 >> gpurun_out/facbench.log 2>&1 || exit $?; done
