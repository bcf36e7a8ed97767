cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err &&
timeout -k 10 300 python tools/gpu_moving_fail.py 1024 > gpurun_out/moving_fail.json 2> gpurun_out/moving_fail.err
