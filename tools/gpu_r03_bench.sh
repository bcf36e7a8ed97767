#!/bin/bash
# round 3: default bench (configs[2]) and the configs[4] moving-gate bench at 8192 episodes x 500 plant steps
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err &&
timeout -k 10 500 python bench.py --workload moving --batch 8192 --plant-steps 500 --steps 1 --warmup 1 > gpurun_out/bench_moving500.json 2> gpurun_out/bench_moving500.err
