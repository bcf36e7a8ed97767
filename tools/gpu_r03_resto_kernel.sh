#!/bin/bash
# round 3: device restoration phase -- its GPU tests, the parity suite, a short bench (each step time-limited)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resto.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r03_resto_tests.log 2>&1
echo "resto tests rc=$?" >> gpurun_out/r03_resto_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03_parity.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r03_bench_resto.json 2> gpurun_out/r03_bench_resto.err
