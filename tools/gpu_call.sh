#!/bin/bash
# One GPU-box call made of named steps, run in order; each GPU step has its own time limit and the call stops at the
# first failing step (no GPU step runs after a failure, a timeout or a fault).  Output under gpurun_out/.
#
#   gpurun -- bash tools/gpu_call.sh STEP [STEP ...]
#
# steps:
#   suite           pytest -m gpu (the whole GPU suite)                 -> gpurun_out/pytest_gpu.log
#   parity          tests/test_gpu_parity.py (PYTEST_K= selects)        -> gpurun_out/pytest_parity.log
#   resto           tests/test_gpu_resto.py                             -> gpurun_out/pytest_resto.log
#   rows            tests/test_gpu_rows.py                              -> gpurun_out/pytest_rows.log
#   smoke           __graft_entry__.smoke()                             -> gpurun_out/smoke.log
#   bench           bench.py default line (BENCH_ARGS= extra flags)     -> gpurun_out/bench.json
#   quick           bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra -> gpurun_out/bench_quick.json
#   moving          bench.py --workload moving (8192 x 500, one step)  -> gpurun_out/bench_moving.json
#   facbench        tools/facbench.py over VARIANTS (liblafse3_<v>.so)  -> gpurun_out/facbench.log
#   variants        tools/gpu_variants.sh (interleaved A/B of liblafse3_V*.so) -> gpurun_out/variants.log
#   timers          tools/gpu_timers.py (diagnostic build liblafse3_timers.so) -> gpurun_out/timers.log
#   placement       tools/gpu_placement.py (RESTO=, OUT=)               -> gpurun_out/placement.log
#   profile         tools/gpu_profile.sh (TAG=): bench + rocprofv3 stats + PMC passes
#   rl              tools/gpu_rl_schedule.py: the reference's RL schedule end to end -> gpurun_out/rl_schedule.log
#   diverge         tools/resto_diverge.py device: IPM traces of the restoration fixtures -> gpurun_out/resto_trace_gpu.npz
#   mprof           rocprofv3 --kernel-trace --stats of the configs[4] moving line -> gpurun_out/mprof/
#   mtrace          rocprofv3 --kernel-trace of tools/gpu_moving_trace.py (RUNS=), cut by tools/trace_moving.py -> gpurun_out/mtrace/
#   side            tools/gpu_moving_side.py: the configs[4] side figure repeated in one process -> gpurun_out/moving_side.log
#   pipe            tools/gpu_pmc_pipe.sh: memory-pipeline PMC passes (PMCDIR=)   -> gpurun_out/pmcpipe/
#   ab              tools/gpu_ab.sh $AB (interleaved quick lines + DNN1 checksum per build) -> gpurun_out/ab.log
#   tests           pytest of TESTS= (files / node ids)                 -> gpurun_out/pytest_tests.log
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/learningagileflight_se3_amd
PT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
for step in "$@"; do
  echo "[gpu_call] $step $(date +%T)"
  case $step in
    suite)     timeout -k 10 840 $PT tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 ;;
    parity)    timeout -k 10 600 $PT tests/test_gpu_parity.py ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_parity.log 2>&1 ;;
    resto)     timeout -k 10 600 $PT tests/test_gpu_resto.py > gpurun_out/pytest_resto.log 2>&1 ;;
    rows)      timeout -k 10 600 $PT tests/test_gpu_rows.py > gpurun_out/pytest_rows.log 2>&1 ;;
    smoke)     timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench)     timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err ;;
    quick)     timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err ;;
    moving)    timeout -k 10 600 python bench.py --workload moving --batch 8192 --plant-steps 500 --steps 1 --warmup 1 > gpurun_out/bench_moving.json 2> gpurun_out/bench_moving.err ;;
    facbench)  : > gpurun_out/facbench.log
               for v in ${VARIANTS:-VF0 VF1}; do
                 LAFSE3_LIB=$L/liblafse3_$v.so timeout -k 10 120 python tools/facbench.py ${B:-8192} >> gpurun_out/facbench.log 2>&1 || exit $?
               done ;;
    variants)  ROUNDS=${ROUNDS:-2} bash tools/gpu_variants.sh > gpurun_out/variants_summary.log 2>&1 ;;
    timers)    timeout -k 10 300 python tools/gpu_timers.py > gpurun_out/timers.log 2>&1 ;;
    placement) timeout -k 10 300 python -u tools/gpu_placement.py > gpurun_out/placement.log 2>&1 ;;
    profile)   TAG=${TAG:-r04} bash tools/gpu_profile.sh ;;
    rl)        timeout -k 10 1100 python -u tools/gpu_rl_schedule.py > gpurun_out/rl_schedule.log 2>&1 ;;
    diverge)   timeout -k 10 300 python -u tools/resto_diverge.py device > gpurun_out/resto_diverge_dev.log 2>&1 ;;
    mprof)     mkdir -p gpurun_out/mprof && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof/trace -o run --output-format csv -- python3 bench.py --workload moving --batch 8192 --plant-steps 500 --steps 1 --warmup 1 > gpurun_out/mprof/bench.json 2> gpurun_out/mprof/err.log && find gpurun_out/mprof -name "*kernel_trace.csv" -delete ;;
    mtrace)    mkdir -p gpurun_out/mtrace && timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/mtrace/trace -o run --output-format csv -- python3 tools/gpu_moving_trace.py ${RUNS:-fresh fresh kept kept} > gpurun_out/mtrace/runs.log 2> gpurun_out/mtrace/err.log && f=$(find gpurun_out/mtrace -name "*kernel_trace.csv" | head -1) && timeout -k 10 300 python3 tools/trace_moving.py "$f" --dump gpurun_out/mtrace/solver_kernels.csv > gpurun_out/mtrace/summary.log 2>&1 && rm -f "$f" ;;
    side)      timeout -k 10 400 python -u tools/gpu_moving_side.py > gpurun_out/moving_side.log 2>&1 ;;
    pipe)      bash tools/gpu_pmc_pipe.sh ;;
    ab)        bash tools/gpu_ab.sh $AB > gpurun_out/ab_summary.log 2>&1 ;;
    tests)     timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread $TESTS > gpurun_out/pytest_tests.log 2>&1 ;;   # no -x: every failure
    *)         echo "[gpu_call] unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "[gpu_call] $step rc=$rc $(date +%T)"
  [ $rc -eq 0 ] || exit $rc
done
