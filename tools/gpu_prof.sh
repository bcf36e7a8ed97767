#!/bin/bash
# Round profile: bench line + rocprofv3 kernel stats + PMC passes (HBM bytes, wave-state counters).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $OUT
B=${B:-4096}
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --batch $B > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --batch $B --no-cpu-baseline > $OUT/bench_kt.json 2> $OUT/kt.err || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --batch $B --no-cpu-baseline > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --batch $B --no-cpu-baseline > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit $?
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --batch $B --no-cpu-baseline > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || exit $?
find $OUT -name "*.csv" | head -50 > $OUT/files.txt
