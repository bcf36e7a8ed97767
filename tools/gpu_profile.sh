#!/bin/bash
# Round profile of the bench launch (the N=1 default workload: one sol_gradient step, B=4096):
#   1. the bench line itself (HIP-event kernel time, value)
#   2. rocprofv3 --kernel-trace --stats of the same bench command (per-kernel average duration)
#   3. PMC passes, one per run: FETCH_SIZE | WRITE_SIZE | SQ instruction/wait mix | LDS counters
# Each GPU step under its own time limit, chained with &&.  Output under gpurun_out/$TAG/.
# Summarise with: python3 tools/make_pmc_current.py gpurun_out/$TAG profiles/$TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r02_prof}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
CMD="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $OUT/trace.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/f -o run --output-format csv -- $CMD > $OUT/f.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/w -o run --output-format csv -- $CMD > $OUT/w.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/s -o run --output-format csv -- $CMD > $OUT/s.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU -d $OUT/l -o run --output-format csv -- $CMD > $OUT/l.log 2>&1
