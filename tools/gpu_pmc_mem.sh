#!/bin/bash
# Memory-side PMC passes of one ipm_kernel launch (tools/gpu_one.py, B samples of sol_gradient):
# FETCH_SIZE, WRITE_SIZE, and the vector-memory / flat (scratch) instruction counts.  Separate --pmc runs,
# each under its own time limit; LAFSE3_LIB selects an alternative build.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${PMCDIR:-pmcmem}
mkdir -p $OUT
export B=${B:-4096}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/f -o run --output-format csv -- python3 tools/gpu_one.py > $OUT/f.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/w -o run --output-format csv -- python3 tools/gpu_one.py > $OUT/w.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $OUT/s -o run --output-format csv -- python3 tools/gpu_one.py > $OUT/s.log 2>&1 || exit $?
