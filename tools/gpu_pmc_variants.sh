#!/bin/bash
# SQ instruction / wait counters of one bench launch for the in-tree build and each liblafse3_V*.so
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcvar
mkdir -p $OUT
CMD="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra"
CTR="SQ_INSTS_FLAT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
timeout -s KILL 180 rocprofv3 --pmc $CTR -d $OUT/base -o run --output-format csv -- $CMD > $OUT/base.log 2>&1 || exit $?
for v in learningagileflight_se3_amd/liblafse3_V*.so; do
  n=$(basename $v .so)
  LAFSE3_LIB=$GRAFT_REPO_ROOT/$v timeout -s KILL 180 rocprofv3 --pmc $CTR -d $OUT/$n -o run --output-format csv -- $CMD > $OUT/$n.log 2>&1 || exit $?
done
