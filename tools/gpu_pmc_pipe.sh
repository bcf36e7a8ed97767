#!/bin/bash
# Memory-pipeline PMC passes of the bench launch (round 6): TA / TD / TCP busy and stall cycles, L1 -> L2 requests and
# their latency, SQ issue levels and FIFO-full cycles.  One --pmc run per pass, each under its own time limit;
# LAFSE3_LIB selects the build.  Summarise with: python3 tools/pmc_summary.py gpurun_out/$PMCDIR
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${PMCDIR:-pmcpipe}
mkdir -p $OUT
CMD="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra"
i=0
while read -r ctrs; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs -d $OUT/p$i -o run --output-format csv -- $CMD > $OUT/p$i.log 2>&1 || exit $?
done <<'PASSES'
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TA_BUSY_sum
TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum
TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_ACCESSES_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL
SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_DATA_FIFO_FULL SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU
PASSES
