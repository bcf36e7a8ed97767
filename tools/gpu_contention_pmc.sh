#!/bin/bash
# round 3: which per-CU resource slows a wave when 4 share a CU -- SQ wait/issue counters of the replicated instance
# (tools/gpu_one.py) at 1 wave per CU (B = 256) and 4 (B = 1024); one --pmc pass per run
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/cont
O=gpurun_out/cont
for B in 256 1024; do
  B=$B timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d $O/a_$B -o run --output-format csv -- python3 tools/gpu_one.py > $O/a_$B.log 2>&1 || exit 1
  B=$B timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_VALU -d $O/b_$B -o run --output-format csv -- python3 tools/gpu_one.py > $O/b_$B.log 2>&1 || exit 1
  B=$B timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum -d $O/c_$B -o run --output-format csv -- python3 tools/gpu_one.py > $O/c_$B.log 2>&1 || exit 1
done
