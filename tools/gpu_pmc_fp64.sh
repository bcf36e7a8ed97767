#!/bin/bash
# FP64 work actually executed by ipm_kernel in the bench launch (one pass, 8 SQ + 1 GRBM counters): f64 MFMA
# instructions and their math ops (MOPS x 512 = flops), MFMA busy cycles, f64 VALU FMA / ADD / MUL / transcendental
# instructions, all VALU instructions.  Output: gpurun_out/pmc_fp64/ (summarise with tools/pmc_fp64_summary.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_fp64
mkdir -p $OUT
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $OUT/p -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra > $OUT/p.log 2>&1
