cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_lds
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_lds -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --batch 2048 --no-cpu-baseline > gpurun_out/pmc_lds/bench.json 2> gpurun_out/pmc_lds/err.txt
