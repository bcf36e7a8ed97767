cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pcs
cd /tmp
B=64 timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $GRAFT_REPO_ROOT/gpurun_out/pcs -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/gpu_lane_timers.py > $GRAFT_REPO_ROOT/gpurun_out/pcs/log.txt 2>&1
rc=$?
ls -la $GRAFT_REPO_ROOT/gpurun_out/pcs >> $GRAFT_REPO_ROOT/gpurun_out/pcs/log.txt
exit $rc
