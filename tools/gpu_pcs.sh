#!/bin/bash
# PC sampling of one sol_gradient launch (rocprofv3 --pc-sampling-beta-enabled), summarised on the box by
# tools/pcs_summary.py (the raw CSV stays on the box).  LIB = the library to sample (default: the -gline-tables-only
# build liblafse3_VG.so, whose instruction comments carry source lines); BATCH = samples (default 1024).
#   gpurun -- bash tools/gpu_pcs.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pcs
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/learningagileflight_se3_amd
export LAFSE3_LIB=${LIB:-$L/liblafse3_VG.so}
CMD="python3 bench.py --batch ${BATCH:-1024} --steps 1 --warmup 0 --no-cpu-baseline --no-extra"
run() {   # method unit interval
  rm -rf /tmp/pcs_$1
  timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $1 --pc-sampling-unit $2 \
    --pc-sampling-interval $3 -d /tmp/pcs_$1 -o run --output-format csv -- $CMD > $OUT/$1.log 2>&1
}
summ() {
  f=$(find /tmp/pcs_$1 -name "*pc_sampling*.csv" | head -1)
  [ -n "$f" ] || { echo "no csv for $1"; ls -R /tmp/pcs_$1 | head -20; return 1; }
  ls -la "$f"
  timeout -k 10 300 python3 tools/pcs_summary.py "$f" ipm_kernel > $OUT/$1_summary.txt 2>&1
}
run stochastic cycles ${SINT:-65536}
rc=$?
echo "stochastic rc=$rc"
case $rc in 124|134|137|139) exit $rc ;; esac
if [ $rc -eq 0 ] && summ stochastic; then exit 0; fi
run host_trap time ${HINT:-50}
rc=$?
echo "host_trap rc=$rc"
[ $rc -eq 0 ] || exit $rc
summ host_trap
