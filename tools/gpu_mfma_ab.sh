#!/bin/bash
# MFMA factorisation stage vs the VALU stage on one box: facbench (liblafse3_VF0 / VF1), stage timers
# (liblafse3_timers.so = MFMA, liblafse3_T0.so = VALU), the FAC_CHECK A/B at the initial point (FC2) and in the
# IPM solve (FC); every step time-limited, the call stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/learningagileflight_se3_amd
: > gpurun_out/mfma_ab.log
for step in ${STEPS:-check facbench timers}; do
  case $step in
    check)    for v in FC2 FC; do [ -f $L/liblafse3_$v.so ] || continue
                LAFSE3_LIB=$L/liblafse3_$v.so timeout -k 10 120 python -u tools/fac_check.py 256 >> gpurun_out/mfma_ab.log 2>&1 || exit $?; done ;;
    facbench) for v in VF0 VF1; do LAFSE3_LIB=$L/liblafse3_$v.so timeout -k 10 120 python tools/facbench.py 8192 >> gpurun_out/mfma_ab.log 2>&1 || exit $?; done ;;
    timers)   for v in liblafse3_timers liblafse3_T0; do [ -f $L/$v.so ] || continue; echo "== timers $v" >> gpurun_out/mfma_ab.log
                BIG=4096 LAFSE3_LIB=$L/$v.so timeout -k 10 200 python -u tools/gpu_timers.py 2>&1 | grep -E "kernel|per stage|cycles/instance" >> gpurun_out/mfma_ab.log || exit $?; done ;;
  esac
done
grep -v amdgpu.ids gpurun_out/mfma_ab.log
