#!/bin/bash
# round 3: price one extra LDS read / f64 FMA per factorisation stage (facbench builds VF0, VFL*, VFV*), two
# interleaved passes
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/cost.log
for pass in 1 2; do
  for v in ${VARIANTS:-VF0 VFL16 VFL32 VFV32 VFV64}; do
    LAFSE3_LIB=$GRAFT_REPO_ROOT/learningagileflight_se3_amd/liblafse3_$v.so timeout -k 10 120 python -u tools/facbench.py ${B:-8192} >> gpurun_out/cost.log 2>&1 || exit $?
  done
done
cat gpurun_out/cost.log
