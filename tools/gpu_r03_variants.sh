#!/bin/bash
# round 3: hot-path kernel time (restoration off) of alternative builds of this tree (VARIANTS env: suffixes of
# learningagileflight_se3_amd/liblafse3_<v>.so), placement records
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/learningagileflight_se3_amd
for v in $VARIANTS; do
  RESTO=${RESTO:-0} LAFSE3_LIB=$L/liblafse3_$v.so timeout -k 10 200 python -u tools/gpu_placement.py > gpurun_out/r03_var_$v.log 2>&1 || exit 1
done
