#!/bin/bash
# Interleaved bench of up to three builds of the same ABI: A = liblafse3_A.so, B = liblafse3.so (in-tree),
# C = liblafse3_B2.so (if present)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/abc.log
D=$GRAFT_REPO_ROOT/learningagileflight_se3_amd
for i in 1 2; do
  LAFSE3_LIB=$D/liblafse3_A.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra | sed 's/^/A /' >> gpurun_out/abc.log || exit $?
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra | sed 's/^/B /' >> gpurun_out/abc.log || exit $?
  if [ -f $D/liblafse3_B2.so ]; then
    LAFSE3_LIB=$D/liblafse3_B2.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra | sed 's/^/C /' >> gpurun_out/abc.log || exit $?
  fi
done
