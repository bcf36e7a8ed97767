#!/bin/bash
# round 3: A/B of the bench kernel time -- round-2 build (81fc901), soft-restoration build (d0c5bc6), this tree with
# the restoration phase off and on (placement records)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/learningagileflight_se3_amd
for v in old head; do
  LAFSE3_LIB=$L/liblafse3_$v.so OUT=gpurun_out/r03_place_$v.npz timeout -k 10 200 python -u tools/gpu_placement.py > gpurun_out/r03_place_$v.log 2>&1 || exit 1
done
RESTO=0 timeout -k 10 200 python -u tools/gpu_placement.py > gpurun_out/r03_place_resto0b.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_resto.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r03_resto_tests.log 2>&1
