#!/bin/bash
# round 3: where the bench kernel's time goes with the restoration phase (placement record), with it off, and the
# round-2 build; the moving-fixture device results for the host comparison
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/gpu_resto_moving.py > gpurun_out/r03_resto_moving.log 2>&1 || exit 1
OUT=gpurun_out/r03_place_resto1.npz timeout -k 10 200 python -u tools/gpu_placement.py > gpurun_out/r03_place_resto1.log 2>&1 || exit 1
RESTO=0 OUT=gpurun_out/r03_place_resto0.npz timeout -k 10 200 python -u tools/gpu_placement.py > gpurun_out/r03_place_resto0.log 2>&1 || exit 1
LAFSE3_LIB=$GRAFT_REPO_ROOT/learningagileflight_se3_amd/liblafse3_old.so OUT=gpurun_out/r03_place_old.npz timeout -k 10 200 python -u tools/gpu_placement.py > gpurun_out/r03_place_old.log 2>&1
