#!/bin/bash
# facbench (tools/facbench.py) over the liblafse3_VF*.so diagnostic builds, B instances each
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/facbench.log
for v in ${VARIANTS:-VF1 VF2 VF3 VF4}; do LAFSE3_LIB=$GRAFT_REPO_ROOT/learningagileflight_se3_amd/liblafse3_$v.so timeout -k 10 120 python tools/facbench.py ${B:-8192} >> gpurun_out/facbench.log 2>&1 || exit $?; done
