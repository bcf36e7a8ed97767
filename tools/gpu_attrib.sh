#!/bin/bash
# Phase attribution: bench of builds in which one phase runs twice per call (liblafse3_rep_<PHASE>.so, built by
# tools/build_attrib.sh) against the plain build; the difference is that phase's share of the step.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/attrib.log
for v in base FAC BWD FWD ADJ RES; do
  if [ $v = base ]; then lib=$GRAFT_REPO_ROOT/learningagileflight_se3_amd/liblafse3.so; else lib=$GRAFT_REPO_ROOT/learningagileflight_se3_amd/liblafse3_rep_$v.so; fi
  LAFSE3_LIB=$lib timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra | sed "s/^/$v /" >> gpurun_out/attrib.log || exit $?
done
