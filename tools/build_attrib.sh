#!/bin/bash
# builds liblafse3_rep_<PHASE>.so (one phase repeated twice per call) for tools/gpu_attrib.sh
cd "$(dirname "$0")/.."
for v in FAC BWD FWD ADJ RES; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -DLAFSE3_REP_$v=2 \
    -o learningagileflight_se3_amd/liblafse3_rep_$v.so learningagileflight_se3_amd/csrc/api.hip &
done
wait
