#!/bin/bash
# Build a diagnostic variant of liblafse3.so: NAME=VX tools/build_variant.sh -DFOO=1 ...
# -> learningagileflight_se3_amd/liblafse3_$NAME.so (same flags as build.py plus the given -D options)
set -e
cd "$(dirname "$0")/.."
: "${NAME:?NAME=<variant>}"
/opt/rocm/bin/hipcc --offload-arch=${ARCH:-gfx950} -O3 -std=c++17 -fPIC -shared -Wall \
  -mllvm -amdgpu-disable-unclustered-high-rp-reschedule=1 -mllvm -amdgpu-mfma-vgpr-form -mllvm -amdgpu-use-amdgpu-trackers \
  -mllvm -amdgpu-max-memory-clause=31 -Iinclude "$@" \
  -o learningagileflight_se3_amd/liblafse3_$NAME.so learningagileflight_se3_amd/csrc/api.hip
