#!/bin/bash
# interleaved quick-bench A/B of liblafse3 variants: bash /tmp/ab.sh name1 name2 ... (main = liblafse3.so)
cd $GRAFT_REPO_ROOT
: > gpurun_out/ab.log
for r in $(seq ${ROUNDS:-2}); do
  for v in "$@"; do
    if [ "$v" = main ]; then L=$PWD/learningagileflight_se3_amd/liblafse3.so; else L=$PWD/learningagileflight_se3_amd/liblafse3_$v.so; fi
    LAFSE3_LIB=$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['value'], d['kernel_ms'], d['ipm_iterations_per_solve'], d['dnn1_param_checksum'])" >> gpurun_out/ab.log || exit 1
  done
done
cat gpurun_out/ab.log
