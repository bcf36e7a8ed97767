#!/bin/bash
# Interleaved bench of the in-tree liblafse3.so ("base") and every learningagileflight_se3_amd/liblafse3_V*.so
# (same ABI, other build flags / sources), ROUNDS rounds; one line per run in gpurun_out/variants.log.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/variants.log
D=$GRAFT_REPO_ROOT/learningagileflight_se3_amd
for i in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS---no-extra} | sed 's/^/base /' >> gpurun_out/variants.log || exit $?
  for v in $D/liblafse3_V*.so; do
    [ -f "$v" ] || continue
    n=$(basename $v .so)
    LAFSE3_LIB=$v timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS---no-extra} | sed "s/^/${n#liblafse3_} /" >> gpurun_out/variants.log || exit $?
  done
done
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
for l in open("gpurun_out/variants.log"):
    n, j = l.split(" ", 1)
    d = json.loads(j); r[n].append((d["value"], d["kernel_ms"], d["ipm_iterations_per_solve"], d.get("ift_grads_per_s"), d.get("ocp_solve_per_s")))
for n, v in r.items():
    print(n, "value", [x[0] for x in v], "kernel_ms", [x[1] for x in v], "iters", v[0][2], "ift", [x[3] for x in v], "ocp", [x[4] for x in v])
PY
