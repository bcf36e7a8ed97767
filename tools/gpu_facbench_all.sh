#!/bin/bash
# facbench over every learningagileflight_se3_amd/liblafse3_VF*.so, ROUNDS interleaved rounds (B = 8192)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/facbench_all.log
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in learningagileflight_se3_amd/liblafse3_VF*.so; do
    LAFSE3_LIB=$GRAFT_REPO_ROOT/$v timeout -k 10 120 python tools/facbench.py ${B:-8192} 2>&1 | grep -v amdgpu.ids >> gpurun_out/facbench_all.log || exit $?
  done
done
python3 - <<'PY'
import re, collections
r = collections.defaultdict(list)
for l in open("gpurun_out/facbench_all.log"):
    m = re.match(r"(\S+) B=\d+ kernel_ms \[([^\]]*)\]", l)
    if m:
        r[m.group(1)].append(min(float(x) for x in m.group(2).split(",")))
for k, v in sorted(r.items()):
    print(f"{k:24s} min kernel ms {min(v):.3f}  runs {['%.3f' % x for x in v]}")
PY
