cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/abg.log
for r in 1 2; do
  for v in graph eager; do
    if [ $v = eager ]; then X=--eager-train; else X=; fi
    timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra $X 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['kernel_ms'], d['host_ms_per_step'], d['dnn1_param_checksum'], d['config']['dnn1_step'])" >> gpurun_out/abg.log || exit 1
  done
done
cat gpurun_out/abg.log
