#!/bin/bash
# A/B of environment switches with extra bench arguments (one GPU box call):
#   tools/ab_args.sh "<bench args>" "ENV=1" "ENV=2" ...
mkdir -p gpurun_out
: > gpurun_out/ab.txt
args=$1; shift
for v in "$@"; do
  env $v timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline $args > gpurun_out/ab_run.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v rc=$rc" | tee -a gpurun_out/ab.txt; tail -5 gpurun_out/ab_run.log; exit $rc; fi
  python - "$v" >> gpurun_out/ab.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_run.log").read().strip().split("\n")[-1])
print(sys.argv[1], "ms/step %.4f" % d["ms_per_step"], json.dumps(d["step_kernel_ms"]))
PY
done
cat gpurun_out/ab.txt
