#!/bin/bash
# A/B bench runs over environment settings: tools/ab_env.sh "NAME=ENV ..." ...
# Each run is bounded; the script stops at the first failure.
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 180 python bench.py --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "FAIL $name"; tail -5 gpurun_out/ab_$name.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/ab_$name.json') if l.startswith('{')][-1]); k=d['step_kernel_ms']
print('$name', round(d['ms_per_step'],4), {a: k[a] for a in list(k)[:6]})"
done
