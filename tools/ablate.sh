#!/bin/bash
# quick A/B of kernel paths / activations (bench JSON summaries)
for cfg in "Sine 1" "ReLU 1" "Tanh 1" "Sine 0" "ReLU 0"; do
  set -- $cfg
  DBSDE_FUSED=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --activation $1 --steps 20 > gpurun_out/ab_$1_$2.json 2> gpurun_out/ab_$1_$2.err || exit $?
  python - "$1" "$2" <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/ab_{sys.argv[1]}_{sys.argv[2]}.json").read())
print(sys.argv[1], "fused" if sys.argv[2]=="1" else "chain", round(d["ms_per_step"],3), {k:v for k,v in list(d["step_kernel_ms"].items())[:4]})
PY
done
