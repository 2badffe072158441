#!/bin/bash
export TMPDIR=/tmp
out=gpurun_out/r5a
mkdir -p $out
B="python bench.py --no-cpu-baseline --no-parity"
for cfg in "20 5" "20 50" "100 5" "20 5"; do
  set -- $cfg
  timeout -k 10 300 $B --steps $1 --warmup $2 > $out/b_$1_$2.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/b_$1_$2.json'));print('steps $1 warmup $2', round(d['value']/1e6,2), round(d['ms_per_step'],4), d['roofline']['avg_launch_ms'], d['step_kernel_ms'])"
done
bash tools/r5_prof.sh r5 bsb
