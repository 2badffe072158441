#!/bin/bash
for cfg in "32 64" "16 64" "16 128" "32 128" "16 256"; do
  set -- $cfg
  DBSDE_TN_KC=$1 DBSDE_TN_SPLITS=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/tn_$1_$2.json 2>/dev/null || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/tn_$1_$2.json')); k=d['step_kernel_ms']
print('KC=$1 S=$2', round(d['ms_per_step'],3), 'tn', k.get('tn_weight_grad'), 'fin', k.get('grad_finalize'))"
done
