#!/bin/bash
for S in 32 64 96 128; do
  DBSDE_TN_SPLITS=$S timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/tn_$S.json 2>/dev/null || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/tn_$S.json')); k=d['step_kernel_ms']
print('S=$S', round(d['ms_per_step'],3), 'tn', k.get('tn_weight_grad'), 'fin', k.get('grad_finalize'), 'A', k.get('fused_fwd_inputgrad'), 'C', k.get('fused_tangent_reverse'))"
done
