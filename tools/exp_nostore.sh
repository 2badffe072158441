#!/bin/bash
L=deep-neural-network-solutions-for-partial-differential-equations_amd/lib/libdbsde.so
cp $L /tmp/keep.so
for v in nostore nobstage nobstage_nostore; do
  cp exp/libdbsde_$v.so $L
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/exp_$v.json 2>/dev/null || { cp /tmp/keep.so $L; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/exp_$v.json')); k=d['step_kernel_ms']; print('$v', round(d['ms_per_step'],3), 'A', k.get('fused_fwd_inputgrad'), 'C', k.get('fused_tangent_reverse'))"
done
cp /tmp/keep.so $L
