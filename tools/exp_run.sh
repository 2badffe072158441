#!/bin/bash
# Bench each experiment library of tools/build_exp.sh (through DBSDE_LIB) and
# print ms/step and the two phase kernels' ms.   tools/exp_run.sh base nostore ...
for v in "$@"; do
  DBSDE_LIB=$PWD/exp/libdbsde_$v.so timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 \
    > gpurun_out/exp_$v.json 2> gpurun_out/exp_$v.err || { echo "FAIL $v"; tail -5 gpurun_out/exp_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/exp_$v.json').read().strip().splitlines()[-1]); k=d['step_kernel_ms']
print('$v', round(d['ms_per_step'], 4), 'A', k.get('fused_fwd_inputgrad'), 'C', k.get('fused_tangent_reverse'), 'tnw', k.get('tn_weight_grad'))"
done
