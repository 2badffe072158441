#!/bin/bash
# config 1 (oned, M=256): one chunk (default by occupancy) vs two chunks with piped chain weight gradients
export TMPDIR=/tmp
out=gpurun_out/r5ab21
mkdir -p $out
for i in 1 2; do
  for ch in 0 2; do
    DBSDE_CHUNKS=$ch timeout -k 10 200 python bench.py --workload oned --no-cpu-baseline --no-parity --steps 60 --warmup 40 > $out/c${ch}_$i.log 2>&1 || { tail -5 $out/c${ch}_$i.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/c${ch}_$i.log').read().strip().split('\n')[-1]); print('chunks=$ch', $i, round(d['ms_per_step'],4), {k: d['step_kernel_ms'][k] for k in list(d['step_kernel_ms'])[:4]})"
  done
done
