#!/bin/bash
# strong shapes: chunk count by occupancy (0) vs always two, on the value-op / held-back-prefetch build
export TMPDIR=/tmp
out=gpurun_out/r5ab22
mkdir -p $out
for i in 1 2; do
  for m in 512 256; do
    for ch in 0 2; do
      DBSDE_CHUNKS=$ch timeout -k 10 200 python bench.py --paths-per-gpu $m --no-cpu-baseline --no-parity --steps 100 --warmup 50 > $out/m${m}_c${ch}_$i.log 2>&1 || { tail -5 $out/m${m}_c${ch}_$i.log; exit 1; }
      python -c "import json; d=json.loads(open('$out/m${m}_c${ch}_$i.log').read().strip().split('\n')[-1]); print('M=$m chunks=$ch', $i, round(d['ms_per_step'],4))"
    done
  done
done
