#!/bin/bash
# stream value waits as CP packets (GPU_STREAMOPS_CP_WAIT=1) vs blit kernels: microbenchmark + bench
export TMPDIR=/tmp
out=gpurun_out/r5ab14
mkdir -p $out
timeout -k 10 60 tools/ubench/stream_gaps 2 > $out/ub_kernel.txt 2>&1 || exit 1
GPU_STREAMOPS_CP_WAIT=1 timeout -k 10 60 tools/ubench/stream_gaps 2 > $out/ub_cp.txt 2>&1 || exit 1
head -3 $out/ub_kernel.txt $out/ub_cp.txt
for i in 1 2; do
  for v in kernel cp; do
    if [ $v = cp ]; then export GPU_STREAMOPS_CP_WAIT=1; else unset GPU_STREAMOPS_CP_WAIT; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 100 --warmup 50 > $out/${v}_$i.log 2>&1 || { echo "fail $v"; tail -5 $out/${v}_$i.log; exit 1; }
    python -c "import json; d=json.loads(open('$out/${v}_$i.log').read().strip().split('\n')[-1]); print('$v $i', round(d['ms_per_step'],4))"
  done
done
