#!/bin/bash
# A/B: base library vs the new in-tree one, bench at M=1024 and M=128
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for i in 1 2; do
for v in base new; do
  if [ $v = base ]; then export DBSDE_LIB=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd/lib/exp/libdbsde_base.so; else unset DBSDE_LIB; fi
  for m in 1024 128; do
    timeout -k 10 200 python bench.py --paths-per-gpu $m --steps 30 --warmup 10 --no-cpu-baseline --no-parity > gpurun_out/ab/${v}_${m}_$i.log 2>&1 || { echo "fail $v $m"; exit 1; }
    echo "$v $m $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/${v}_${m}_$i.log) $(grep -o '"fused_phases_pipelined": [0-9.]*' gpurun_out/ab/${v}_${m}_$i.log)"
  done
done
done
