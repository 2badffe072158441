#!/bin/bash
# A/B of exp builds (lib/exp/<name>/libdbsde.so) against the in-tree library:
# bench.py at the headline shape, alternating, two rounds.
#   tools/ab_variants.sh name1 name2 ...
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
L=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd/lib/exp
for i in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then unset DBSDE_LIB; else export DBSDE_LIB=$L/$v/libdbsde.so; fi
    timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity ${AB_ARGS} > gpurun_out/ab/${v}_$i.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/ab/${v}_$i.log; exit 1; }
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/${v}_$i.log) $(grep -o '"step_kernel_ms": {[^}]*}' gpurun_out/ab/${v}_$i.log)"
  done
done
