#!/bin/bash
# finalize with two 16-slab groups' loads in flight (base) vs one (prevfin): bitwise, A/B M=1024, M=128
export TMPDIR=/tmp
out=gpurun_out/r5ab15
mkdir -p $out
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
for M in 1024 128; do
  timeout -k 10 120 python tools/grad_dump.py $out/new_$M.npy $M || exit 1
  DBSDE_LIB=$PKG/lib/exp/prevfin/libdbsde.so timeout -k 10 120 python tools/grad_dump.py $out/old_$M.npy $M || exit 1
  python -c "import numpy as np; a=np.load('$out/new_$M.npy'); b=np.load('$out/old_$M.npy'); print('M $M bitwise equal:', np.array_equal(a,b))"
done
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" prevfin || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50 --paths-per-gpu 128" prevfin || exit 1
