#!/bin/bash
# weight-gradient L2 touch loads two steps ahead: bitwise check against the previous build, A/B (touch / no touch / previous)
export TMPDIR=/tmp
out=gpurun_out/r5ab8
mkdir -p $out
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
for M in 1024 128; do
  timeout -k 10 120 python tools/grad_dump.py $out/new_$M.npy $M || exit 1
  DBSDE_LIB=$PKG/lib/exp/r5pre/libdbsde.so timeout -k 10 120 python tools/grad_dump.py $out/old_$M.npy $M || exit 1
  python -c "import numpy as np; a=np.load('$out/new_$M.npy'); b=np.load('$out/old_$M.npy'); print('M $M bitwise equal:', np.array_equal(a,b), 'max abs diff', float(np.abs(a-b).max()))"
done
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" nopf r5pre || exit 1
