#!/bin/bash
# LDS-transposed weight-gradient operands: bitwise check against the previous build, GPU suite, A/B
export TMPDIR=/tmp
out=gpurun_out/r5ab7
mkdir -p $out
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
for M in 1024 128; do
  timeout -k 10 120 python tools/grad_dump.py $out/new_$M.npy $M || exit 1
  DBSDE_LIB=$PKG/lib/exp/r5pre/libdbsde.so timeout -k 10 120 python tools/grad_dump.py $out/old_$M.npy $M || exit 1
  python -c "import numpy as np; a=np.load('$out/new_$M.npy'); b=np.load('$out/old_$M.npy'); print('M $M bitwise equal:', np.array_equal(a,b), 'max abs diff', float(np.abs(a-b).max()))"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" r5pre || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 30 --warmup 10 --workload basket" r5pre || exit 1
