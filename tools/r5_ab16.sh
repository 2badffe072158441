#!/bin/bash
# prefetched rollout ordered through the join (base) vs its own wait before phase A (prevj)
export TMPDIR=/tmp
out=gpurun_out/r5ab16
mkdir -p $out
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
timeout -k 10 120 python tools/grad_dump.py $out/new.npy 1024 || exit 1
DBSDE_LIB=$PKG/lib/exp/prevj/libdbsde.so timeout -k 10 120 python tools/grad_dump.py $out/old.npy 1024 || exit 1
python -c "import numpy as np; a=np.load('$out/new.npy'); b=np.load('$out/old.npy'); print('bitwise equal:', np.array_equal(a,b))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" prevj || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 30 --warmup 20 --workload basket" prevj || exit 1
