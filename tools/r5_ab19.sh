#!/bin/bash
# chunk fork written by the first phase-A launch (base) vs a value-write launch (forkw)
export TMPDIR=/tmp
out=gpurun_out/r5ab19
mkdir -p $out
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
timeout -k 10 120 python tools/grad_dump.py $out/new.npy 1024 || exit 1
DBSDE_LIB=$PKG/lib/exp/forkw/libdbsde.so timeout -k 10 120 python tools/grad_dump.py $out/old.npy 1024 || exit 1
python -c "import numpy as np; a=np.load('$out/new.npy'); b=np.load('$out/old.npy'); print('bitwise equal:', np.array_equal(a,b))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" forkw || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50 --paths-per-gpu 512" forkw || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 40 --warmup 30 --workload heston" forkw || exit 1
bash tools/r5_tr.sh fk "DBSDE_X=1" --steps 60 --warmup 40 || exit 1
