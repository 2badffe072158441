#!/bin/bash
# prefetched diagonal rollout on the chunked step's second stream (base) vs on pf_stream (nodefer)
export TMPDIR=/tmp
out=gpurun_out/r5ab17
mkdir -p $out
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
timeout -k 10 120 python tools/grad_dump.py $out/new.npy 1024 || exit 1
DBSDE_LIB=$PKG/lib/exp/nodefer/libdbsde.so timeout -k 10 120 python tools/grad_dump.py $out/old.npy 1024 || exit 1
python -c "import numpy as np; a=np.load('$out/new.npy'); b=np.load('$out/old.npy'); print('bitwise equal:', np.array_equal(a,b))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" nodefer || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50 --paths-per-gpu 128" nodefer || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50 --paths-per-gpu 512" nodefer || exit 1
bash tools/r5_tr.sh def "DBSDE_X=1" --steps 60 --warmup 40 || exit 1
