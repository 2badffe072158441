#!/bin/bash
# chunk fork / join as stream memory ops (base) vs no-fence events (evnf) vs default events (evdef):
# bitwise check, GPU suite, A/B at M = 1024, M = 128, basket
export TMPDIR=/tmp
out=gpurun_out/r5ab10
mkdir -p $out
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
timeout -k 10 120 python tools/grad_dump.py $out/base.npy 1024 || exit 1
DBSDE_LIB=$PKG/lib/exp/evdef/libdbsde.so timeout -k 10 120 python tools/grad_dump.py $out/evdef.npy 1024 || exit 1
python -c "import numpy as np; a=np.load('$out/base.npy'); b=np.load('$out/evdef.npy'); print('memops vs events bitwise equal:', np.array_equal(a,b))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" evnf evdef || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50 --paths-per-gpu 128" evnf evdef || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 30 --warmup 20 --workload basket" evdef || exit 1
