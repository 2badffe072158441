#!/bin/bash
# stream-ordering event flags: no system-scope fence / device-scope release vs default; bitwise check; A/B
export TMPDIR=/tmp
out=gpurun_out/r5ab9
mkdir -p $out
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
timeout -k 10 120 python tools/grad_dump.py $out/base.npy 1024 || exit 1
for v in evnofence evdev; do
  DBSDE_LIB=$PKG/lib/exp/$v/libdbsde.so timeout -k 10 120 python tools/grad_dump.py $out/$v.npy 1024 || exit 1
  python -c "import numpy as np; a=np.load('$out/base.npy'); b=np.load('$out/$v.npy'); print('$v bitwise equal:', np.array_equal(a,b))"
done
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" evnofence evdev || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50 --paths-per-gpu 128" evnofence evdev || exit 1
