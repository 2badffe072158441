#!/bin/bash
# tn_x3 at three waves per SIMD (w3, 168 registers) vs two (base)
export TMPDIR=/tmp
mkdir -p gpurun_out/abw3
DBSDE_LIB=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd/lib/exp/w3/libdbsde.so timeout -k 10 300 python -u -m pytest tests/test_gpu_round4.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "w256 or hjb or oned or FC or Resnet or splits" > gpurun_out/abw3/tests.txt 2>&1
rc=$?; tail -2 gpurun_out/abw3/tests.txt; [ $rc -eq 0 ] || exit $rc
tools/ab_libs.sh "--workload hjb --no-cpu-baseline --no-parity --steps 50" w3 > gpurun_out/abw3/hjb.txt 2>&1; cat gpurun_out/abw3/hjb.txt
tools/ab_libs.sh "--workload oned --no-cpu-baseline --no-parity --steps 50" w3 > gpurun_out/abw3/oned.txt 2>&1; cat gpurun_out/abw3/oned.txt
