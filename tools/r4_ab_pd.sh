#!/bin/bash
# tn_x3 two-step prefetch (base) vs one step (pd1) on HJB and config 1, after
# the width-256 parity tests
export TMPDIR=/tmp
mkdir -p gpurun_out/abpd
timeout -k 10 300 python -u -m pytest tests/test_gpu_round4.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "w256 or hjb or oned or chunk or splits" > gpurun_out/abpd/tests.txt 2>&1
rc=$?; tail -3 gpurun_out/abpd/tests.txt; [ $rc -le 1 ] || exit $rc
tools/ab_libs.sh "--workload hjb --no-cpu-baseline --no-parity --steps 50" pd1 > gpurun_out/abpd/hjb.txt 2>&1; cat gpurun_out/abpd/hjb.txt
tools/ab_libs.sh "--workload oned --no-cpu-baseline --no-parity --steps 50" pd1 > gpurun_out/abpd/oned.txt 2>&1; cat gpurun_out/abpd/oned.txt
