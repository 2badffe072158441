#!/bin/bash
# chain weight-gradient rows per split: 128 (base) vs 512 (s512), with the
# output-layer GEMV; after the chain/width-256 parity tests
export TMPDIR=/tmp
mkdir -p gpurun_out/absp
timeout -k 10 300 python -u -m pytest tests/test_gpu_round4.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "w256 or hjb or oned or chunk or splits or chain or FC or Resnet" > gpurun_out/absp/tests.txt 2>&1
rc=$?; tail -3 gpurun_out/absp/tests.txt; grep FAILED gpurun_out/absp/tests.txt | head; [ $rc -le 1 ] || exit $rc
tools/ab_libs.sh "--workload hjb --no-cpu-baseline --no-parity --steps 50" s512 > gpurun_out/absp/hjb.txt 2>&1; cat gpurun_out/absp/hjb.txt
tools/ab_libs.sh "--workload oned --no-cpu-baseline --no-parity --steps 50" s512 > gpurun_out/absp/oned.txt 2>&1; cat gpurun_out/absp/oned.txt
