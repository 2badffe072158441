#!/bin/bash
# float4 slab sums in the chain-layout finalize: GPU suite, then A/B on HJB and
# config 1 against the previous library.
export TMPDIR=/tmp
out=gpurun_out/r6s
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/gpu_tests.txt | head -20; exit $rc; }
VARIANTS=head BENCH_ARGS="--workload hjb" tools/r6_ab_phase.sh || exit 1
VARIANTS=head BENCH_ARGS="--workload oned" tools/r6_ab_phase.sh
