#!/bin/bash
# Balanced block -> wave assignment in the correlated rollout: GPU suite, then
# basket A/B (in-step and prefetched) against the previous library.
export TMPDIR=/tmp
out=gpurun_out/r6
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests12.txt 2>&1; rc=$?
tail -2 $out/gpu_tests12.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/gpu_tests12.txt | head -20; exit $rc; }
VARIANTS=head BENCH_ARGS="--workload basket --no-prefetch" tools/r6_ab_phase.sh || exit 1
VARIANTS=head BENCH_ARGS="--workload basket" tools/r6_ab_phase.sh
