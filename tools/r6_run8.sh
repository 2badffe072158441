#!/bin/bash
# Double-buffered row stage in the correlated rollout: GPU suite, then basket
# A/B (prefetched and in-step) against the previous library (lib/exp/head).
export TMPDIR=/tmp
out=gpurun_out/r6
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests8.txt 2>&1; rc=$?
tail -3 $out/gpu_tests8.txt
[ $rc -eq 0 ] || exit $rc
VARIANTS=head BENCH_ARGS="--workload basket --no-prefetch" tools/r6_ab_phase.sh || exit 1
VARIANTS=head BENCH_ARGS="--workload basket" tools/r6_ab_phase.sh
