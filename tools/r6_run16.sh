#!/bin/bash
# Held-back rollout after the chunk join (beside the step tail): GPU suite,
# then A/B against the previous library at the north star, M = 128, basket,
# Heston.
export TMPDIR=/tmp
out=gpurun_out/r6j
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/gpu_tests.txt | head -20; exit $rc; }
VARIANTS=head tools/r6_ab_phase.sh || exit 1
VARIANTS=head BENCH_ARGS="--paths-per-gpu 128" tools/r6_ab_phase.sh || exit 1
VARIANTS=head BENCH_ARGS="--workload basket" tools/r6_ab_phase.sh || exit 1
VARIANTS=head BENCH_ARGS="--workload heston" tools/r6_ab_phase.sh
