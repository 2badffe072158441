#!/bin/bash
# Slice-group sums in the weight-gradient kernels (S / 4 slabs): GPU suite,
# then A/B against the previous library at M = 1024 and M = 128.
export TMPDIR=/tmp
out=gpurun_out/r6
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests10.txt 2>&1; rc=$?
tail -3 $out/gpu_tests10.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/gpu_tests10.txt | head -20; exit $rc; }
VARIANTS=head tools/r6_ab_phase.sh || exit 1
VARIANTS=head BENCH_ARGS="--paths-per-gpu 128" tools/r6_ab_phase.sh
