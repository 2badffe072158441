#!/bin/bash
# tests + A/B of the spread stores and the step-parallel rollout (north star and M = 128)
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/gpu_tests2.txt 2>&1; rc=$?
tail -2 gpurun_out/r6/gpu_tests2.txt; grep -E "FAILED|ERROR" gpurun_out/r6/gpu_tests2.txt | head
[ $rc -eq 0 ] || exit $rc
VARIANTS="nospread rs0" bash tools/r6_ab_phase.sh || exit 1
BENCH_ARGS="--paths-per-gpu 128" VARIANTS="nospread rs0" bash tools/r6_ab_phase.sh
