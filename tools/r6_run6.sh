#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/gpu_tests6.txt 2>&1; rc=$?
tail -1 gpurun_out/r6/gpu_tests6.txt; grep -E "^FAILED|^ERROR" gpurun_out/r6/gpu_tests6.txt | head
[ $rc -eq 0 ] || exit $rc
VARIANTS="notile headlib" bash tools/r6_ab_phase.sh || exit 1
BENCH_ARGS="--paths-per-gpu 128" VARIANTS="notile headlib" bash tools/r6_ab_phase.sh
