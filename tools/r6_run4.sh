#!/bin/bash
# tests + A/B of the tile-order operand stores (north star and M = 128)
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/gpu_tests4.txt 2>&1; rc=$?
tail -2 gpurun_out/r6/gpu_tests4.txt; grep -E "FAILED|ERROR" gpurun_out/r6/gpu_tests4.txt | head
[ $rc -eq 0 ] || exit $rc
VARIANTS="notile" bash tools/r6_ab_phase.sh || exit 1
BENCH_ARGS="--paths-per-gpu 128" VARIANTS="notile" bash tools/r6_ab_phase.sh || exit 1
timeout -k 10 300 python tools/clock_probe.py --steps 100 --warmup 0 --out gpurun_out/r6/clocks.json > gpurun_out/r6/clocks.log 2>&1; rc=$?; head -2 gpurun_out/r6/clocks.log; exit $rc
