#!/bin/bash
# GPU suite; A/B: tail-kernel load rounds vs the previous commit (r5pre); tnw split ablations (timing only)
export TMPDIR=/tmp
out=gpurun_out/r5ab5
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" r5pre nosplitb nosplit || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50 --paths-per-gpu 128" r5pre || exit 1
