#!/bin/bash
# GPU suite, interleaved A/B of the tail-kernel load rounds against the previous commit (lib/exp/r5pre),
# and the new build's kernel stats
export TMPDIR=/tmp
out=gpurun_out/r5ab4
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" r5pre || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50 --paths-per-gpu 128" r5pre || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/st -o run --output-format csv -- python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 > $out/st.log 2>&1 || exit 1
f=$(ls $out/st/*/run_kernel_stats.csv $out/st/run_kernel_stats.csv 2>/dev/null | head -1)
cut -d, -f1-4 $f | sed 's/(dbsde[^"]*//' | head -14
