#!/bin/bash
# GPU suite on the stream-restructured build, then interleaved A/B against the
# previous commit's library (lib/exp/r5pre) and a kernel trace of the new one
export TMPDIR=/tmp
out=gpurun_out/r5ab3
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -3 $out/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" r5pre || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 20 --warmup 5" r5pre || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 30 --warmup 10 --workload basket" r5pre || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr -o run --output-format csv -- python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 > $out/tr.log 2>&1 || exit 1
python tools/steps_view.py $(ls $out/tr/*/run_kernel_trace.csv $out/tr/run_kernel_trace.csv 2>/dev/null | head -1)
