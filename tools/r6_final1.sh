#!/bin/bash
# Round-6 final pass 1: GPU suite, tilefin A/B at M = 128 against the previous
# library (lib/exp/head), kernel stats + counter passes at the north star and
# at M = 128, and the stream-order auto-detection under rocprofv3 --pmc
# (no DBSDE_STREAM_ORDER override).
export TMPDIR=/tmp
out=gpurun_out/r6
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/gpu_tests_final.txt 2>&1; rc=$?
tail -3 $out/gpu_tests_final.txt
[ $rc -eq 0 ] || exit $rc
VARIANTS=head BENCH_ARGS="--paths-per-gpu 128" tools/r6_ab_phase.sh || exit 1
tools/profile_round.sh r6 bsb || exit 1
tools/profile_round.sh r6m128 bsb --paths-per-gpu 128 || exit 1
mkdir -p gpurun_out/prof_r6_autodetect
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d gpurun_out/prof_r6_autodetect/pmc -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/prof_r6_autodetect/run.log 2>&1; rc=$?
echo "autodetect rc=$rc"; grep "dbsde:" gpurun_out/prof_r6_autodetect/run.log
exit $rc
