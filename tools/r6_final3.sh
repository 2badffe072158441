#!/bin/bash
# Round-6 counter tables for the other workloads: kernel
# stats + FETCH / WRITE / SQ passes of basket, HJB and config 1.
export TMPDIR=/tmp
for w in basket hjb oned; do tools/profile_round.sh r6 $w || exit 1; done
mkdir -p gpurun_out/r6f
timeout -k 10 300 python tools/plugin_bench.py > gpurun_out/r6f/plugin_bench.log 2>&1 || { tail -20 gpurun_out/r6f/plugin_bench.log; exit 1; }
cat gpurun_out/r6f/plugin_bench.log
