#!/bin/bash
# Round-5 evidence on the current tree: smoke + GPU suite, bench lines (driver window and
# settled window, workloads, strong shapes), kernel stats + counter passes (bsb, M = 128)
export TMPDIR=/tmp
bash tools/r5_final_tests.sh || exit $?
bash tools/r5_final_bench.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 100 --warmup 50 > gpurun_out/final5/bench_100_50.log 2>&1 || exit 1
tail -1 gpurun_out/final5/bench_100_50.log > gpurun_out/final5/bench_100_50.json
bash tools/profile_round.sh r5 bsb || exit $?
bash tools/profile_round.sh r5m128 bsb --paths-per-gpu 128 || exit $?
