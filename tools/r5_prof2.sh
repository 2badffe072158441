#!/bin/bash
# the value-wait fallback under counter collection (auto-detected), then the round-5 profiles
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_chk
timeout -k 10 300 python -u -m pytest tests/test_gpu_round5.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prof_chk/t.txt 2>&1; rc=$?
tail -2 gpurun_out/prof_chk/t.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_chk/f -o run --output-format csv -- python bench.py --no-cpu-baseline --no-parity --steps 3 --warmup 1 > gpurun_out/prof_chk/f.log 2>&1; rc=$?
echo "auto-detected pmc pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh r5 bsb || exit $?
bash tools/profile_round.sh r5m128 bsb --paths-per-gpu 128 || exit $?
