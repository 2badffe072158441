#!/bin/bash
# chain weight gradients piped per chunk (base) vs after the section (notnp): tests, A/B HJB, bsb
export TMPDIR=/tmp
out=gpurun_out/r5ab20
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/gpu_tests.txt | head; exit $rc; }
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 40 --warmup 30 --workload hjb" notnp || exit 1
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100 --warmup 50" notnp || exit 1
