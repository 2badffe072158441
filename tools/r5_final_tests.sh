#!/bin/bash
# Round-end evidence 1/2: smoke and the whole GPU test suite
export TMPDIR=/tmp
out=gpurun_out/final5
mkdir -p $out
timeout -k 10 300 python __graft_entry__.py smoke > $out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 $out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
grep -E "passed|failed" $out/gpu_tests.txt | tail -3; grep -E "FAILED|ERROR" $out/gpu_tests.txt | head -20
exit $rc
