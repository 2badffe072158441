#!/bin/bash
# Round-6 GPU check: environment probe (stream-order selection), smoke, the
# whole GPU suite, then the default bench line.
export TMPDIR=/tmp
out=gpurun_out/r6
mkdir -p $out
env | grep -E "^(ROCP|HSA_TOOLS|AMD_SERIALIZE|HIP_LAUNCH_BLOCKING|DBSDE_)" > $out/env_probe.txt || true
python -c "
import sys; sys.path.insert(0, '.')
import importlib; p = importlib.import_module('deep-neural-network-solutions-for-partial-differential-equations_amd')
print('order_by_events', p._lib.load().dbsde_stream_order_by_events(None))" >> $out/env_probe.txt 2>&1
cat $out/env_probe.txt
timeout -k 10 300 python __graft_entry__.py smoke > $out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 $out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $out/gpu_tests.txt 2>&1; rc=$?
grep -E "passed|failed" $out/gpu_tests.txt | tail -3; grep -E "FAILED|ERROR" $out/gpu_tests.txt | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py > $out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 600 $out/bench.log
