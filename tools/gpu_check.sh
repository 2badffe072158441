#!/bin/bash
# GPU-box validation: smoke + parity tests, then optional named steps given as
# "name=command".  Each step has its own time limit; a crash, fault or timeout
# (any rc other than 0/1) stops the script.
#   tools/gpu_check.sh ["bench=python bench.py --steps 20 --warmup 5"] ...
mkdir -p gpurun_out
: > gpurun_out/steps.log
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log
  case $rc in 0|1) return 0;; *) echo "stopping after $name (rc=$rc)"; tail -30 "gpurun_out/$name.log"; exit $rc;; esac
}
if [ -z "$SKIP_TESTS" ]; then
  step smoke 300 python __graft_entry__.py smoke
  step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3
fi
export TMPDIR=/tmp
for extra in "$@"; do
  step "${extra%%=*}" 600 bash -c "${extra#*=}"
done
