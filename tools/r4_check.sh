#!/bin/bash
# Smoke + GPU tests, then bench lines given as "name=args" (bench.py args;
# an optional leading ENV=VAL list before "::" is exported for that line).
# Each step has its own time limit; a crash or timeout stops the script.
out=gpurun_out/chk
mkdir -p $out
: > $out/summary.txt
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $out/steps.log
  case $rc in 0|1) return 0;; *) echo "stopping after $name (rc=$rc)"; tail -30 "$out/$name.log"; exit $rc;; esac
}
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
except Exception as e:
    print(sys.argv[2], "no result", e); sys.exit(0)
k = d["step_kernel_ms"]
print(sys.argv[2], "value %.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"], "frac %.3f" % d["roofline"]["frac"],
      {n: k[n] for n in list(k)[:7]})
PY
}
if [ -z "$SKIP_TESTS" ]; then
  step smoke 300 python __graft_entry__.py smoke
  step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  grep -E "passed|failed" $out/gpu_tests.log | tail -3
fi
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}
  envs=""; args="$rest"
  if [[ "$rest" == *"::"* ]]; then envs=${rest%%::*}; args=${rest#*::}; fi
  env $envs timeout -k 10 400 python bench.py $args > $out/$name.log 2>&1 || { echo "fail $name"; tail -20 $out/$name.log; exit 1; }
  summ $out/$name.log "$name" | tee -a $out/summary.txt
done
