#!/bin/bash
# Smoke + GPU tests, then an interleaved A/B of the one-tile (DBSDE_NT=1) and
# two-tile (DBSDE_NT=2) phase kernels on the headline bench.  Each step has its
# own time limit; a crash or timeout stops the script.
mkdir -p gpurun_out/abnt
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/abnt/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/abnt/steps.log
  case $rc in 0|1) return 0;; *) echo "stopping after $name (rc=$rc)"; tail -30 "gpurun_out/abnt/$name.log"; exit $rc;; esac
}
if [ -z "$SKIP_TESTS" ]; then
  step smoke 300 python __graft_entry__.py smoke
  step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  grep -E "passed|failed" gpurun_out/abnt/gpu_tests.log | tail -3
fi
for i in 1 2; do
  for nt in 1 2; do
    DBSDE_NT=$nt step bench_nt${nt}_$i 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity ${BENCH_ARGS}
    python - gpurun_out/abnt/bench_nt${nt}_$i.log "nt$nt run $i" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], "frac %.3f" % d["roofline"]["frac"],
      {n: k[n] for n in list(k)[:6]})
PY
  done
done
