#!/bin/bash
# Smoke + GPU tests, then interleaved A/Bs of the phase-kernel forms on the
# headline bench (DBSDE_NT / DBSDE_ADOT) and of the fused width-256 kernels
# against the per-layer chain on config 4 (DBSDE_FUSED=0).  Each step has its
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
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
except Exception as e:
    print(sys.argv[2], "no result", e); sys.exit(0)
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], "frac %.3f" % d["roofline"]["frac"],
      {n: k[n] for n in list(k)[:6]})
PY
}
if [ -z "$SKIP_TESTS" ]; then
  step smoke 300 python __graft_entry__.py smoke
  step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  grep -E "passed|failed" gpurun_out/abnt/gpu_tests.log | tail -3
fi
for i in 1 2; do
  for v in "DBSDE_NT=1" "DBSDE_NT=2" "DBSDE_NT=2 DBSDE_ADOT=1"; do
    tag=$(echo $v | tr ' =' '_-')
    env $v timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity > gpurun_out/abnt/b_${tag}_$i.log 2>&1 || { echo "fail $v"; tail -20 gpurun_out/abnt/b_${tag}_$i.log; exit 1; }
    summ gpurun_out/abnt/b_${tag}_$i.log "$v run $i" | tee -a gpurun_out/abnt/summary.txt
  done
  for v in "DBSDE_W256=0" "DBSDE_W256=1"; do
    env $v timeout -k 10 300 python bench.py --workload hjb --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abnt/h_${v}_$i.log 2>&1 || { echo "fail hjb $v"; tail -20 gpurun_out/abnt/h_${v}_$i.log; exit 1; }
    summ gpurun_out/abnt/h_${v}_$i.log "hjb $v run $i" | tee -a gpurun_out/abnt/summary.txt
  done
done
