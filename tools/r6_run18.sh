#!/bin/bash
# Clip norm from the finalize's partials (default) vs sqnorm_kernel's pass
# (DBSDE_SQNORM_PASS=1): GPU suite, then interleaved A/B on the clip workloads.
export TMPDIR=/tmp
out=gpurun_out/r6q
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/gpu_tests.txt | head -20; exit $rc; }
for w in basket hjb oned; do
  for i in 1 2; do
    for v in fin pass; do
      if [ $v = pass ]; then export DBSDE_SQNORM_PASS=1; else unset DBSDE_SQNORM_PASS; fi
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --workload $w --steps 100 --warmup 30 > $out/run.log 2>&1 || { echo "fail $v $w"; tail -5 $out/run.log; exit 1; }
      python - $out/run.log "$w $v $i" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], "sqnorm %.4f" % k.get("grad_sqnorm", 0), "optim %.4f" % k.get("optimizer", 0), "fin %.4f" % k.get("grad_finalize", 0), flush=True)
PY
    done
  done
done
