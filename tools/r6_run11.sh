#!/bin/bash
# Weight-gradient workgroups grouped by shared operands (launch_tnw order) vs
# index order (DBSDE_TNW_ORDER=0): GPU suite, then interleaved A/B.
export TMPDIR=/tmp
out=gpurun_out/r6o
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
tail -2 $out/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/gpu_tests.txt | head -20; exit $rc; }
for args in "" "--paths-per-gpu 128" "--workload basket"; do
  for i in 1 2; do
    for v in grouped index; do
      if [ $v = index ]; then export DBSDE_TNW_ORDER=0; else unset DBSDE_TNW_ORDER; fi
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 100 --warmup 50 $args > $out/run.log 2>&1 || { echo "fail $v $args"; tail -5 $out/run.log; exit 1; }
      python - $out/run.log "$v $i $args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], "tnw %.4f" % k["tn_weight_grad"], flush=True)
PY
    done
  done
done
