#!/bin/bash
# Two-pass rollout for in-step rollouts only: GPU suite, then A/B.
export TMPDIR=/tmp
out=gpurun_out/r6r
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests2.txt 2>&1; rc=$?
tail -2 $out/gpu_tests2.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/gpu_tests2.txt | head -20; exit $rc; }
for args in "" "--paths-per-gpu 128" "--paths-per-gpu 128 --no-prefetch" "--no-prefetch"; do
  for i in 1 2; do
    for v in two one; do
      if [ $v = one ]; then export DBSDE_ROLLOUT2=0; else unset DBSDE_ROLLOUT2; fi
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 100 --warmup 50 $args > $out/run.log 2>&1 || { echo "fail $v $args"; tail -5 $out/run.log; exit 1; }
      python - $out/run.log "$v $i $args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
ph = k.get("fused_phases_pipelined", k.get("fused_fwd_inputgrad", 0))
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], "rollout %.4f" % k.get("rollout", 0), "phases %.4f" % ph, flush=True)
PY
    done
  done
done
