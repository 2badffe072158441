#!/bin/bash
# rollout prefetch: default (launched at the step start, overlapping the phases) vs in-step
export TMPDIR=/tmp
mkdir -p gpurun_out/pf
for i in 1 2; do
for w in bsb basket; do
for a in "" "--no-prefetch"; do
  timeout -k 10 200 python bench.py --workload $w $a --no-cpu-baseline --no-parity --steps 30 > gpurun_out/pf/b.log 2>&1 || { tail -5 gpurun_out/pf/b.log; exit 1; }
  python - gpurun_out/pf/b.log "$w $a $i" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], {n: k[n] for n in list(k)[:4]})
PY
done
done
done
