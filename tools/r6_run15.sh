#!/bin/bash
# Workgroup size of the prefetched single-pass rollout (DBSDE_R4_WG), interleaved.
export TMPDIR=/tmp
out=gpurun_out/r6w
mkdir -p $out
for args in "" "--paths-per-gpu 128"; do
  for i in 1 2; do
    for v in 256 128 64; do
      export DBSDE_R4_WG=$v
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
