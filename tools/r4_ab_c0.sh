#!/bin/bash
# bsb: first phase chunk of 6/7/9/10 of 16 units vs even halves
export TMPDIR=/tmp
mkdir -p gpurun_out/abc0
for i in 1 2; do
for v in "X=1" "DBSDE_CHUNK0=6" "DBSDE_CHUNK0=7" "DBSDE_CHUNK0=9" "DBSDE_CHUNK0=10"; do
  env $v timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 100 > gpurun_out/abc0/b.log 2>&1 || { tail -5 gpurun_out/abc0/b.log; exit 1; }
  python - gpurun_out/abc0/b.log "bsb $v $i" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], {n: k[n] for n in list(k)[:3]})
PY
done
done
