#!/bin/bash
# deferred prefetch (default) vs at once (DBSDE_PF_DEFER=0); prefetch tests first
export TMPDIR=/tmp
mkdir -p gpurun_out/abpf
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/abpf/tests.txt 2>&1
rc=$?; tail -2 gpurun_out/abpf/tests.txt; grep -E "FAILED|ERROR" gpurun_out/abpf/tests.txt | head; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for w in bsb basket heston; do
for v in "X=1" "DBSDE_PF_DEFER=0"; do
  env $v timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-parity --steps 30 > gpurun_out/abpf/b.log 2>&1 || { echo fail; tail -5 gpurun_out/abpf/b.log; exit 1; }
  python - gpurun_out/abpf/b.log "$w $v $i" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], {n: k[n] for n in list(k)[:4]})
PY
done
done
done
