#!/bin/bash
# GPU suite, then the clip-path workloads
export TMPDIR=/tmp
out=gpurun_out/opt
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/tests.txt 2>&1
rc=$?; tail -2 $out/tests.txt; grep -E "FAILED|ERROR" $out/tests.txt | head; [ $rc -eq 0 ] || exit $rc
for w in oned hjb basket heston; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-parity --steps 50 > $out/b.log 2>&1 || { tail -5 $out/b.log; exit 1; }
  python - $out/b.log "$w" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], k)
PY
done
