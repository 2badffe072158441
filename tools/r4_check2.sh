#!/bin/bash
# the GPU suite, then the headline and the small shapes (fused RtR + packing)
export TMPDIR=/tmp
out=gpurun_out/chk2
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/tests.txt 2>&1
rc=$?; tail -3 $out/tests.txt; grep -E "FAILED|ERROR" $out/tests.txt | head; [ $rc -eq 0 ] || exit $rc
for a in "" "--paths-per-gpu 128" "--paths-per-gpu 256"; do
  timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-parity --steps 100 > $out/b.log 2>&1 || { tail -5 $out/b.log; exit 1; }
  python - $out/b.log "$a" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print("bsb", sys.argv[2], "ms/step %.4f" % d["ms_per_step"], d["step_kernel_ms"])
PY
done
