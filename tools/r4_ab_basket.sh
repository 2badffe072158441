#!/bin/bash
# basket (M=4096) and bsb: phase chunk layouts with the weight-gradient slices
# piped behind every chunk; the chunk-invariance test first
export TMPDIR=/tmp
mkdir -p gpurun_out/abbk
timeout -k 10 300 python -u -m pytest tests/test_gpu_round4.py -q --timeout 120 --timeout-method thread -k "chunk" > gpurun_out/abbk/tests.txt 2>&1
rc=$?; tail -2 gpurun_out/abbk/tests.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for w in basket bsb; do
for v in "X=1" "DBSDE_CHUNKS=3" "DBSDE_CHUNKS=4"; do
  env $v timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-parity --steps 30 > gpurun_out/abbk/b.log 2>&1 || { echo fail $v; tail -5 gpurun_out/abbk/b.log; exit 1; }
  python - gpurun_out/abbk/b.log "$w $v $i" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], {n: k[n] for n in list(k)[:4]})
PY
done
done
done
