#!/bin/bash
# A/Bs: piece vmcnt counts (vm0 = earlier counts), HJB one-tile fragment pairs
# (p2np = none), tn_x3 XCD order (xcd0 = none); strong-scaling shapes with the
# occupancy-chosen chunk count against two chunks
export TMPDIR=/tmp
mkdir -p gpurun_out/ablib
timeout -k 10 400 python -u -m pytest tests/test_gpu_round4.py -x -v --timeout 120 --timeout-method thread -k "width256 or chunk" > gpurun_out/ablib/tests.txt 2>&1
rc=$?; tail -15 gpurun_out/ablib/tests.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --workload oned --no-cpu-baseline --no-parity --steps 50 > gpurun_out/ablib/oned.log 2>&1 && tail -c 700 gpurun_out/ablib/oned.log
timeout -k 10 120 tools/ubench/piece_x3 > gpurun_out/ablib/piece5.txt 2>&1 || exit 1
tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100" vm0 tnwchain > gpurun_out/ablib/bsb.txt 2>&1 || { cat gpurun_out/ablib/bsb.txt; exit 1; }
cat gpurun_out/ablib/bsb.txt
tools/ab_libs.sh "--workload hjb --no-cpu-baseline --no-parity --steps 50" p2np xcd0 > gpurun_out/ablib/hjb.txt 2>&1 || { cat gpurun_out/ablib/hjb.txt; exit 1; }
cat gpurun_out/ablib/hjb.txt
for m in 128 256 512; do
  for ch in 0 2; do
    DBSDE_CHUNKS=$ch timeout -k 10 200 python bench.py --paths-per-gpu $m --no-cpu-baseline --no-parity --steps 100 > gpurun_out/ablib/m${m}_c$ch.log 2>&1 || { echo fail m$m; exit 1; }
    python - gpurun_out/ablib/m${m}_c$ch.log "M=$m chunks=$ch" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], {n: k[n] for n in list(k)[:9]})
PY
  done
done
