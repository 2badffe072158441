#!/bin/bash
# HJB / config 1: one-tile fragment pairs (p2np = none), tn_x3 XCD order
# (xcd0 = none), chunk layouts; the oned workload line
export TMPDIR=/tmp
mkdir -p gpurun_out/ablib
timeout -k 10 200 python bench.py --workload oned --no-cpu-baseline --no-parity --steps 50 > gpurun_out/ablib/oned.log 2>&1 && tail -c 700 gpurun_out/ablib/oned.log
tools/ab_libs.sh "--workload hjb --no-cpu-baseline --no-parity --steps 50" p2np xcd0 > gpurun_out/ablib/hjb.txt 2>&1 || { cat gpurun_out/ablib/hjb.txt; exit 1; }
cat gpurun_out/ablib/hjb.txt
for v in "DBSDE_CHUNKS=3" "DBSDE_CHUNKS=4" "DBSDE_CHUNK0=12"; do
  env $v timeout -k 10 200 python bench.py --workload hjb --no-cpu-baseline --no-parity --steps 50 > gpurun_out/ablib/hjb_$v.log 2>&1 || { echo fail $v; exit 1; }
  python - gpurun_out/ablib/hjb_$v.log "hjb $v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], {n: k[n] for n in list(k)[:4]})
PY
done
timeout -k 10 120 tools/ubench/piece_x3 > gpurun_out/ablib/piece5.txt 2>&1
