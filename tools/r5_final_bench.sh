#!/bin/bash
# Round-end evidence 2/2: the headline bench line (CPU baseline, parity
# trajectory), the other BASELINE workloads and the strong-scaling shapes
export TMPDIR=/tmp
out=gpurun_out/final5
mkdir -p $out
timeout -k 10 600 python bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json; tail -c 400 $out/bench.json
: > $out/workloads.jsonl
for wl in oned basket hjb heston; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > $out/wl_$wl.log 2>&1 || { echo "fail $wl"; tail -20 $out/wl_$wl.log; exit 1; }
  tail -1 $out/wl_$wl.log >> $out/workloads.jsonl
done
: > $out/shapes.jsonl
for m in 128 256 512; do
  timeout -k 10 300 python bench.py --paths-per-gpu $m --no-cpu-baseline --no-parity --steps 100 > $out/m$m.log 2>&1 || { echo "fail m$m"; exit 1; }
  tail -1 $out/m$m.log >> $out/shapes.jsonl
done
python - <<'PY'
import json
for f in ["gpurun_out/final5/workloads.jsonl", "gpurun_out/final5/shapes.jsonl"]:
    for l in open(f):
        d = json.loads(l)
        print(d["config"].get("name", d["config"].get("workload"))[:40], d["config"].get("paths_per_gpu"), "%.4g" % d["value"], "ms %.4f" % d["ms_per_step"], "frac %.3f" % d["roofline"]["frac"])
PY
