#!/bin/bash
# store-path ablations + kernel stats (rollout kernel durations) at M = 1024 and 128
export TMPDIR=/tmp
VARIANTS="ab2048 ab4096" bash tools/r6_ab_phase.sh || exit 1
for m in 1024 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6prof/m$m -o run --output-format csv -- python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 --paths-per-gpu $m > gpurun_out/r6prof/m$m.log 2>&1 || { echo "prof $m failed"; tail -5 gpurun_out/r6prof/m$m.log; exit 1; }
  f=$(find gpurun_out/r6prof/m$m -name "*kernel_stats.csv" | head -1)
  echo "== M=$m"; python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print("%-60s n=%6s avg_us=%8.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
