#!/bin/bash
# Round-5 evidence on the final tree: smoke + GPU suite, bench lines (default window with CPU
# baseline and parity, the driver's 20/5 window twice, the settled 100/50 window, workloads,
# strong shapes).  Kernel stats / counters: tools/r5_prof2.sh (kernels unchanged since).
export TMPDIR=/tmp
bash tools/r5_final_tests.sh || exit $?
bash tools/r5_final_bench.sh || exit $?
o=gpurun_out/final5
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench_20_5_$i.log 2>&1 || exit 1
  tail -1 $o/bench_20_5_$i.log > $o/bench_20_5_$i.json
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 100 --warmup 50 > $o/bench_100_50.log 2>&1 || exit 1
tail -1 $o/bench_100_50.log > $o/bench_100_50.json
python - <<'PY'
import json
for f in ["bench.json", "bench_20_5_1.json", "bench_20_5_2.json", "bench_100_50.json"]:
    d = json.loads(open("gpurun_out/final5/" + f).read())
    print(f, d["steps"], d["warmup"], "%.4f ms" % d["ms_per_step"], "%.2f M" % (d["value"] / 1e6), "frac %.3f" % d["roofline"]["frac"])
PY
