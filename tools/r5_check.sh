#!/bin/bash
# Round-5 check: smoke, the whole GPU suite, the driver's bench command beside
# the default window, and the long-run accuracy runs (tools/long_run.py)
export TMPDIR=/tmp
out=gpurun_out/r5
mkdir -p $out
timeout -k 10 300 python __graft_entry__.py smoke > $out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $out/gpu_tests.txt 2>&1; rc=$?
grep -E "passed|failed" $out/gpu_tests.txt | tail -2; grep -E "FAILED|ERROR" $out/gpu_tests.txt | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench_driver.log || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $out/bench_50.json 2> $out/bench_50.log || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $out/bench_driver2.json 2> $out/bench_driver2.log || exit 1
python - <<'PY'
import json
for f in ("bench_driver", "bench_50", "bench_driver2"):
    d = json.load(open(f"gpurun_out/r5/{f}.json"))
    print(f, round(d["value"] / 1e6, 2), "M", round(d["ms_per_step"], 4), "ms", "section", d["roofline"]["avg_launch_ms"])
PY
timeout -k 10 600 python -u tools/long_run.py --out $out/long_run.json > $out/long_run.log 2>&1; rc=$?
tail -4 $out/long_run.log
exit $rc
