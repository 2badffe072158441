#!/bin/bash
# Prefetched vs in-step rollout for the basket / Heston workloads, interleaved.
export TMPDIR=/tmp
out=gpurun_out/r6pf
mkdir -p $out
for i in 1 2; do
  for w in basket heston; do
    for v in pf nopf; do
      a=""; [ $v = nopf ] && a="--no-prefetch"
      timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-parity --steps 50 --warmup 20 $a > $out/${w}_${v}_$i.log 2>&1 || { echo "fail $w $v"; tail -5 $out/${w}_${v}_$i.log; exit 1; }
      python - $out/${w}_${v}_$i.log "$w $v $i" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], " ".join("%s %.4f" % (n, k[n]) for n in list(k)[:4]), flush=True)
PY
    done
  done
done
