#!/bin/bash
# Round-6 closing bench lines of the final build.
export TMPDIR=/tmp
out=gpurun_out/r6k
mkdir -p $out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$out/$name.log"; exit $rc; }
}
B="bench.py --no-cpu-baseline --no-parity"
step bench 600 python bench.py
for i in 1 2 3; do step driver_$i 200 python $B --gpus 1 --steps 20 --warmup 5; done
step bench_100_50 200 python $B --steps 100 --warmup 50
for w in oned basket hjb heston; do step wl_$w 300 python $B --workload $w --steps 50 --warmup 10; done
for m in 128 256 512; do step strong_$m 200 python $B --paths-per-gpu $m --steps 100 --warmup 10; done
echo done
