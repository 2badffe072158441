#!/bin/bash
# GPU-box measurement set: the headline bench line (CPU baseline + Y0 parity
# trajectory), the BASELINE workloads 3-5, the per-rank shapes of 2/4/8-GPU
# strong scaling (M = 512/256/128 on one GPU), and a rocprofv3 kernel-trace
# summary of the headline.  Each step has its own time limit; a crash or
# timeout stops the script.   tools/measure.sh <tag>
tag=${1:-r3}
out=gpurun_out/meas_$tag
mkdir -p $out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $out/steps.log
  [ $rc -eq 0 ] || { tail -20 "$out/$name.log"; exit $rc; }
}
step bench 400 python bench.py
for w in basket hjb heston; do
  step wl_$w 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline
done
for m in 512 256 128; do
  step m$m 300 python bench.py --paths-per-gpu $m --steps 50 --warmup 10 --no-cpu-baseline --no-parity
done
step stats 300 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity
echo done
