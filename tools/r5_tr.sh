#!/bin/bash
# kernel-trace timeline of bench.py under an env setting: tools/r5_tr.sh <tag> "<env>" [bench args]
export TMPDIR=/tmp
tag=$1; envs=$2; shift 2
out=gpurun_out/r5tr_$tag
mkdir -p $out
env $envs timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr -o run --output-format csv -- python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 "$@" > $out/tr.log 2>&1 || exit 1
python tools/steps_view.py $(ls $out/tr/*/run_kernel_trace.csv $out/tr/run_kernel_trace.csv 2>/dev/null | head -1)
