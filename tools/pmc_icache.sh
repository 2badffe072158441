#!/bin/bash
# Instruction-cache / instruction-fetch counters over a short bench run (one
# --pmc pass each; no tracing domains).  Outputs gpurun_out/pmc_<tag>_ic{1,2}/.
#   tools/pmc_icache.sh <tag> [bench args...]
tag=${1:-x}; shift
export TMPDIR=/tmp
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set -d gpurun_out/pmc_${tag}_ic$i -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_${tag}_ic$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc_${tag}_ic$i.log; exit 1; }
done
echo ok
