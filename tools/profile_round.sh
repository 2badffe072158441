#!/bin/bash
# Round profile on the GPU box for one workload: kernel-trace stats of the
# bench, HBM counter passes (FETCH_SIZE and WRITE_SIZE in separate --pmc
# passes, no tracing domains) and two SQ counter sets.  Outputs under
# gpurun_out/prof_<tag>_<workload>/; copy the summaries into profiles/ afterwards.
#   tools/profile_round.sh <tag> [workload] [extra bench args...]
set -o pipefail
tag=${1:-r4}
wl=${2:-bsb}
shift 2 2>/dev/null
extra="$*"
out=gpurun_out/prof_${tag}_${wl}
mkdir -p $out
export TMPDIR=/tmp
# counter passes serialise kernels: order the streams with events (the engine
# also falls back by itself under rocprofv3 --pmc), never with spinning value waits
export DBSDE_STREAM_ORDER=events
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$wl $name rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$out/$name.log"; exit $rc; }
}
B="bench.py --workload $wl --no-cpu-baseline --no-parity $extra"
run stats 300 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- python $B --steps 20 --warmup 5
run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python $B --steps 3 --warmup 1
run pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python $B --steps 3 --warmup 1
run pmc_sq1 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $out/pmc_sq1 -o run --output-format csv -- python $B --steps 3 --warmup 1
run pmc_sq2 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH -d $out/pmc_sq2 -o run --output-format csv -- python $B --steps 3 --warmup 1
echo done
