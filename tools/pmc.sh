#!/bin/bash
# Counter passes over a short bench run, one rocprofv3 --pmc pass each (no
# tracing domains), outputs under gpurun_out/pmc_<tag>_<i>/.  Extra env
# (e.g. DBSDE_CHUNKS=1 to time phase A and C separately) is inherited.
#   tools/pmc.sh <tag> [bench args...]
tag=${1:-x}; shift
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set -d gpurun_out/pmc_${tag}_$i -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_${tag}_$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc_${tag}_$i.log; exit 1; }
done
echo ok
