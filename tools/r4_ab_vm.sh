#!/bin/bash
# A/B of the piece vmcnt counts (base = DBSDE_VMCOUNT 1, vm0 = the earlier counts)
export TMPDIR=/tmp
mkdir -p gpurun_out/ablib
timeout -k 10 120 tools/ubench/piece_x3 > gpurun_out/ablib/piece5.txt 2>&1 || exit 1
tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 100" vm0 > gpurun_out/ablib/bsb.txt 2>&1 || { cat gpurun_out/ablib/bsb.txt; exit 1; }
cat gpurun_out/ablib/bsb.txt
timeout -k 10 200 python bench.py --workload hjb --no-cpu-baseline --no-parity --steps 50 > gpurun_out/ablib/hjb.log 2>&1 && tail -c 600 gpurun_out/ablib/hjb.log
