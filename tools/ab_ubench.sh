#!/bin/bash
mkdir -p gpurun_out/ub
timeout -k 10 120 tools/ubench/piece_x3 > gpurun_out/ub/piece2.txt 2>&1 || { echo "ubench rc=$?"; cat gpurun_out/ub/piece2.txt; exit 1; }
cat gpurun_out/ub/piece2.txt
