#!/bin/bash
mkdir -p gpurun_out/ub
timeout -k 10 200 tools/ubench/piece_x3 > gpurun_out/ub/piece5.txt 2>&1
rc=$?
cat gpurun_out/ub/piece5.txt
exit $rc
