#!/bin/bash
# column-split register feed: two pieces in flight (base) vs three (cs3)
export TMPDIR=/tmp
tools/ab_libs.sh "--paths-per-gpu 128 --no-cpu-baseline --no-parity --steps 100" cs3 > gpurun_out/ablib/cs3.txt 2>&1; cat gpurun_out/ablib/cs3.txt
export DBSDE_CS=1 DBSDE_CHUNKS=1
tools/ab_libs.sh "--paths-per-gpu 256 --no-cpu-baseline --no-parity --steps 100" cs3 > gpurun_out/ablib/cs3_256.txt 2>&1; cat gpurun_out/ablib/cs3_256.txt
