#!/bin/bash
# column-split register feed: two pieces in flight (base) vs three (cs3)
export TMPDIR=/tmp
mkdir -p gpurun_out/ablib
tools/ab_libs.sh "--paths-per-gpu 128 --no-cpu-baseline --no-parity --steps 100" cs3 > gpurun_out/ablib/cs3.txt 2>&1; cat gpurun_out/ablib/cs3.txt
timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 100 > gpurun_out/ablib/bsb_tf.log 2>&1 && tail -c 400 gpurun_out/ablib/bsb_tf.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_round3.py tests/test_gpu_round4.py -q --timeout 120 --timeout-method thread > gpurun_out/ablib/tests_tf.txt 2>&1; tail -2 gpurun_out/ablib/tests_tf.txt
export DBSDE_CS=1 DBSDE_CHUNKS=1
tools/ab_libs.sh "--paths-per-gpu 256 --no-cpu-baseline --no-parity --steps 100" cs3 > gpurun_out/ablib/cs3_256.txt 2>&1; cat gpurun_out/ablib/cs3_256.txt
