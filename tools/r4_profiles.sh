#!/bin/bash
# Round-4 rocprofv3 stats + counter passes for the other BASELINE workloads and
# the M=128 strong-scaling shape (tools/profile_round.sh each)
mkdir -p gpurun_out/prof4
timeout -k 10 300 python -u -m pytest tests/test_gpu_round4.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "w256 or hjb or oned or chunk or splits" > gpurun_out/prof4/tests.txt 2>&1; tail -3 gpurun_out/prof4/tests.txt
timeout -k 10 200 python bench.py --workload oned --no-cpu-baseline --no-parity --steps 50 > gpurun_out/prof4/oned.log 2>&1 && tail -c 300 gpurun_out/prof4/oned.log
tools/ab_libs.sh "--workload hjb --no-cpu-baseline --no-parity --steps 50" pd1 > gpurun_out/prof4/ab_pd.txt 2>&1; cat gpurun_out/prof4/ab_pd.txt
tools/ab_libs.sh "--workload oned --no-cpu-baseline --no-parity --steps 50" pd1 > gpurun_out/prof4/ab_pd_oned.txt 2>&1; cat gpurun_out/prof4/ab_pd_oned.txt
tools/profile_round.sh r4 basket || exit $?
tools/profile_round.sh r4 heston || exit $?
tools/profile_round.sh r4m128 bsb --paths-per-gpu 128 || exit $?
tools/profile_round.sh r4 oned || exit $?
