#!/bin/bash
# Round-5 profile of one workload: tools/profile_round.sh (kernel stats + FETCH /
# WRITE / SQ counter passes) and the per-step kernel timeline of the timed steps
#   tools/r5_prof.sh <tag> <workload> [extra bench args]
set -o pipefail
tag=$1; wl=$2; shift 2
bash tools/profile_round.sh $tag $wl "$@" || exit $?
out=gpurun_out/prof_${tag}_${wl}
python tools/timeline.py $out/stats/run_kernel_trace.csv 2 $out/timeline.txt | tail -45
