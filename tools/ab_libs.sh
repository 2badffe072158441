#!/bin/bash
# Interleaved A/B of experimental libraries (lib/exp/<name>/libdbsde.so; "base"
# = the in-tree one) on bench.py: tools/ab_libs.sh "<bench args>" name1 name2 ...
mkdir -p gpurun_out/ablib
args=$1; shift
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
for i in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then unset DBSDE_LIB; else export DBSDE_LIB=$PKG/lib/exp/$v/libdbsde.so; fi
    timeout -k 10 200 python bench.py $args > gpurun_out/ablib/${v}_$i.log 2>&1 || { echo "fail $v rc=$?"; tail -5 gpurun_out/ablib/${v}_$i.log; exit 1; }
    python - gpurun_out/ablib/${v}_$i.log "$v $i" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], {n: k[n] for n in list(k)[:4]})
PY
  done
done
