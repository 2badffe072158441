#!/bin/bash
# Timing-only attribution of the phase section: the
# DBSDE_AB_PHASE variants of engine.hip (csrc/phase.hpp) against the in-tree
# library, interleaved, two rounds, bench.py bsb --steps 100 --warmup 50.
export TMPDIR=/tmp
out=gpurun_out/r6ab
mkdir -p $out
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
for i in 1 2; do
  for v in base ${VARIANTS:-ab1 ab2 ab4 ab6 ab8 ab9 ab16 ab32}; do
    if [ $v = base ]; then unset DBSDE_LIB; else export DBSDE_LIB=$PKG/lib/exp/$v/libdbsde.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 100 --warmup 50 ${BENCH_ARGS} > $out/${v}_$i.log 2>&1 || { echo "fail $v rc=$?"; tail -5 $out/${v}_$i.log; exit 1; }
    python - $out/${v}_$i.log "$v $i" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
k = d["step_kernel_ms"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], " ".join("%s %.4f" % (n, k[n]) for n in list(k)[:5]), flush=True)
PY
  done
done
