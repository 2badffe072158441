#!/bin/bash
# Timing-experiment variants of libdbsde.so (never the product): engine.hip
# rebuilt with -DDBSDE_EXP_<NAME> for each name given, linked with the normal
# tnw object, into exp/libdbsde_<name>.so ("base" = no flag).  Run after
# __graft_entry__.py build.   tools/build_exp.sh base nostore nostage cheapact
set -e
cd "$(dirname "$0")/.."
PKG=deep-neural-network-solutions-for-partial-differential-equations_amd
mkdir -p exp
pids=()
for v in "$@"; do
  flag=""
  [ "$v" != base ] && flag="-DDBSDE_EXP_$(echo "$v" | tr a-z A-Z)"
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC $flag -c -o exp/engine_$v.o $PKG/csrc/engine.hip &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o exp/libdbsde_$v.so exp/engine_$v.o $PKG/lib/obj/tnw.o ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la exp/*.so
