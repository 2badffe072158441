#!/bin/bash
# Build A/B variants of libdbsde.so that differ only in engine.hip compile
# definitions: tools/exp_build.sh name "-DFOO=1 -DBAR=2" [name2 "defs2" ...]
# -> <pkg>/lib/exp/<name>/libdbsde.so (the other units' objects from lib/obj).
set -e
PKG=deep-neural-network-solutions-for-partial-differential-equations_amd
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC"
pids=()
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p $PKG/lib/exp/$name
  ( $H $F $defs -c -o $PKG/lib/exp/$name/engine.o $PKG/csrc/engine.hip && \
    $H --offload-arch=gfx950 -shared -fPIC -o $PKG/lib/exp/$name/libdbsde.so $PKG/lib/exp/$name/engine.o \
       $PKG/lib/obj/phase2.o $PKG/lib/obj/phasecs.o $PKG/lib/obj/evals.o $PKG/lib/obj/tnw.o $PKG/lib/obj/tnwx3.o && \
    rm $PKG/lib/exp/$name/engine.o && echo "built $name" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
