#!/bin/bash
# A/B builds that differ only in tnwx3.hip definitions: tools/exp_tnw.sh name "-DFOO=1" [...]
set -e
PKG=deep-neural-network-solutions-for-partial-differential-equations_amd
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p $PKG/lib/exp/$name
  $H $F $defs -c -o $PKG/lib/exp/$name/tnwx3.o $PKG/csrc/tnwx3.hip
  $H --offload-arch=gfx950 -shared -fPIC -o $PKG/lib/exp/$name/libdbsde.so $PKG/lib/obj/engine.o \
     $PKG/lib/obj/phase2.o $PKG/lib/obj/phasecs.o $PKG/lib/obj/evals.o $PKG/lib/obj/tnw.o $PKG/lib/exp/$name/tnwx3.o
  rm $PKG/lib/exp/$name/tnwx3.o; echo "built $name"
done
