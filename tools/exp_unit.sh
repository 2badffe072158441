#!/bin/bash
# A/B builds that differ in one source unit's definitions:
#   [SRC=file.hip] tools/exp_unit.sh <unit> name "-DFOO=1" [name2 "-DBAR=1" ...]
# (unit = engine | tnwx3 | phase2 | ...; the other objects are the in-tree ones)
set -e
PKG=deep-neural-network-solutions-for-partial-differential-equations_amd
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC"
unit=$1; shift
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p $PKG/lib/exp/$name
  src=${SRC:-$PKG/csrc/$unit.hip}
  $H $F $defs -I$PKG/csrc -c -o $PKG/lib/exp/$name/$unit.o $src
  objs=""
  for u in engine phase2 phasecs evals tnw tnwx3; do
    if [ $u = $unit ]; then objs="$objs $PKG/lib/exp/$name/$u.o"; else objs="$objs $PKG/lib/obj/$u.o"; fi
  done
  $H --offload-arch=gfx950 -shared -fPIC -o $PKG/lib/exp/$name/libdbsde.so $objs
  rm $PKG/lib/exp/$name/$unit.o; echo "built $name"
done
