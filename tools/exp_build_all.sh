#!/bin/bash
# Like exp_build.sh, but every translation unit is compiled with the variant's
# definitions: tools/exp_build_all.sh name "-DFOO=1" [name2 "defs2" ...]
set -e
PKG=deep-neural-network-solutions-for-partial-differential-equations_amd
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  d=$PKG/lib/exp/$name; mkdir -p $d
  pids=()
  for u in engine phase2 phasecs evals tnwx3; do $H $F $defs -c -o $d/$u.o $PKG/csrc/$u.hip & pids+=($!); done
  $H $F $defs -mllvm -amdgpu-mfma-vgpr-form=true -c -o $d/tnw.o $PKG/csrc/tnw.hip & pids+=($!)
  for p in "${pids[@]}"; do wait $p; done
  $H --offload-arch=gfx950 -shared -fPIC -o $d/libdbsde.so $d/*.o && rm $d/*.o && echo "built $name"
done
