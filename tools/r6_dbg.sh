#!/bin/bash
PKG=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd
T="tests/test_gpu_fullshape_oracle.py::test_config3_full_shape_matches_oracle tests/test_gpu_parity.py"
for v in headlib base headlib; do
  unset DBSDE_LIB DBSDE_TNW_X3
  [ $v != base ] && export DBSDE_LIB=$PKG/lib/exp/$v/libdbsde.so
  timeout -k 10 300 python -u -m pytest $T -q --timeout 120 --timeout-method thread > gpurun_out/dbg_$v.txt 2>&1
  echo "$v: $(tail -1 gpurun_out/dbg_$v.txt)"; grep "^FAILED" gpurun_out/dbg_$v.txt | head -5
done
