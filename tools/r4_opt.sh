#!/bin/bash
# vectorized chain slab sums (lib/exp/vec) against the in-tree build: the
# chain / width-256 parity tests on the variant, then HJB and config 1 A/B
export TMPDIR=/tmp
out=gpurun_out/opt
mkdir -p $out
DBSDE_LIB=$PWD/deep-neural-network-solutions-for-partial-differential-equations_amd/lib/exp/vec/libdbsde.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/tests_vec.txt 2>&1
rc=$?; tail -2 $out/tests_vec.txt; grep -E "FAILED|ERROR" $out/tests_vec.txt | head; [ $rc -eq 0 ] || exit $rc
tools/ab_libs.sh "--workload hjb --no-cpu-baseline --no-parity --steps 50" vec > $out/hjb.txt 2>&1; cat $out/hjb.txt
tools/ab_libs.sh "--workload oned --no-cpu-baseline --no-parity --steps 50" vec > $out/oned.txt 2>&1; cat $out/oned.txt
