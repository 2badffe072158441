#!/bin/bash
# Round-end evidence: smoke, the GPU test suite, then the bench lines
tools/r4_final_tests.sh || exit $?
tools/r4_final_bench.sh
