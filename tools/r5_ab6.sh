#!/bin/bash
# tnw load ablations (timing only): a quarter of the operand loads, no operand loads
export TMPDIR=/tmp
bash tools/ab_libs.sh "--no-cpu-baseline --no-parity --steps 60 --warmup 30" quarterld noload || exit 1
