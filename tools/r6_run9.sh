#!/bin/bash
# Timing-only attribution of the correlated rollout (DBSDE_AB_CORR bits,
# paths.hpp): basket, in-step rollout, the rollout record.
VARIANTS="c1 c2 c4 c8 c3" BENCH_ARGS="--workload basket --no-prefetch" tools/r6_ab_phase.sh
