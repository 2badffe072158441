#!/bin/bash
# profiles of the chain-layout workloads on the final build
tools/profile_round.sh r4 hjb || exit $?
tools/profile_round.sh r4 oned || exit $?
