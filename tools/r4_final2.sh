#!/bin/bash
# round-end evidence on the final build, then the headline workload's profile
tools/r4_final.sh || exit $?
tools/profile_round.sh r4 bsb
