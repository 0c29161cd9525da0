#!/bin/bash
# round 3 (ae): bulk depth at 65536^2 with the pre-shifted production (K = 10 / 12 / 14 / 16,
# pre-heated, lockstep rounds) -- the planner's rate table
set -u
O=gpurun_out/r03ae
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
AB_STEPS=672 $G 400 $O/ab_depth.log python3 scripts/ab_variant.py 65536 10,12,14,16 prod 11 || exit $?
tail -4 $O/ab_depth.log
AB_STEPS=112 $G 400 $O/ab_depth_262144.log python3 scripts/ab_variant.py 262144 12,14,16 prod 5 || exit $?
tail -3 $O/ab_depth_262144.log
