#!/bin/bash
# round 3 (af): host side of the 20-turn region (golhip_step return time vs the region)
set -u
O=gpurun_out/r03af
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 200 $O/host_submit.log python3 scripts/host_submit.py 15 || exit $?
grep "^{" $O/host_submit.log
