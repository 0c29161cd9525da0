#!/bin/bash
# round 5: the persistent call on 16 x 4 boards beside configs[4] / configs[1] (4096-turn calls)
set -u
O=gpurun_out/r05zb
mkdir -p $O
G=scripts/guard.sh
$G 300 $O/probe.log python3 scripts/probe_slabq.py 4096 3 3968x4096,2048,4096,5120 || exit $?
grep -E "^[0-9]" $O/probe.log
