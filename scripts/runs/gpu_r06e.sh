#!/bin/bash
# round 6 (e): the host contract with per-turn CellFlipped events, pipelined vs unpipelined
# (configs[4]'s board and images/512x512.pgm), and smoke()
set -u
O=gpurun_out/r06e
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/host_flips_ab.log python -u scripts/host_flips_ab.py 100000 10000 || exit $?
tail -1 $O/host_flips_ab.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -2 $O/smoke.log
