#!/bin/bash
# round 4 (n): phase stamps of the production gol_slab2 launches (configs[1] 5120^2, configs[4]
# 4096^2; with and without per-turn counts): ramp, row loads, generation loop, count flush, tail
set -u
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 120 $O/slab_stamps_counts.log python3 scripts/slab_stamps.py 5120,4096 4 1 || exit $?
grep '"launch": 3' $O/slab_stamps_counts.log | cut -c1-700
$G 120 $O/slab_stamps_nocounts.log python3 scripts/slab_stamps.py 5120,4096 4 0 || exit $?
grep '"launch": 3' $O/slab_stamps_nocounts.log | cut -c1-700
