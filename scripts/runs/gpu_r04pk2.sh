#!/bin/bash
# round 4 (pk2): gol_slabp at launch depths 8 / 12 against 16 on narrow boards (1600 turns)
set -u
O=gpurun_out/r04pk2
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/narrow.log python3 -u scripts/tune_narrow.py 512x512,64x64,4096x512 auto,140403,140603,140803,140403@12,140803@12,140403@8,140803@8,140404@8 1600 || exit $?
