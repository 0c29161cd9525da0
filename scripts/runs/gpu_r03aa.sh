#!/bin/bash
# round 3 (aa): launch splits of the driver's 20-turn region on the dense random start (planner
# 12 + 8 vs fixed 10 + 10, 14 + 6, 16 + 4), both geometries
set -u
O=gpurun_out/r03aa
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/ab_split.log python3 scripts/ab_split.py prod,pre63 0,10,12,14,16 9 || exit $?
tail -11 $O/ab_split.log
