#!/bin/bash
# round 4 (p5): gol_slabp on P = 2 boards (640 / 768 wide), wider P and tall narrow boards
set -u
O=gpurun_out/r04p5
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
C=auto,121207,140403,140603,140803,140405,140406,140404,140806,141203,140206
$G 700 $O/narrow.log python3 -u scripts/tune_narrow.py 640x640,768x768,384x384,4096x512,16384x256,2048x128 $C 1600 || exit $?
grep -v '^{"narrow' $O/narrow.log
