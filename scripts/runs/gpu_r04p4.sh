#!/bin/bash
# round 4 (p4): gol_slabp shape sweep on narrow boards, long runs (per-call overhead out)
set -u
O=gpurun_out/r04p4
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
C=auto,121207,140803,140804,140403,140404,140405,140406,140603,140806,141203,141603,140206,140208,120803@12,120403@12,80803@8,80403@8,80404@8
$G 600 $O/narrow.log python3 -u scripts/tune_narrow.py 512x512,256x256,64x64,16x16,960x960,2048x512 $C 1600 || exit $?
grep -v '^{"narrow' $O/narrow.log
