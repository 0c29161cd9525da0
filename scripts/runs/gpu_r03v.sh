#!/bin/bash
# round 3 (v): exact-fill band schedules (model: whole rounds of resident waves with the 8-step
# band alignment, two band heights) vs the automatic band, K = 12 at 65536^2, both geometries,
# pre-heated lockstep A/B
set -u
O=gpurun_out/r03v
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
AB_STEPS=480 $G 400 $O/ab_sched_k12.log python3 scripts/ab_variant.py 65536 12 prod,prod@184:111:176,prod@168:19:160,pre63,pre63@184:364:176 9 || exit $?
tail -2 $O/ab_sched_k12.log
