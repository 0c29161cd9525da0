#!/bin/bash
# round 4 (l): boundary-band waves at raised issue priority (s_setprio) -- rank-process rehearsal
# (ring of one + torch nccl group) with and without, the plain N = 1 line, the prediction
set -u
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
F="--no-cpu --no-sweep --no-strong --no-configs --no-flips"
TL=distributed-gol_amd/lib_tuning/libgolhip.so
for steps in "20 5" "1000 8"; do
  set -- $steps; S=$1; W=$2
  $G 200 $O/plain_s$S.log python3 bench.py --steps $S --warmup $W $F || exit $?
  GOLHIP_RING_SELF=1 $G 200 $O/ring_s$S.log python3 bench.py --steps $S --warmup $W --pg-always $F || exit $?
  GOLHIP_LIB=$TL GOLHIP_EDGE_SETPRIO=0 GOLHIP_RING_SELF=1 $G 200 $O/ring_noprio_s$S.log python3 bench.py --steps $S --warmup $W --pg-always $F || exit $?
  GOLHIP_LIB=$TL GOLHIP_EDGE_SETPRIO=1 GOLHIP_RING_SELF=1 $G 200 $O/ring_tprio_s$S.log python3 bench.py --steps $S --warmup $W --pg-always $F || exit $?
done
for f in $O/*.log; do echo "$f: $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["transport"], d["parity"]["ok"], d["parity"].get("digest_ok"))')"; done
GPU_MAX_HW_QUEUES=8 $G 300 $O/predict.log python3 scripts/predict_scaling.py 5 20,1000 160 || exit $?
grep "^{\"shape" $O/predict.log | cut -c1-250
