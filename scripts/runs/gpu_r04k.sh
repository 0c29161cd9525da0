#!/bin/bash
# round 4 (k): rehearsal of a rank's process at N > 1 on one GPU (torch nccl process group +
# the engine as the RCCL ring of one), hardware queues 4 (the box's default) vs 8 (bench default),
# against the plain N = 1 line; 1000-turn default and the 20/5 driver shape
set -u
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
F="--no-cpu --no-sweep --no-strong --no-configs --no-flips"
for steps in "1000 8" "20 5"; do
  set -- $steps; S=$1; W=$2
  $G 200 $O/plain_s$S.log python3 bench.py --steps $S --warmup $W $F || exit $?
  for q in 0 8; do
    GOLHIP_RING_SELF=1 $G 200 $O/ring_q${q}_s$S.log python3 bench.py --steps $S --warmup $W --pg-always --hw-queues $q $F || exit $?
  done
done
for f in $O/*.log; do echo "$f: $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["transport"], d["process"], d["parity"]["ok"], d["parity"].get("digest_ok"))')"; done
