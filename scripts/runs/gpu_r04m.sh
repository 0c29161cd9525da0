#!/bin/bash
# round 4 (m): the 20-turn ring of one's timeline; the rank rehearsal with the shared-memory
# barrier vs the RCCL one; band-height sweep of the streaming launch with per-wave stamps (the
# trapezoid against the tail)
set -u
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for ring in 1 0; do
  $G 200 $O/run20_ring$ring.log rocprofv3 --kernel-trace --output-format csv -d /tmp/r04m_$ring -o t -- python3 scripts/ring_timeline.py run 65536 20 $ring 5 || exit $?
  grep "^{" $O/run20_ring$ring.log
  python3 scripts/ring_timeline.py /tmp/r04m_$ring 3 3 > $O/timeline20_ring$ring.txt 2>&1
  cut -c1-900 $O/timeline20_ring$ring.txt
done
F="--no-cpu --no-sweep --no-strong --no-configs --no-flips"
for b in "" "--rccl-barrier"; do
  GOLHIP_RING_SELF=1 $G 200 $O/ring_s20$b.log python3 bench.py --steps 20 --warmup 5 --pg-always $b $F || exit $?
  grep '^{' $O/ring_s20$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["process"], d["instrumented_pass"]["kernel_ms"], d["parity"]["ok"], d["parity"].get("digest_ok"))'
done
for kb in "14 0" "14 106" "14 150" "14 264" "14 330" "14 422" "14 660" "12 0" "12 240" "12 336"; do
  set -- $kb; K=$1; B=$2
  GOLHIP_BAND_ROWS=$B $G 120 $O/stamps_k${K}_b$B.log python3 scripts/stamp_launch.py 65536 $K 4 300 || exit $?
  echo "K=$K band=$B: $(grep '"launch": 3' $O/stamps_k${K}_b$B.log | cut -c1-330)"
done
