#!/bin/bash
# round 4 (i): kernel timeline of the split step on the ring of one (65536^2, 1000 turns) against
# the single strip: where the bands, the interior and the send/recv of each block run
set -u
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for ring in 1 0; do
  $G 200 $O/run_ring$ring.log rocprofv3 --kernel-trace --output-format csv -d /tmp/r04i_$ring -o t -- python3 scripts/ring_timeline.py run 65536 1000 $ring || exit $?
  grep "^{" $O/run_ring$ring.log
  python3 scripts/ring_timeline.py /tmp/r04i_$ring 8 70 > $O/timeline_ring$ring.txt 2>&1
  cut -c1-900 $O/timeline_ring$ring.txt
done
