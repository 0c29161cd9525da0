#!/bin/bash
# round 4 (q): the 20-turn ring of one and the single strip, last dispatches raw (where the
# ring's extra ~40 us of kernel span go)
set -u
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for ring in 1 0; do
  $G 200 $O/run20_ring$ring.log rocprofv3 --kernel-trace --output-format csv -d /tmp/r04q_$ring -o t -- python3 scripts/ring_timeline.py run 65536 20 $ring 5 || exit $?
  grep "^{" $O/run20_ring$ring.log
  python3 scripts/ring_timeline.py /tmp/r04q_$ring tail 14 > $O/tail20_ring$ring.txt 2>&1
  cat $O/tail20_ring$ring.txt
done
