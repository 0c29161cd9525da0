#!/bin/bash
# round 2 (w): dispatch timeline of configs[1]'s production path (5120^2, k=16, counts)
set -u
O=gpurun_out/r02w
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for C in counts nc; do
  A=""; [ $C = counts ] && A=counts
  $G 200 $O/tl_$C.log rocprofv3 --kernel-trace --output-format csv -d $O/tl_$C -o tl -- python3 scripts/profile_small.py 5120 16 2048 $A || exit $?
  python3 scripts/launch_timeline.py $O/tl_$C 100 > $O/timeline_$C.txt 2>&1
done
echo done
