#!/bin/bash
set -u
O=gpurun_out/r02l
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
TUNE_COUNTS=0 $G 300 $O/tune_nocount.log python3 scripts/tune_tile.py 512,5120 0,t16,s0808,s1604 8,16 || exit $?
for S in 1604 0808; do
  GOLHIP_SLAB=$S $G 200 $O/tl_s$S.log rocprofv3 --kernel-trace --output-format csv -d $O/tl_s$S -o tl -- python3 scripts/profile_small.py 512 16 1024 counts || exit $?
  python3 scripts/launch_timeline.py $O/tl_s$S 100 > $O/timeline_s$S.txt 2>&1
  GOLHIP_SLAB=$S $G 200 $O/tl_s${S}_nc.log rocprofv3 --kernel-trace --output-format csv -d $O/tl_s${S}_nc -o tl -- python3 scripts/profile_small.py 512 16 1024 || exit $?
  python3 scripts/launch_timeline.py $O/tl_s${S}_nc 100 > $O/timeline_s${S}_nc.txt 2>&1
done
echo done
