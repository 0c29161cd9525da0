#!/bin/bash
# round 3 (t): where the time of the compact flips path goes: rocprofv3 kernel + memory-copy
# traces of golhip_step_flips_rows and golhip_step_flips at 5120^2 on the same turns; PMC passes
# of the production K = 16 launch (fixed depth)
set -u
O=gpurun_out/r03t
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for m in rows pairs; do
  F=""; [ $m = rows ] && F="--rows"
  $G 300 $O/prof_$m.log rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/prof_$m -o f -- python3 scripts/flips_profile.py --calls 4 --snapshots 0 $F || exit $?
  grep "^{" $O/prof_$m.log
  find /tmp/prof_$m -name "*stats.csv" | while read f; do cp "$f" $O/${m}_$(basename "$f"); done
done
ls $O
$G 400 $O/pmc16.log bash scripts/pmc_passes.sh 16 || exit $?
tail -1 $O/pmc16.log
