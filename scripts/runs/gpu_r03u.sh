#!/bin/bash
# round 3 (u): device -> host copy rates (pinned / pageable) and the flips profiler's own byte
# counts for both list forms
set -u
O=gpurun_out/r03u
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 200 $O/d2h.log python3 scripts/d2h_rate.py || exit $?
grep "^{" $O/d2h.log
$G 300 $O/flips_rows.log python3 scripts/flips_profile.py --calls 8 --snapshots 0 --rows || exit $?
grep "^{" $O/flips_rows.log
$G 300 $O/flips_pairs.log python3 scripts/flips_profile.py --calls 8 --snapshots 0 || exit $?
grep "^{" $O/flips_pairs.log
