#!/bin/bash
# round 3 (al): rocprofv3 kernel stats of the default bench command (legs off) now that the
# bulk launch is K = 14: its gol_stencil<14> average against the line's HIP-event average
set -u
O=gpurun_out/r03al
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profd -o b -- python3 bench.py --no-cpu --no-sweep --no-strong --no-flips --no-configs || exit $?
tail -5 $O/prof.log | cut -c1-300
find /tmp/profd -name "*kernel_stats.csv" -exec cp {} $O/prof_kernel_stats.csv \;
grep "^{" $O/prof.log > $O/prof_line.json
echo done
