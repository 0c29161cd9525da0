#!/bin/bash
# round 3 (s): PMC passes of the production K = 16 launch (pre-shifted 63-word geometry) and of
# K = 12, rocprofv3 kernel stats of the driver's 20/5 command, and the full 20/5 bench line (flips
# leg with both forms on the same turns)
set -u
O=gpurun_out/r03s
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/pmc16.log bash scripts/pmc_passes.sh 16 || exit $?
tail -1 $O/pmc16.log
$G 400 $O/pmc12.log bash scripts/pmc_passes.sh 12 || exit $?
tail -1 $O/pmc12.log
$G 300 $O/prof20.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof20 -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-sweep --no-strong --no-flips --no-configs || exit $?
find /tmp/prof20 -name "*kernel_stats.csv" -exec cp {} $O/prof20_kernel_stats.csv \;
grep "^{" $O/prof20.log > $O/prof20_line.json
$G 400 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep "^{" $O/bench20.log | cut -c1-300
