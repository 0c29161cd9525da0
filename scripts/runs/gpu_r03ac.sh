#!/bin/bash
# round 3 (ac): PMC passes of the production K = 12 and K = 8 launches (now pre-shifted, fixed
# depth) for pmc_traffic.json, and rocprofv3 kernel stats of the driver's 20/5 command
set -u
O=gpurun_out/r03ac
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
rm -rf gpurun_out/pmc_k12 gpurun_out/pmc_k8
$G 400 $O/pmc12.log bash scripts/pmc_passes.sh 12 || exit $?
$G 400 $O/pmc8.log bash scripts/pmc_passes.sh 8 || exit $?
$G 300 $O/prof20.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof20 -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-sweep --no-strong --no-flips --no-configs || exit $?
find /tmp/prof20 -name "*kernel_stats.csv" -exec cp {} $O/prof20_kernel_stats.csv \;
grep "^{" $O/prof20.log > $O/prof20_line.json
echo done
