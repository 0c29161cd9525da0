#!/bin/bash
# round 3 (c): rocprof of the flips / snapshot driver: kernel stats + HIP API stats (csv), and the
# hipMalloc/hipFree calls issued while the 5120^2 snapshots run
set -u
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/rocprof_flips.log rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d /tmp/prof_r03c -o flips -- python3 scripts/flips_profile.py --calls 4 --snapshots 8 || exit $?
find /tmp/prof_r03c -name "*stats.csv" -exec cp {} $O/ \;
T=$(find /tmp/prof_r03c -name "*hip_api_trace.csv" | head -1)
python3 scripts/hip_alloc_calls.py "$T" > $O/hip_alloc_calls.txt 2>&1
ls -la $O
