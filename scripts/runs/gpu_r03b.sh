#!/bin/bash
# round 3 (b): per-generation ring flips (gol_slab LD = 2, multi-block scan, pinned host list):
# flips tests, the flips profile (kernel + HIP API trace), the flips leg of the bench
set -u
O=gpurun_out/r03b
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/pytest_flips.log python -u -m pytest tests/test_gpu_parity.py -k "flips or store_interleaved or slab" -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
tail -1 $O/pytest_flips.log
$G 300 $O/flips_profile.log python3 scripts/flips_profile.py || exit $?
tail -1 $O/flips_profile.log
# the raw traces exceed what gpurun copies back: keep only the stats summaries
$G 300 $O/rocprof_flips.log rocprofv3 --kernel-trace --hip-trace --stats -d /tmp/prof_r03b -o flips -- python3 scripts/flips_profile.py --calls 4 --snapshots 8 || exit $?
find /tmp/prof_r03b -name "*stats*.csv" -exec cp {} $O/ \;
ls -la $O
