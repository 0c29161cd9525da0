#!/bin/bash
# round 6 (h): the batched end-of-launch count flush (flush_counts_strided): 512^2 counting packed
# slab under rocprof (compare r06g: 7.24 us per 16-generation launch), the slab parity tests, and
# the configs leg's three boards through bench.py's configs timing
set -u
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 500 $O/parity.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_board.py tests/test_gpu_activity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 280 --timeout-method thread || exit $?
tail -2 $O/parity.log
for N in 512 5120 4096; do
  $G 120 $O/trace_${N}.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06h_$N -o t -- python3 scripts/profile_small.py $N 16 4096 counts || exit $?
  find /tmp/r06h_$N -name "t_kernel_stats.csv" -exec cp {} $O/kernel_stats_${N}_counts.csv \;
done
$G 300 $O/configs.log python3 -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench; r = bench.configs_leg(); print(json.dumps({k: (v.get('us_per_turn') if isinstance(v, dict) else v) for k, v in r.items()}))" || exit $?
tail -1 $O/configs.log
