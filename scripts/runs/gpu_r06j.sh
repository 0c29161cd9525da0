#!/bin/bash
# round 6 (j): the driver's bench command under rocprofv3 with the other boards' legs off, so the
# kernel statistics hold only the 65536^2 launches the roofline times (cold pass, pre-heat, timed and
# instrumented passes): gol_stencil<12> / <8> averages against the line's avg_launch_us
set -u
O=gpurun_out/r06j
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/bench20_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06j_prof -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-sweep --no-strong --no-flips --no-configs --no-host || exit $?
grep '^{' $O/bench20_prof.log > $O/bench20_under_rocprof.json || true
find /tmp/r06j_prof -name "b_kernel_stats.csv" -exec cp {} $O/bench20_kernel_stats.csv \;
find /tmp/r06j_prof -name "b_kernel_trace.csv" -exec cp {} $O/bench20_kernel_trace.csv \;
