#!/bin/bash
# round 4 (pz): rocprofv3 kernel stats of the final tree (packed slab, pinned counts)'s default bench command and of the
# driver-shaped 20/5 command (the lines under rocprof beside them)
set -u
O=gpurun_out/r04pz
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 600 $O/bench_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r04pz_prof -o b -- python3 bench.py || exit $?
grep "^{" $O/bench_prof.log > $O/bench_under_rocprof.json
find /tmp/r04pz_prof -name "*kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
$G 400 $O/bench20_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r04pz_prof20 -o b -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-sweep --no-strong --no-flips || exit $?
grep "^{" $O/bench20_prof.log > $O/bench20_under_rocprof.json
find /tmp/r04pz_prof20 -name "*kernel_stats.csv" -exec cp {} $O/bench20_kernel_stats.csv \;
for f in bench bench20; do python3 -c "import json; d=json.load(open('$O/${f}_under_rocprof.json')); print('$f', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['parity']['digest_ok'])"; done
grep -E "gol_stencil<14,|gol_stencil<12,|gol_stencil<8,|gol_slab2" $O/bench_kernel_stats.csv | cut -c1-60,100-260 | head
