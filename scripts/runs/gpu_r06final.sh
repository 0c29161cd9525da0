#!/bin/bash
# round 6 final validation of the tree as the driver will run it: the GPU suite (lib_tuning not
# pushed), smoke(), the driver's bench command, the same command under rocprofv3 --kernel-trace
# --stats (the roofline kernel's average against the line's HIP-event average), the default bench
set -u
R=${R06_OUT:-r06final}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 1000 $O/suite.log python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread || exit $?
tail -2 $O/suite.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -1 $O/smoke.log
$G 400 $O/bench20.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep '^{' $O/bench20.log > $O/bench20.json || true
$G 500 $O/bench20_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${R}_prof -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep '^{' $O/bench20_prof.log > $O/bench20_under_rocprof.json || true
find /tmp/${R}_prof -name "b_kernel_stats.csv" -exec cp {} $O/bench20_kernel_stats.csv \;
$G 400 $O/bench.log python -u bench.py --no-cpu || exit $?
grep '^{' $O/bench.log > $O/bench.json || true
python3 -c "
import json
for f in ('bench20', 'bench20_under_rocprof', 'bench'):
    d = json.load(open('$O/' + f + '.json'))
    r = d['roofline']
    print(f, d['value'], r['kernel'], r['avg_launch_us'], r['frac'], d['parity']['ok'], d['parity'].get('digest_ok'))
" || true
