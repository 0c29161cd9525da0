#!/bin/bash
# round 5 (final): GPU suite, smoke, the default and driver-shaped bench lines, and rocprofv3
# kernel stats of the default bench command (the line under rocprof beside it)
set -u
O=gpurun_out/${R05_OUT:-r05final}
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 900 $O/suite.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
tail -3 $O/suite.log
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -2 $O/smoke.log
$G 400 $O/bench.log python3 bench.py || exit $?
$G 300 $O/bench20.log python3 bench.py --steps 20 --warmup 5 || exit $?
for f in bench bench20; do grep '^{' $O/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$f'", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["parity"]["ok"], d["parity"].get("digest_ok"), (d.get("configs") or {}).get("ok"))'; done
$G 600 $O/bench_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05_prof -o b -- python3 bench.py || exit $?
grep "^{" $O/bench_prof.log > $O/bench_under_rocprof.json
find /tmp/r05_prof -name "*kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
python3 -c "import json; d=json.load(open('$O/bench_under_rocprof.json')); print('prof', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['parity']['digest_ok'])"
