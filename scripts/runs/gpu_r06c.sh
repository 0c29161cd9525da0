#!/bin/bash
# round 6 (c): the whole production GPU suite (lib_tuning not pushed: its module skips; the fault
# library's smoke runs), the persistent hand-off A/B (fenced default vs sc1), and the driver's
# bench command with the new cfg5_host leg
set -u
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 1000 $O/suite.log python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread || exit $?
tail -3 $O/suite.log
$G 200 $O/probe_slabq.log python -u scripts/probe_slabq.py 4096 3 || exit $?
tail -2 $O/probe_slabq.log
$G 400 $O/bench20.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep '^{' $O/bench20.log > $O/bench20.json || true
python3 -c "import json;d=json.load(open('$O/bench20.json'));print(d['value'],d['roofline']['frac'],json.dumps(d.get('cfg5_host'))[:1500])" || true
$G 300 $O/cfg5_sparse.log python -u scripts/probe_cfg5_sparse.py 100000 || exit $?
tail -1 $O/cfg5_sparse.log
