#!/bin/bash
# round 6 (l): the last tree -- smoke(), the driver's bench command (roofline.kernel now names every
# timed depth), the plain-launch and persistent GPU tests
set -u
O=gpurun_out/r06l
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 200 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -1 $O/smoke.log
$G 400 $O/bench20.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep '^{' $O/bench20.log > $O/bench20.json || true
python3 -c "import json;d=json.load(open('$O/bench20.json'));r=d['roofline'];print(d['value'],r['kernel'],r['avg_launch_us'],r['frac'],d['parity']['digest_ok'],d['configs']['ok'],d['cfg5_host']['ok'])" || true
$G 400 $O/tests.log python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_rank_host.py tests/test_gpu_failfast.py tests/test_host.py || exit $?
tail -2 $O/tests.log
