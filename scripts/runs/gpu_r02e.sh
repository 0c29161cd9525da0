#!/bin/bash
# Round-2 GPU session E: full GPU suite on the planner + per-depth production variant; benches
# (driver's 20/5 and the default) against the round-1 variant in the same call.
set -u
O=gpurun_out/r02e
mkdir -p $O
export TMPDIR=/tmp
scripts/guard.sh 300 $O/bench20.log python -u bench.py --steps 20 --warmup 5 --no-cpu --no-strong || exit $?
GOLHIP_VARIANT=driftlds scripts/guard.sh 300 $O/bench20_driftlds.log python -u bench.py --steps 20 --warmup 5 --no-cpu --no-strong --no-sweep || exit $?
scripts/guard.sh 300 $O/bench20b.log python -u bench.py --steps 20 --warmup 5 --no-cpu --no-strong --no-sweep || exit $?
scripts/guard.sh 900 $O/pytest.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit $?
scripts/guard.sh 400 $O/bench.log python -u bench.py --no-cpu || exit $?
GOLHIP_VARIANT=driftlds scripts/guard.sh 400 $O/bench_driftlds.log python -u bench.py --no-cpu --no-sweep --no-strong || exit $?
