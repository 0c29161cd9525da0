#!/bin/bash
set -u
O=gpurun_out/r02f
mkdir -p $O
export TMPDIR=/tmp
scripts/guard.sh 300 $O/bench20.log python -u bench.py --steps 20 --warmup 5 --no-cpu --no-strong --no-sweep || exit $?
scripts/guard.sh 300 $O/bench20b.log python -u bench.py --steps 20 --warmup 5 --no-cpu --no-strong --no-sweep || exit $?
scripts/guard.sh 300 $O/pytest_cfg.log python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -x || exit $?
scripts/guard.sh 400 $O/bench.log python -u bench.py || exit $?
