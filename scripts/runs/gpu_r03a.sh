#!/bin/bash
# round 3 (a): the round-3 tree's first GPU call -- smoke, the new rank-engine (host transport) and
# staged-transfer tests, the driver's bench command, then the whole GPU suite
set -u
O=gpurun_out/r03a
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
$G 900 $O/pytest_new.log python -u -m pytest tests/test_gpu_rank_host.py tests/test_gpu_parity.py -k "rank_engine or bench_rank or store_interleaved" -m gpu -x -v --timeout 700 --timeout-method thread || exit $?
$G 600 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
tail -1 $O/bench20.log
$G 1000 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
tail -1 $O/pytest_gpu.log
