#!/bin/bash
# round 6: persistent slab with release/acquire hand-off + residency refusal + timeout restore;
# fixed_k vs the board kernel; plain `bench.py --gpus 2` launch; fenced vs sc1-only hand-off A/B
set -u
O=gpurun_out/r06a
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/tests.log python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "persistent" tests/test_gpu_board.py tests/test_gpu_failfast.py::test_persistent_slab_timeout_restores_board || exit $?
tail -3 $O/tests.log
$G 200 $O/probe_fenced.log python -u scripts/probe_slabq.py 4096 3 || exit $?
GOLHIP_LIB=distributed-gol_amd/lib_sc1/libgolhip.so $G 200 $O/probe_sc1.log python -u scripts/probe_slabq.py 4096 3 || exit $?
$G 300 $O/plain.log python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu \
  tests/test_gpu_rank_host.py::test_bench_plain_launch_real_rccl_shared_gpu || exit $?
tail -3 $O/plain.log
