#!/bin/bash
# round 6 (b): the round's new GPU tests (persistent slab: release/acquire hand-off, residency
# refusal, timeout restore; 12 x 4 slabs; fixed_k vs the board kernel; host_bench configs[4];
# the fault library smoke; plain `bench.py --gpus 2`), then the A/Bs: persistent hand-off fenced vs
# sc1-only, 12 x 4 vs 16 x 4 slabs with and without counts, and the PMC of the production configs[4]
# counting slab.
set -u
O=gpurun_out/r06b
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
PT="python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu"
$G 500 $O/tests.log $PT tests/test_gpu_parity.py -k "persistent or 12x4 or 16x4" tests/test_gpu_board.py \
  tests/test_gpu_failfast.py::test_persistent_slab_timeout_restores_board tests/test_gpu_failfast.py::test_fault_library_selectors_smoke \
  tests/test_host.py tests/test_gpu_rank_host.py::test_bench_plain_launch_real_rccl_shared_gpu || exit $?
tail -3 $O/tests.log
$G 200 $O/probe_fenced.log python -u scripts/probe_slabq.py 4096 3 || exit $?
GOLHIP_LIB=distributed-gol_amd/lib_sc1/libgolhip.so $G 200 $O/probe_sc1.log python -u scripts/probe_slabq.py 4096 3 || exit $?
GOLHIP_LIB=distributed-gol_amd/lib_faults/libgolhip.so $G 300 $O/tune_12x4.log python -u scripts/tune_slab.py 2048,5120x512,1024 0,121604,91604 4096 || exit $?
P=/tmp/r06b_4096
$G 120 $O/trace_4096.log rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o t -- python3 scripts/profile_small.py 4096 16 4096 counts || exit $?
cp $P/trace/*/t_kernel_stats.csv $O/trace_4096_kernel_stats.csv 2>/dev/null || find $P/trace -name "*stats*" -exec cp {} $O/ \;
i=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  $G 90 $O/pmc_4096_p$i.log timeout -s KILL 80 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $P/p$i -o p -- python3 scripts/profile_small.py 4096 16 4096 counts || exit $?
done
python3 scripts/pmc_kernel_avg.py "gol_slab|count_finalize" $P/p1 $P/p2 > $O/pmc_4096.json 2>&1
head -c 3000 $O/pmc_4096.json
