#!/bin/bash
# round 4 (y): PMC of the production end-flush slab launches (configs[1] 5120^2 16 x 6 and
# configs[4] 4096^2 12 x 7, every count), per-kernel keys; kernel-trace timeline beside them
set -u
O=gpurun_out/r04y
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for N in 5120 4096; do
  P=/tmp/r04y_${N}
  $G 120 $O/trace_${N}.log rocprofv3 --kernel-trace --output-format csv -d $P/trace -o t -- python3 scripts/profile_small.py $N 16 4096 counts || exit $?
  python3 scripts/launch_timeline.py $P/trace 400 > $O/timeline_${N}.txt 2>&1
  i=0
  for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
              "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
              "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $P/p$i -o p -- python3 scripts/profile_small.py $N 16 4096 counts > $O/pmc_${N}_p$i.log 2>&1 || exit 99
  done
  python3 scripts/pmc_kernel_avg.py "gol_slab|count_finalize" $P/p1 $P/p2 $P/p3 > $O/pmc_${N}.json 2>&1
  head -3 $O/timeline_${N}.txt
done
