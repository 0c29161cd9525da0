#!/bin/bash
# round 3 (d): PMC + kernel-trace profile of the production small-board slab (configs[1] 5120^2,
# configs[4]-sized 4096^2 random, K = 16, with every count; 5120^2 also without counts)
set -u
O=gpurun_out/r03d
mkdir -p $O
export TMPDIR=/tmp
for cfg in "5120 counts" "4096 counts" "5120 nocounts"; do
  set -- $cfg; N=$1; C=$2
  P=/tmp/r03d_${N}_${C}
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $P/trace -o t -- python3 scripts/profile_small.py $N 16 4096 $C > $O/trace_${N}_${C}.log 2>&1 || exit 99
  python3 scripts/launch_timeline.py $P/trace 400 > $O/timeline_${N}_${C}.txt 2>&1
  i=0
  for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
              "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
              "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $P/p$i -o p -- python3 scripts/profile_small.py $N 16 4096 $C > $O/pmc_${N}_${C}_p$i.log 2>&1 || exit 99
  done
  python3 scripts/pmc_kernel_avg.py "gol_slab|count_finalize" $P/p1 $P/p2 $P/p3 > $O/pmc_${N}_${C}.json 2>&1
done
ls $O
