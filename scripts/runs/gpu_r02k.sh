#!/bin/bash
# Why is gol_tile slow?  Kernel durations + PMC (issue/wait/ifetch) at 5120^2 k=16, tile T=16
# and the streaming split kernel, from scripts/profile_small.py.
set -u
O=gpurun_out/r02k
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for T in 16 0; do
  GOLHIP_TILE=$T $G 200 $O/tl_T$T.log rocprofv3 --kernel-trace --output-format csv -d $O/tl_T$T -o tl -- python3 scripts/profile_small.py 5120 16 1024 counts || exit $?
  python3 scripts/launch_timeline.py $O/tl_T$T 100 > $O/timeline_T$T.txt 2>&1
  i=0
  for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
              "SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
              "SQC_ICACHE_HITS SQC_ICACHE_MISSES"; do
    i=$((i+1))
    GOLHIP_TILE=$T $G 120 $O/pmc_T${T}_p$i.log rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $O/pmc_T${T}_p$i -o pmc -- python3 scripts/profile_small.py 5120 16 256 counts || exit $?
  done
done
echo done
