#!/bin/bash
# round 3 (w): why 33 chunks (pre63) run no faster than 34 at K = 12: SQ_INSTS_VALU, busy/wait
# cycles and the effective clock of one fixed-depth K = 12 launch of each geometry
set -u
O=gpurun_out/r03w
mkdir -p $O
export TMPDIR=/tmp GOLHIP_FIXED_K=1
BENCH="python3 bench.py --no-cpu --no-sweep --no-strong --no-flips --no-configs --preheat-ms 0 --steps 24 --warmup 0 --k 12"
for v in prod pre63; do
  i=0
  for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
              "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
              "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    GOLHIP_VARIANT=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $O/${v}_p$i -o pmc -- $BENCH > $O/${v}_p$i.log 2>&1 || { echo "pass $v $i failed"; exit 1; }
  done
done
echo pmc done
