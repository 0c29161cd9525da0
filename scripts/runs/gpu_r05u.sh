#!/bin/bash
# round 5 (u): PMC of the whole-board kernel (512^2 forced, 256^2 and 64^2 automatic) and of the
# packed slab at 512^2, per kernel key: VALU instructions, wave cycles, VALU-active share, waits
set -u
O=gpurun_out/r05u
mkdir -p $O
export TMPDIR=/tmp
for cfg in "512 1 b512" "512 0 s512" "256 -1 b256" "64 -1 b64"; do
  set -- $cfg; N=$1; M=$2; TAG=$3
  P=/tmp/r05u_$TAG
  i=0
  for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
              "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $P/p$i -o p -- python3 scripts/profile_board.py $N 1000 $M > $O/pmc_${TAG}_p$i.log 2>&1 || exit 99
  done
  python3 scripts/pmc_kernel_avg.py "gol_board|gol_slabp" $P/p1 $P/p2 > $O/pmc_${TAG}.json 2>&1
done
for f in $O/pmc_*.json; do echo "== $f"; head -c 1500 $f; echo; done
