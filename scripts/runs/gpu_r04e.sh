#!/bin/bash
# round 4 (e): PMC of the production gol_slab2 launches (configs[1] 5120^2 and 4096^2 with every
# count; per-kernel keys), the driver's 20-turn split A/B, and the default bench line (CPU
# baseline with the T sweep) under rocprofv3 kernel stats
set -u
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for cfg in "5120 counts" "4096 counts"; do
  set -- $cfg; N=$1; C=$2
  P=/tmp/r04e_${N}_${C}
  $G 120 $O/trace_${N}_${C}.log rocprofv3 --kernel-trace --output-format csv -d $P/trace -o t -- python3 scripts/profile_small.py $N 16 4096 $C || exit $?
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
$G 300 $O/ab_split.log python3 scripts/ab_split.py prod 0,10,12,14,16 9 || exit $?
tail -8 $O/ab_split.log
$G 600 $O/bench_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r04e_prof -o b -- python3 bench.py || exit $?
grep "^{" $O/bench_prof.log > $O/bench_under_rocprof.json
find /tmp/r04e_prof -name "*kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
cut -c1-400 $O/bench_under_rocprof.json
