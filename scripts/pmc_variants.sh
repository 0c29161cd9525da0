#!/bin/bash
# SQ counters + kernel durations of the stencil for several variants at one k (GPU box, repo root).
# Usage: scripts/pmc_variants.sh K "variant1 variant2 ..." [size]
K=${1:-8}; VARS=${2:-"chainlds chainlds2"}; SIZE=${3:-65536}
OUT=gpurun_out/pmcv_k${K}
mkdir -p $OUT
export TMPDIR=/tmp
# the variants live in the tuning build (lib/libgolhip.so has only the production kernels)
export GOLHIP_LIB=$PWD/distributed-gol_amd/lib_tuning/libgolhip.so
for V in $VARS; do
  export GOLHIP_VARIANT=$V
  BENCH="python3 bench.py --no-cpu --no-sweep --steps $((4*K)) --warmup $K --k $K --size $SIZE"
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$V/trace -o t -- $BENCH > $OUT/$V.trace.log 2>&1 || exit 99
  i=0
  for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
              "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/$V/p$i -o pmc -- $BENCH > $OUT/$V.p$i.log 2>&1 || exit 99
  done
done
python3 scripts/pmc_variants_summary.py $OUT
