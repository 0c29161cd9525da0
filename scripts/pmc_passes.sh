#!/bin/bash
# PMC passes for the stencil kernel (run on the GPU box from the repo root).
# One counter group per rocprofv3 run (no --sys-trace / --runtime-trace with --pmc); --kernel-trace
# beside each gives the dispatch durations (effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration).
# Usage: scripts/pmc_passes.sh <k> [extra bench args]
set -e
K=${1:-8}; shift || true
OUT=gpurun_out/pmc_k${K}
mkdir -p $OUT
export TMPDIR=/tmp
# --fixed-k: the launches are exactly K deep (the planner would run its best depth <= K: at
# 65536^2 that is 12 for K = 16, which the round-3 "pmc_k16" passes caught instead)
BENCH="python3 bench.py --no-cpu --no-sweep --no-strong --no-flips --no-configs --preheat-ms 0 --fixed-k --steps $((2*K)) --warmup 0 --k $K $*"
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $OUT/p$i -o pmc -- $BENCH > $OUT/p$i.log 2>&1
done
echo "pmc passes done: $OUT"
