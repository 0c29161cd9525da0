#!/bin/bash
# Round-2 GPU session C: why is the drift kernel at ~78% of its VALU mix?  Counter list, per-variant
# SQ/SQC counters + kernel durations at K=16, interleaved tune of the variants.
set -u
O=gpurun_out/r02c
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
scripts/guard.sh 300 $O/pytest_nf.log python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "variant and driftnf" || exit $?
grep -q " failed" $O/pytest_nf.log && exit 1
TUNE_STEPS=256 scripts/guard.sh 300 $O/tune.log python -u scripts/tune.py 65536 12,16 0 driftlds,driftnf,drift62,driftzip || exit $?
for V in driftlds driftnf driftzip; do
  export GOLHIP_VARIANT=$V
  BENCH="python3 bench.py --no-cpu --no-sweep --no-strong --steps 64 --warmup 16 --k 16"
  mkdir -p $O/$V
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$V/trace -o t -- $BENCH > $O/$V.trace.log 2>&1 || exit 99
  i=0
  for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
              "SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_IFETCH SQ_INSTS_SMEM"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $O/$V/p$i -o pmc -- $BENCH > $O/$V.p$i.log 2>&1 || exit 99
  done
done
echo done > $O/done.txt
