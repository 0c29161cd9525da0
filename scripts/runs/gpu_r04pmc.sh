#!/bin/bash
# round 4: PMC passes of the final tree's K = 14 and K = 12 launches at 65536^2 (fixed depth, the
# dense start), summarised with the calibrated HBM scales (scripts/pmc_summary.py)
set -u
for K in 14 12; do
  timeout -k 10 900 bash scripts/pmc_passes.sh $K || exit $?
  python3 scripts/pmc_summary.py gpurun_out/pmc_k$K $K 536870912 gpurun_out/r04_pmc_traffic.json 65536x65536_k$K > gpurun_out/pmc_k${K}_summary.txt 2>&1 || exit $?
  tail -12 gpurun_out/pmc_k${K}_summary.txt
done
