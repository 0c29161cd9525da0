#!/bin/bash
# round 2 (y): gol_slab halo waves skip counts, stores and all-garbage generations; 12x8 shapes
set -o pipefail
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "slab or small_board or register" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for S in 20812 21208 1208 20812; do
    GOLHIP_SLAB=$S timeout -k 10 120 python3 scripts/cfg2_time.py > $O/s$S.$rep.json 2> $O/s$S.$rep.err || { echo "FAIL $S"; tail -3 $O/s$S.$rep.err; exit 1; }
    echo "$S $rep $(cat $O/s$S.$rep.json)"
  done
done
