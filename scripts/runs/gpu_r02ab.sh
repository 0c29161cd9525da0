#!/bin/bash
# round 2 (ab): slab parity, then configs[1] and configs[4] (every count) per slab shape, old vs new
set -o pipefail
O=gpurun_out/r02ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "slab or small_board or register or count" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for V in old:20812 new:20812 new:21208 new:1208; do
    L=${V%%:*}; S=${V##*:}; LIB=distributed-gol_amd/lib/libgolhip.so; [ $L = old ] && LIB=distributed-gol_amd/lib_old/libgolhip.so
    GOLHIP_LIB=$LIB GOLHIP_SLAB=$S timeout -k 10 120 python3 scripts/cfg2_time.py > $O/$L$S.$rep.json 2> $O/$L$S.$rep.err || { echo "FAIL $V"; tail -3 $O/$L$S.$rep.err; exit 1; }
    GOLHIP_LIB=$LIB GOLHIP_SLAB=$S timeout -k 10 120 python3 scripts/cfg2_time.py cfg5 > $O/c5_$L$S.$rep.json 2> $O/c5_$L$S.$rep.err || { echo "FAIL cfg5 $V"; tail -3 $O/c5_$L$S.$rep.err; exit 1; }
    echo "$V $rep $(cat $O/$L$S.$rep.json) $(cat $O/c5_$L$S.$rep.json)"
  done
done
