#!/bin/bash
# round 2 (z): same-call A/B of gol_slab before (lib_old) / after the halo-wave skip (lib), cfg2
set -o pipefail
O=gpurun_out/r02z; mkdir -p $O
for rep in 1 2; do
  for V in old:20812 new:20812 new:21208 new:1208; do
    L=${V%%:*}; S=${V##*:}; LIB=distributed-gol_amd/lib/libgolhip.so; [ $L = old ] && LIB=distributed-gol_amd/lib_old/libgolhip.so
    GOLHIP_LIB=$LIB GOLHIP_SLAB=$S timeout -k 10 120 python3 scripts/cfg2_time.py > $O/$L$S.$rep.json 2> $O/$L$S.$rep.err || { echo "FAIL $V"; tail -3 $O/$L$S.$rep.err; exit 1; }
    echo "$V $rep $(cat $O/$L$S.$rep.json)"
  done
done
