#!/bin/bash
# round 2 (x): where configs[1]'s count cost goes -- gol_slab builds: production (uniform-mask
# counts), OLDSEL (previous select), NOPOP (no per-row popcounts), NOFLUSH (no end-of-launch flush)
set -o pipefail
O=gpurun_out/r02x; mkdir -p $O
for rep in 1 2; do
  for L in lib lib_OLDSEL lib_NOPOP lib_NOFLUSH; do
    GOLHIP_LIB=distributed-gol_amd/$L/libgolhip.so timeout -k 10 120 python3 scripts/cfg2_time.py > $O/$L.$rep.json 2> $O/$L.$rep.err || { echo "FAIL $L"; tail -3 $O/$L.$rep.err; exit 1; }
    echo "$L $rep $(cat $O/$L.$rep.json)"
  done
done
