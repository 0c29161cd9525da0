#!/bin/bash
# round 3 (i): same-call A/B of the small-board slab: B = the previous library (lib_prev, commit
# 9e14dbf: sums exchange + shape model, no packing) vs A = packing of the narrow last chunk
# (GOLHIP_SLAB_PACK=1) vs A without packing (=0); two interleaved rounds each
set -u
O=gpurun_out/r03i
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for r in 1 2; do
  GOLHIP_LIB=distributed-gol_amd/lib_prev/libgolhip.so $G 200 $O/B_$r.log python3 scripts/tune_slab.py 4096,5120 0,21207,21208,20812 || exit $?
  $G 200 $O/Apack_$r.log python3 scripts/tune_slab.py 4096,5120 0,21207,21208,20812,21206 || exit $?
  GOLHIP_SLAB_PACK=0 $G 200 $O/Anopack_$r.log python3 scripts/tune_slab.py 4096,5120 0,21207,21208,20812,21206 || exit $?
done
for f in $O/*.log; do echo "== $f"; grep "^{" $f | cut -c1-600; done
