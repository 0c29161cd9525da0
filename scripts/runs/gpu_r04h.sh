#!/bin/bash
# round 4 (h): A/B of the split step's edge-stream priority and submission order on the ring of
# one (r04g ran both changes together: 1000-turn ring 16 % slower than r04f), tuning library
set -u
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for prio in 0 1; do for first in 0 1; do
  GOLHIP_LIB=distributed-gol_amd/lib_tuning/libgolhip.so GOLHIP_EDGE_PRIO=$prio GOLHIP_EDGE_FIRST=$first \
    $G 300 $O/predict_p${prio}_f${first}.log python3 scripts/predict_scaling.py 5 20,1000 160 1,8 || exit $?
  echo "prio=$prio first=$first"; grep "^{\"shape" $O/predict_p${prio}_f${first}.log | cut -c1-250
done; done
