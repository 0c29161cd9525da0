#!/bin/bash
# round 3 (p): pre-heated lockstep A/B of pre63 vs the production geometry (65536^2 at K = 8/12/16,
# 262144^2 at K = 12/16), and the driver's 20/5 bench line under each (legs off)
set -u
O=gpurun_out/r03p
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
AB_STEPS=480 $G 300 $O/ab_65536.log python3 scripts/ab_variant.py 65536 8,12,16 prod,pre63 9 || exit $?
tail -3 $O/ab_65536.log
AB_STEPS=96 $G 400 $O/ab_262144.log python3 scripts/ab_variant.py 262144 12,16 prod,pre63 5 || exit $?
tail -2 $O/ab_262144.log
for i in 1 2; do
for v in prod pre63; do
GOLHIP_VARIANT=$v $G 300 $O/bench20_${v}_$i.log python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-configs --no-flips --no-sweep --no-strong || exit $?
grep "^{" $O/bench20_${v}_$i.log | cut -c1-120
done
done
