#!/bin/bash
# round 2 (ao): bench with the device-wide sync closing the timed region: default and 20/5 x 2
set -u
O=gpurun_out/r02ao
mkdir -p $O
G=scripts/guard.sh
$G 400 $O/bench.log python3 bench.py || exit $?
$G 300 $O/bench20.log python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$G 300 $O/bench20b.log python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-sweep --no-strong --no-flips --no-configs || exit $?
echo done
