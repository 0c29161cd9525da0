#!/bin/bash
# round 2 (ae): bulk depth 12 vs 16 on the 262144^2 leg and on a 16384^2 board (pre-heated chip)
set -o pipefail
O=gpurun_out/r02ae; mkdir -p $O
for rep in 1 2; do
  for K in 16 12; do
    timeout -k 10 300 python3 bench.py --no-cpu --no-flips --no-configs --no-sweep --steps 20 --k $K > $O/s$K.$rep.json 2> $O/s$K.$rep.err || { echo "FAIL $K"; tail -3 $O/s$K.$rep.err; exit 1; }
    timeout -k 10 300 python3 bench.py --no-cpu --no-flips --no-configs --no-sweep --no-strong --size 16384 --steps 2000 --k $K > $O/m$K.$rep.json 2> $O/m$K.$rep.err || { echo "FAIL m$K"; tail -3 $O/m$K.$rep.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/s$K.$rep.json'));m=json.load(open('$O/m$K.$rep.json'))
print('k$K', $rep, 'strong262144', d['strong_262144']['gcups'], d['strong_262144']['parity']['ok'], '16384:', m['value'], m['roofline']['launch_depths'])"
  done
done
