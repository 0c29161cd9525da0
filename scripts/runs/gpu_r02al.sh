#!/bin/bash
# round 2 (al): 262144^2 leg at max depth 16 vs 14 (pre-heated main run first)
set -o pipefail
O=gpurun_out/r02al; mkdir -p $O
for rep in 1 2; do
  for K in 16 14; do
    timeout -k 10 300 python3 bench.py --no-cpu --no-flips --no-configs --no-sweep --steps 20 --k $K > $O/s$K.$rep.json 2> $O/s$K.$rep.err || { echo "FAIL $K"; tail -3 $O/s$K.$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/s$K.$rep.json'));print('k$K', $rep, d['strong_262144']['gcups'], d['strong_262144']['parity']['ok'])"
  done
done
