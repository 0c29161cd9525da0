#!/bin/bash
# round 2 (af): bulk depth 12 vs 16 at 32768^2 and 131072^2 (pre-heated chip)
set -o pipefail
O=gpurun_out/r02af; mkdir -p $O
for rep in 1 2; do
  for K in 16 12; do
    for N in 32768 131072; do
      timeout -k 10 300 python3 bench.py --no-cpu --no-flips --no-configs --no-sweep --no-strong --size $N --steps 480 --k $K > $O/n$N.k$K.$rep.json 2> $O/n$N.k$K.$rep.err || { echo "FAIL $N $K"; tail -3 $O/n$N.k$K.$rep.err; exit 1; }
      python3 -c "import json;m=json.load(open('$O/n$N.k$K.$rep.json'));print('n$N k$K', $rep, m['value'], m['roofline']['launch_depths'])"
    done
  done
done
