#!/bin/bash
# round 2 (ad): bulk depth A/B on a pre-heated chip: bench with max depth k = 12 / 14 / 16, alternating
set -o pipefail
O=gpurun_out/r02ad; mkdir -p $O
B="python3 bench.py --no-cpu --no-strong --no-flips --no-configs --no-sweep"
for rep in 1 2; do
  for K in 16 12 14; do
    timeout -k 10 200 $B --k $K > $O/k$K.$rep.json 2> $O/k$K.$rep.err || { echo "FAIL $K"; tail -3 $O/k$K.$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/k$K.$rep.json'));print('k$K', $rep, d['value'], 'cold', d['cold_start']['value'], d['parity']['ok'], d['roofline']['avg_launch_us'], d['roofline']['launch_depths'])"
  done
done
