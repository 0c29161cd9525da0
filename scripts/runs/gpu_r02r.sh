#!/bin/bash
# round 2 (r): does the driver's 20-turn run sit in a clock transient? bench with and without a
# pre-heat of the chip (untimed K-deep launches, board re-initialised before warmup + timed turns)
set -o pipefail
mkdir -p gpurun_out/r02r
B="python3 bench.py --steps 20 --warmup 5 --no-sweep --no-cpu --no-strong --no-flips"
for v in 0 100 300 0 100; do
  timeout -k 10 120 $B --preheat-ms $v > gpurun_out/r02r/b20_pre$v.json 2> gpurun_out/r02r/b20_pre$v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r02r/b20_pre$v.json'));print('preheat $v', d['value'], d['roofline']['avg_launch_us'], d['parity'])"
done
