#!/bin/bash
# round 2 (an): host submit/sync latency of the 20-turn region with HSA signal waits polled
# (HSA_ENABLE_INTERRUPT=0) vs the default interrupt-driven waits, alternating
set -o pipefail
O=gpurun_out/r02an; mkdir -p $O
for r in 1 2; do
  for V in default poll; do
    E=""; [ $V = poll ] && E="HSA_ENABLE_INTERRUPT=0"
    env $E timeout -k 10 200 python3 bench.py --no-cpu --no-sweep --no-strong --no-flips --no-configs --steps 20 --warmup 5 > $O/$V.$r.json 2> $O/$V.$r.err || { tail -3 $O/$V.$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$V.$r.json'));r=d['roofline'];w=d['ms_per_step']*20*1e3;k=r['avg_launch_us']*r['launches'];print('$V', d['value'], 'wall_us', round(w,1), 'kernel_us', round(k,1), 'host_us', round(w-k,1), 'cold', d['cold_start']['value'])"
  done
done
