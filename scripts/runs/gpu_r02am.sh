#!/bin/bash
# round 2 (am): timing events created outside the timed region; 20/5 runs x 3 + default, wall vs kernel time
set -o pipefail
O=gpurun_out/r02am; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-sweep --no-strong --no-flips --no-configs --steps 20 --warmup 5 > $O/b20.$r.json 2> $O/b20.$r.err || { tail -3 $O/b20.$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b20.$r.json'));r=d['roofline'];w=d['ms_per_step']*20*1e3;k=r['avg_launch_us']*r['launches'];print('20/5', d['value'], 'wall_us', round(w,1), 'kernel_us', round(k,1), 'host_us', round(w-k,1), 'cold', d['cold_start']['value'])"
done
timeout -k 10 200 python3 bench.py --no-cpu --no-sweep --no-strong --no-flips --no-configs > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));r=d['roofline'];w=d['ms_per_step']*1000*1e3;k=r['avg_launch_us']*r['launches'];print('default', d['value'], 'wall_us', round(w,1), 'kernel_us', round(k,1), 'host_us', round(w-k,1))"
