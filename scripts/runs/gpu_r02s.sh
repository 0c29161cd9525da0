#!/bin/bash
# round 2 (s): bench with the cold-start leg, pre-heat and configs leg: driver shape (20/5) and default
set -o pipefail
mkdir -p gpurun_out/r02s
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r02s/bench20.json 2> gpurun_out/r02s/bench20.err || { tail -5 gpurun_out/r02s/bench20.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r02s/bench20.json'));print('20/5', d['value'], d['cold_start'], d['parity'], json.dumps(d['configs']))"
timeout -k 10 300 python3 bench.py > gpurun_out/r02s/bench.json 2> gpurun_out/r02s/bench.err || { tail -5 gpurun_out/r02s/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r02s/bench.json'));print('default', d['value'], d['cold_start'], d['parity'], d['roofline']['frac'])"
