#!/usr/bin/env python3
"""k = 1 tuning: GCUPS of gol_step1 at 65536^2 per GOLHIP_STEP1 config (P*10 + NT) x band rows,
one process per config (the knob is read once).  Usage: tune_step1.py [cfgs] [bands] [size]"""
import json
import os
import subprocess
import sys

cfgs = (sys.argv[1] if len(sys.argv) > 1 else "40,41,42,43,80,81,82,83,120,122,160,162").split(",")
bands = sys.argv[2] if len(sys.argv) > 2 else "0,32,64,128,256,512"
size = sys.argv[3] if len(sys.argv) > 3 else "65536"
res = {}
for c in cfgs:
    env = {**os.environ, "GOLHIP_STEP1": c}
    out = subprocess.run([sys.executable, "scripts/tune.py", size, "1", bands, "lds"],
                         capture_output=True, text=True, env=env, timeout=300)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    res[c] = json.loads(line[0]) if line else out.stderr[-300:]
    print(c, res[c], flush=True)
print(json.dumps(res))
