#!/usr/bin/env python3
"""GCUPS of one (variant, k) at 65536^2 under several GOLHIP_LDS_PAD values (one process per
setting, since the pad is read once).  Usage: tune_env.py variant k pad1,pad2,..."""
import json
import subprocess
import sys

variant, k, pads = sys.argv[1], sys.argv[2], sys.argv[3].split(",")
res = {}
for pad in pads:
    env = {"GOLHIP_VARIANT": variant, "GOLHIP_LDS_PAD": pad}
    out = subprocess.run([sys.executable, "scripts/tune.py", "65536", k, "0", variant],
                         capture_output=True, text=True, env={**__import__("os").environ, **env})
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    res[f"{variant}_k{k}_pad{pad}"] = json.loads(line[0]) if line else out.stderr[-300:]
print(json.dumps(res))
