#!/usr/bin/env python3
"""Device -> host copy rate on the GPU box (the transfer that bounds the per-turn flips list):
torch page-locked and pageable destinations, several sizes, hipMemcpyAsync underneath.
Usage: python scripts/d2h_rate.py"""
import json
import time

import torch

res = {}
for mb in (2, 8, 64, 256):
    n = mb << 20
    dev = torch.empty(n, dtype=torch.uint8, device="cuda").fill_(1)
    for kind in ("pinned", "pageable"):
        host = torch.empty(n, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        host.copy_(dev, non_blocking=True)
        torch.cuda.synchronize()
        reps = max(3, 512 // mb)
        t = time.perf_counter()
        for _ in range(reps):
            host.copy_(dev, non_blocking=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / reps
        res[f"{kind}_{mb}MiB"] = round(n / dt / 1e9, 1)
print(json.dumps({"d2h_GBps": res}))
