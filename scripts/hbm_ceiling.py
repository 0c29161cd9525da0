#!/usr/bin/env python3
"""Achievable HBM rate on this box for the step1 traffic shape: a 512 MiB -> 512 MiB device copy
(torch copy_ kernel and hipMemcpy DtoD via torch), the same bytes a one-generation launch moves at
65536^2.  Prints GB/s (read + write bytes / time)."""
import json
import torch

n = 1 << 29
a = torch.empty(n, dtype=torch.uint8, device="cuda").random_()
b = torch.empty_like(a)
res = {}
for name, f in [("copy_u8", lambda: b.copy_(a)),
                ("copy_i64view", lambda: b.view(torch.int64).copy_(a.view(torch.int64))),
                ("clone", lambda: a.clone())]:
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        f()
    e.record()
    e.synchronize()
    t = s.elapsed_time(e) / 50 / 1e3
    res[name] = {"us": round(t * 1e6, 1), "GBps": round(2 * n / t / 1e9, 1)}
print(json.dumps(res))
