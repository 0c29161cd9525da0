#!/usr/bin/env python3
"""From a rocprofv3 --hip-trace CSV: every device allocation / free call with its timestamp, plus
the kernel-free windows -- used to show that the snapshot (`s` key) path issues no hipMalloc or
hipFree once the engine exists (the per-shard stage is allocated at create).
Usage: hip_alloc_calls.py <hip_api_trace.csv>"""
import csv
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
names = Counter(r["Function"] for r in rows)
alloc = [r for r in rows if r["Function"] in ("hipMalloc", "hipFree", "hipHostMalloc", "hipHostFree",
                                               "hipMallocAsync", "hipFreeAsync", "hipExtMallocWithFlags")]
print(f"{len(rows)} HIP API calls; allocation/free calls: {len(alloc)}")
for fn in ("hipMalloc", "hipFree", "hipHostMalloc", "hipHostFree", "hipMemcpy2DAsync", "hipMemcpyAsync",
           "hipStreamSynchronize", "hipLaunchKernel", "hipGraphLaunch"):
    print(f"  {fn:24s} {names.get(fn, 0)}")
t0 = min(int(r["Start_Timestamp"]) for r in rows)
print("allocation/free calls in time order (ms since the first HIP call):")
for r in sorted(alloc, key=lambda r: int(r["Start_Timestamp"])):
    print(f"  {(int(r['Start_Timestamp']) - t0) / 1e6:10.3f}  {r['Function']}")
