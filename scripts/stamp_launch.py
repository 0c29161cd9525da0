#!/usr/bin/env python3
"""Where a streaming launch's time goes, from per-wave timestamps (tuning build,
GOLHIP_VARIANT=stamp: the production gol_stencil plus s_memrealtime / s_memtime stamps at each
wave's start and end and its HW_ID / XCC_ID).  Per launch:
  span          first wave start -> last wave end (us)
  start_skew    spread of the start times of the first round of waves (dispatch ramp, us)
  wave_us       per-wave duration: mean / p5 / p95
  clock_ghz     in-kernel shader clock: median over waves of cycles / duration
  tail_us       per SIMD: kernel end - the SIMD's last wave end (mean, p95): the idle tail
  occupancy     wave-slot-time the waves used / (SIMDs x resident waves x span)
Usage: stamp_launch.py [size] [k list] [launches per k] [preheat ms]"""
import ctypes
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
os.environ.setdefault("GOLHIP_LIB", str(ROOT / "distributed-gol_amd" / "lib_tuning" / "libgolhip.so"))
os.environ["GOLHIP_VARIANT"] = "stamp"
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import golhip  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
ks = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "12,8,14,16").split(",")]
nl = int(sys.argv[3]) if len(sys.argv) > 3 else 4
preheat_ms = float(sys.argv[4]) if len(sys.argv) > 4 else 300.0
L = golhip.load_library()
L.golhip_tuning_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t)]
L.golhip_tuning_stamps.restype = ctypes.c_int


def stamps(e):
    n = ctypes.c_size_t(0)
    assert L.golhip_tuning_stamps(e._h, None, 0, ctypes.byref(n)) == 0
    out = np.zeros((max(n.value, 1), 4), dtype=np.uint64)
    assert L.golhip_tuning_stamps(e._h, out.ctypes.data, n.value, ctypes.byref(n)) == 0
    return out[: n.value]


def analyse(st):
    t0 = st[:, 0].astype(np.int64)
    t1 = st[:, 1].astype(np.int64)
    cyc = st[:, 2].astype(np.float64)
    hw = st[:, 3].astype(np.uint64)
    base = t0.min()
    t0, t1 = (t0 - base) * 10.0 / 1e3, (t1 - base) * 10.0 / 1e3  # 100 MHz ticks -> us
    dur = t1 - t0
    span = float(t1.max())
    # SIMD key: XCC, SE, SH, CU, SIMD of HW_ID (wave id and queue fields dropped)
    h = hw & np.uint64(0xFFFFFFFF)
    key = ((hw >> np.uint64(32)) << np.uint64(16)) | (((h >> np.uint64(13)) & np.uint64(7)) << np.uint64(10)) | \
        (((h >> np.uint64(12)) & np.uint64(1)) << np.uint64(9)) | (((h >> np.uint64(8)) & np.uint64(15)) << np.uint64(4)) | \
        ((h >> np.uint64(4)) & np.uint64(3))
    simds = {}
    for k_, a, b in zip(key.tolist(), t0.tolist(), t1.tolist()):
        simds.setdefault(k_, []).append((a, b))
    def max_conc(iv):
        ev = sorted([(a, 1) for a, _ in iv] + [(b, -1) for _, b in iv], key=lambda x: (x[0], x[1]))
        c = m = 0
        for _, d in ev:
            c += d
            m = max(m, c)
        return m
    resident = max(max_conc(v) for v in simds.values())  # waves per SIMD the launch reached
    tails = [span - max(b for _, b in v) for v in simds.values()]
    heads = [min(a for a, _ in v) for v in simds.values()]
    first_round = np.sort(t0)[: min(len(t0), len(simds) * resident)]
    ghz = cyc / (dur * 1e3)
    return {"waves": int(len(st)), "simds_seen": len(simds), "resident_per_simd": resident,
            "span_us": round(span, 2),
            "start_skew_us": round(float(first_round.max() - first_round.min()), 2),
            "wave_us": {"mean": round(float(dur.mean()), 2), "p5": round(float(np.percentile(dur, 5)), 2),
                        "p95": round(float(np.percentile(dur, 95)), 2)},
            "clock_ghz_median": round(float(np.median(ghz)), 3),
            "head_us": {"mean": round(statistics.mean(heads), 2), "max": round(max(heads), 2)},
            "tail_us": {"mean": round(statistics.mean(tails), 2), "p95": round(float(np.percentile(tails, 95)), 2),
                        "max": round(max(tails), 2)},
            "occupancy": round(float(dur.sum()) / (len(simds) * resident * span), 4)}


res = {}
e = golhip.Engine(size, size, k=max(ks))
e.set_fixed_k(True)
e.init_random(3)
t = time.perf_counter()
while (time.perf_counter() - t) * 1e3 < preheat_ms:
    e.step(16)
    e.sync()
for K in ks:
    e.set_k(K)
    e.init_random(3)
    e.step(5)  # the driver's warmup: the densest turns follow
    out = []
    for i in range(nl):
        e.step(K)
        e.sync()
        a = analyse(stamps(e))
        out.append(a)
        print(json.dumps({"k": K, "launch": i, **a}), flush=True)
    res[str(K)] = out
print(json.dumps({"size": size, "stamps": res}))
