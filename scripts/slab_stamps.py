#!/usr/bin/env python3
"""Where a small-board gol_slab2 launch's time goes, from per-wave phase stamps (tuning build,
GOLHIP_VARIANT=stamp; graphs off so every launch goes through the stamped path).  Per launch:
  span      first wave start -> last wave end (us)
  ramp      spread of the waves' start times (dispatch of the grid)
  load      start -> rows loaded (the wave's S input rows from L2/HBM)
  gens      rows loaded -> K generations done (the barrier-paced generation loop)
  flush     generations done -> end (the count flush and the last stores leaving the wave)
  drain     last wave end - the median wave end (the launch's tail)
Usage: slab_stamps.py [sizes] [launches] [counts 0/1]"""
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
os.environ.setdefault("GOLHIP_LIB", str(ROOT / "distributed-gol_amd" / "lib_tuning" / "libgolhip.so"))
os.environ["GOLHIP_VARIANT"] = "stamp"
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import golhip  # noqa: E402

sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "5120,4096").split(",")]
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 4
counts = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
L = golhip.load_library()
L.golhip_tuning_stamps_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int)]
L.golhip_tuning_stamps_ex.restype = ctypes.c_int


def stamps(e):
    n, wpw = ctypes.c_size_t(0), ctypes.c_int(0)
    assert L.golhip_tuning_stamps_ex(e._h, None, 0, ctypes.byref(n), ctypes.byref(wpw)) == 0
    out = np.zeros(max(n.value, 8), dtype=np.uint64)
    assert L.golhip_tuning_stamps_ex(e._h, out.ctypes.data, out.size, ctypes.byref(n), ctypes.byref(wpw)) == 0
    assert wpw.value == 8, f"not a gol_slab2 launch ({wpw.value} words per wave)"
    st = out[: n.value].reshape(-1, 8)
    return st[st[:, 0] != 0]  # the host's wave count is an upper bound: records of waves that ran


def pct(a, q):
    return round(float(np.percentile(a, q)), 2)


def analyse(st):
    t = st[:, :4].astype(np.int64)
    t = (t - t[:, 0].min()) * 10.0 / 1e3  # 100 MHz ticks -> us from the first start
    load, gens, flush = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    dur = t[:, 3] - t[:, 0]
    ghz = st[:, 4].astype(np.float64) / (dur * 1e3)
    end_med = float(np.median(t[:, 3]))
    return {"waves": int(len(st)), "workgroups": int(len(set(st[:, 6].tolist()))),
            "span_us": round(float(t[:, 3].max()), 2),
            "ramp_us": {"p50": pct(t[:, 0], 50), "p95": pct(t[:, 0], 95), "max": round(float(t[:, 0].max()), 2)},
            "load_us": {"p50": pct(load, 50), "p95": pct(load, 95)},
            "gens_us": {"p50": pct(gens, 50), "p95": pct(gens, 95)},
            "flush_us": {"p50": pct(flush, 50), "p95": pct(flush, 95)},
            "wave_us": {"p50": pct(dur, 50), "p95": pct(dur, 95)},
            "drain_us": round(float(t[:, 3].max()) - end_med, 2),
            "clock_ghz_median": round(float(np.median(ghz)), 3)}


res = {}
for n in sizes:
    e = golhip.Engine(n, n, k=16)
    e.set_graphs(0)
    e.init_random(2)
    e.step(512, counts=counts)  # pre-heat
    e.sync()
    e.step(16, counts=counts)
    e.sync()
    raw = stamps(e)
    np.save(ROOT / "gpurun_out" / f"slab_stamps_{n}_{int(counts)}.npy", raw)
    out = []
    for i in range(nl):
        e.step(16, counts=counts)
        e.sync()
        a = analyse(stamps(e))
        out.append(a)
        print(json.dumps({"size": n, "launch": i, "counts": counts, **a}), flush=True)
    res[str(n)] = out
    e.close()
print(json.dumps({"slab_stamps": res}))
