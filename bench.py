#!/usr/bin/env python3
"""Benchmark of the hot path: GCUPS and % of the HBM roofline of the gfx950 stencil.

A "step" is one generation (turn) of the whole board: one Broker.Publish -> 4x GolOP.Work round
of the reference (broker/broker.go:157-180, server/server.go:77-107).

Workload (BASELINE.json configs[2], the metric's "65536^2 @1 GPU"): a 65536 x 65536 random
board (p = 0.5, seed 3) per GPU.  With --gpus N (one process per GPU, launched by
torch.distributed.run) the board is 65536 wide and 65536*N tall, split into N row strips with
k-row RCCL halo exchange over xGMI (weak scaling: per-GPU work fixed).  --size/--height select
other boards (e.g. --size 262144 for configs[3], strong scaling).

Prints ONE JSON line on rank 0 (keys per the driver contract), plus:
  roofline     : algorithmic bytes (0.25 B per cell-update) per stencil launch / the launch's
                 average duration from HIP events recorded on the engine's compute stream;
  valu_roofline: the stencil's actual bound for k >= 4 -- algorithmic wave64 VALU instructions
                 (13 per 32-cell word per generation) per second vs the issue peak of that mix;
  cpu_baseline : the reference algorithm (oracle/ port of server/server.go + broker split,
                 byte per cell, 4 servers x T threads) timed on this host on a bounded sample;
  k_sweep      : GCUPS per temporal-blocking depth k (N == 1 only);
  hbm_roofline_k1: the k = 1 kernel (gol_step1, no temporal reuse) against the HBM peak;
  strong_262144: configs[3] -- the 262144^2 board (seed 4) split over the N ranks, GCUPS and
                 GCUPS per GPU (strong scaling of one fixed board; --no-strong skips it).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))

import torch  # noqa: E402  (first: one HIP runtime per process, see golhip.py)
import torch.distributed as dist  # noqa: E402

import golhip  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BYTES_PER_CELL_UPDATE = 0.25  # 1 packed bit read + 1 packed bit written per cell per generation
# VALU roofline of the stencil (the bound for k >= 4): 12 wave64 VALU
# instructions per 32-cell word per generation with drifting row sums (9 v_bitop3 at full rate,
# 2 v_alignbit + 1 DPP move at half rate).  Peak issue = 1024 SIMDs x 2.4 GHz / cycles per
# instruction, where a full-rate wave64 op takes 2 cycles (SIMD-32) and a half-rate one 4: the
# mix averages 30 cycles per 12 instructions.  Reported as instruction issue rate (wave64 VALU
# instructions per second).
VALU_PER_WORD_GEN = 12
VALU_CYCLES_PER_WORD_GEN = 9 * 2 + 3 * 4
SIMDS, PEAK_CLOCK_GHZ = 1024, 2.4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000, help="timed generations (configs[2]: 1000 turns)")
    ap.add_argument("--warmup", type=int, default=8, help="untimed generations")
    ap.add_argument("--size", type=int, default=65536, help="board width")
    ap.add_argument("--height", type=int, default=0,
                    help="total board height (default: size * N, weak scaling)")
    ap.add_argument("--k", type=int, default=16, help="generations per stencil launch")
    ap.add_argument("--band-rows", type=int, default=0)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-sweep", action="store_true", help="skip the k sweep")
    ap.add_argument("--cpu-size", type=int, default=16384)
    ap.add_argument("--cpu-turns", type=int, default=96)
    ap.add_argument("--no-timing", action="store_true",
                    help="no per-launch HIP events in the timed region (roofline from wall time)")
    ap.add_argument("--pmc-file", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the configs[3] leg (262144^2 board split over the N ranks)")
    ap.add_argument("--strong-size", type=int, default=262144)
    ap.add_argument("--strong-steps", type=int, default=160)
    return ap.parse_args()


def timed_steps(eng: golhip.Engine, steps: int, world: int) -> float:
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.sync()
    t0 = time.perf_counter()
    eng.step(steps)
    eng.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def cpu_baseline(size: int, turns: int, threads_per_server: int) -> dict:
    """The reference's algorithm (oracle/gol_oracle.c oracle_ref_*), timed on this host."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np

    import oracle

    board = oracle.unpack(oracle.init_random(size, size, seed=3), size)
    t0 = time.perf_counter()
    oracle.ref_run(board, turns, threads=threads_per_server, servers=4, fanout_copy=False)
    dt = time.perf_counter() - t0
    cups = size * size * turns / dt
    del board, np
    return {
        "value": round(cups / 1e9, 4),
        "unit": "GCUPS",
        "cores": 4 * threads_per_server,
        "kind": "port",
        "sample": (f"{size}x{size} random p=0.5 seed 3, {turns} turns of the reference algorithm "
                   f"(byte cells, branchy torus wrap + /255, fresh rows per turn, 4 broker strips x "
                   f"{threads_per_server} goroutine-threads = {4 * threads_per_server} OS threads); "
                   f"gob/TCP fan-out excluded; {dt:.1f} s"),
    }


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)

    width = a.size
    height = a.height or a.size * world
    nccl_id = None
    if world > 1:
        obj = [golhip.nccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        nccl_id = obj[0]
    eng = golhip.Engine(width, height, k=a.k, rank=rank, world_size=world, device=local,
                        nccl_id=nccl_id)
    if a.band_rows:
        eng.set_band_rows(a.band_rows)
    eng.init_random(a.seed)
    local_rows = eng.info.rows
    local_cells = local_rows * width

    eng.step(a.warmup)
    eng.sync()

    # timed region: exactly a.steps generations, per-launch HIP events on the compute stream
    eng.timing(not a.no_timing)
    dt = timed_steps(eng, a.steps, world)
    kern_ms, launches, gens = eng.kernel_time()
    eng.timing(False)
    # regression canary: alive cells after exactly warmup + steps generations (deterministic for
    # the seed; compare across kernel versions)
    alive_timed = eng.alive_count()
    if a.no_timing:
        launches = -(-a.steps // a.k)
        kern_ms, gens = dt * 1e3, a.steps

    total_updates = width * height * a.steps
    gcups = total_updates / dt / 1e9
    ms_per_step = dt * 1e3 / a.steps

    # roofline of the dominant kernel (gol_stencil<k>) on this rank
    avg_launch_ms = kern_ms / max(launches, 1)
    gens_per_launch = gens / max(launches, 1)
    alg_bytes_per_launch = BYTES_PER_CELL_UPDATE * local_cells * gens_per_launch
    achieved = alg_bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9
    # VALU roofline: algorithmic wave-instructions per launch (the cells it updates, no halo or
    # pipeline-fill work) over the launch time, against the issue peak for the same mix
    words_per_launch = local_cells / 32 * gens_per_launch
    valu_instr = words_per_launch / 64 * VALU_PER_WORD_GEN
    valu_achieved = valu_instr / (avg_launch_ms * 1e-3) / 1e12
    valu_peak = SIMDS * PEAK_CLOCK_GHZ * 1e9 / (VALU_CYCLES_PER_WORD_GEN / VALU_PER_WORD_GEN) / 1e12
    valu = {"bound": "valu", "achieved": round(valu_achieved, 4), "peak": round(valu_peak, 4),
            "unit": "T wave64-instr/s", "frac": round(valu_achieved / valu_peak, 4),
            "mix": "12 per 32-cell word per generation: 9 v_bitop3 (2 cyc) + 2 v_alignbit + 1 DPP (4 cyc)",
            "note": "peak at 2.4 GHz; the dense start runs at 1.9-2.2 GHz (power)"}
    traffic = None
    try:
        pmc = json.loads(Path(a.pmc_file).read_text())
        key = f"{width}x{eng.info.rows}_k{a.k}"
        if key in pmc:
            traffic = pmc[key]["hbm_bytes_per_launch"]
    except Exception:
        pass

    sweep = None
    k1_launch_us = None
    if world == 1 and not a.no_sweep:
        sweep = {}
        for kk in (1, 2, 4, 8, 16, 32):
            eng.set_k(kk)
            # the first ~250 one-generation launches of a process run ~10 % slower (measured,
            # scripts/diag_k1.py), so k = 1 gets a longer untimed warmup
            eng.step(256 if kk == 1 else 2 * kk)
            n = max(4 * kk, 256)
            eng.timing(kk == 1)
            t = timed_steps(eng, n, 1)
            if kk == 1:
                ms1, l1, _ = eng.kernel_time()
                k1_launch_us = ms1 * 1e3 / max(l1, 1)
                eng.timing(False)
            sweep[str(kk)] = round(width * height * n / t / 1e9, 1)
        eng.set_k(a.k)

    checksum = eng.alive_count()  # collective
    eng.close()
    del eng

    # configs[3]: the 262144^2 board (seed 4) row-strip sharded over the N ranks (strong scaling
    # of a fixed board; per-GPU rate comparable across N), RCCL halos when N > 1
    strong = None
    if not a.no_strong:
        n = a.strong_size
        sid = None
        if world > 1:  # a fresh RCCL unique id per communicator
            obj = [golhip.nccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            sid = obj[0]
        se = golhip.Engine(n, n, k=a.k, rank=rank, world_size=world, device=local, nccl_id=sid)
        se.init_random(4)
        se.step(a.k)
        se.sync()
        t = timed_steps(se, a.strong_steps, world)
        strong_alive = se.alive_count()  # collective
        se.close()
        del se
        g = n * n * a.strong_steps / t / 1e9
        strong = {"board": f"{n}x{n}", "seed": 4, "steps": a.strong_steps, "k": a.k,
                  "rows_per_gpu": -(-n // world), "gcups": round(g, 1),
                  "gcups_per_gpu": round(g / world, 1), "ms_per_step": round(t * 1e3 / a.strong_steps, 4),
                  "alive_after": int(strong_alive)}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(a.cpu_size, a.cpu_turns, threads_per_server=4)

    if rank == 0:
        line = {
            "metric": "cell-updates/sec (GCUPS)",
            "value": round(gcups, 2),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak" if not a.height else "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (counter-based splitmix64 random board, p=0.5, generated on device)",
            "config": {
                "workload": (f"{width}x{height} torus, random p=0.5 seed {a.seed}, "
                             f"{world} row strip(s) of {local_rows} rows, k={a.k} gens/launch"),
                "width": width, "height": height, "k": a.k, "parallelism": f"rows{world}",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "gol_step1" if a.k == 1 else f"gol_stencil<{a.k}>",
                "avg_launch_us": round(avg_launch_ms * 1e3, 2),
                "gens_per_launch": gens_per_launch,
            },
            "valu_roofline": valu,
            "cpu_baseline": cpu,
            "k_sweep_gcups": sweep,
            # the north star's HBM figure for the one-generation kernel (no temporal reuse):
            # k = 1 sweep rate x 0.25 B per cell-update vs the 8 TB/s peak
            # (algorithmic bytes of one launch over its HIP-event duration, as for "roofline")
            "hbm_roofline_k1": None if not k1_launch_us else {
                "kernel": "gol_step1", "gcups_wall": sweep["1"],
                "avg_launch_us": round(k1_launch_us, 2),
                "achieved": round(BYTES_PER_CELL_UPDATE * local_cells / k1_launch_us / 1e3, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(BYTES_PER_CELL_UPDATE * local_cells / k1_launch_us / 1e3 / HBM_PEAK_GBS, 4)},
            "strong_262144": strong,
            "alive_after_timed": int(alive_timed),
            "alive_after": int(checksum),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
