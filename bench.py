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
  roofline     : the bound of the timed kernel.  k >= 2 (temporal blocking, VALU-bound):
                 algorithmic wave64 VALU instructions (12 per 32-cell word per generation) per
                 launch / the launch's average duration from HIP events on the engine's compute
                 stream, against the VALU issue peak (1024 SIMDs x 2.4 GHz / 2 cycles per wave64
                 instruction, MI355X_MICROARCH.md "Wave scheduling"); the PMC-measured issued
                 count (SQ_INSTS_VALU) and clock (GRBM_GUI_ACTIVE / 8 / duration) of the same
                 kernel from profiles/pmc_traffic.json beside it.  k == 1: HBM bytes (0.25 B per
                 cell-update) against 8 TB/s;
  hbm_roofline : the algorithmic-HBM figure of the same timed launches (exceeds 1 for k > 1:
                 temporal blocking reads and writes the board once per k generations);
  parity       : alive cells after warmup + steps generations == the oracle's golden count
                 (tests/golden/cfg3_65536_seed3_counts.csv) when that turn is pinned, and the
                 whole board's digest (SHA-256 of 4096-row chunk SHA-256s, each rank hashing its
                 own strip after the timed pass) == the oracle's (tests/golden synthetic_golden.json
                 digest_65536x*, turns 25 and 1008): bit-exact, not only count-exact;
  cpu_baseline : the reference algorithm (oracle/ port of server/server.go + broker split,
                 byte per cell, 4 servers x T goroutine-threads from a persistent pool, full-world
                 fan-out copy per server per turn, per-turn alive scan) timed on this host: a T sweep
                 (T = 1, 2, 4, 8, 16, the cgroup quota / 4 and every host core / 4) on configs[0]
                 (512^2 x 100, bit-exact) and the first 20 turns of configs[1]; the bench board at the
                 best T; configs[4]'s first turns; configs[3] (262144^2) extrapolated;
  k_sweep      : GCUPS per temporal-blocking depth k (N == 1 only);
  hbm_roofline_k1: the k = 1 kernel (gol_step1, no temporal reuse) against the HBM peak;
  strong_262144: configs[3] -- the 262144^2 board (seed 4) split over the N ranks, GCUPS and
                 GCUPS per GPU (strong scaling of one fixed board; --no-strong skips it);
  configs      : configs[0], [1], [4] on the GPU (512^2 PGM x 100, 5120^2 x 10 000 and 4096^2 x
                 1e6 turns, every count), each checked against the reference fixture / goldens;
  cold_start   : the same warmup + timed turns run first, on the chip as the process found it.

Timing order: cold-start pass (warmup + steps, reported as cold_start) -> --preheat-ms of untimed
K-deep launches -> the board is re-initialised from the seed -> warmup -> the timed steps (value).
The MI355X's clock ramps over the first tens of ms of load: a 20-turn region right after an idle
start runs ~10 % slower than the same turns on a loaded chip (profiles/r02/r02r_preheat.txt), so
value is the loaded-clock rate and cold_start keeps the idle-start figure beside it.
"""
from __future__ import annotations

import argparse
import datetime
import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))


def _hw_queues(argv) -> int:
    """--hw-queues N (default 8; 0 leaves the environment alone), read before anything starts
    the HIP runtime: it reads GPU_MAX_HW_QUEUES once, at its initialisation."""
    for i, x in enumerate(argv):
        if x == "--hw-queues" and i + 1 < len(argv):
            return int(argv[i + 1])
        if x.startswith("--hw-queues="):
            return int(x.split("=", 1)[1])
    return 8


# HIP gives a process GPU_MAX_HW_QUEUES hardware queues (4 on the box) and maps further streams
# onto them, serialising whatever shares one.  A rank at N > 1 runs the null stream, torch's
# process-group streams, two RCCL communicators' internal streams and the engine's compute /
# comm / edge streams: with 4 queues the boundary bands can land behind the interior and the
# split step loses its overlap (the ring of one in a process holding two engines: 41-42 ms per
# 1000 turns at 4 queues, 35.4 at 8 -- profiles/r04/r04j_hw_queues.log).
_HWQ = _hw_queues(sys.argv[1:])
if _HWQ > 0:
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(_HWQ, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def _argv_int(argv, name: str, default: int) -> int:
    """--name N / --name=N from argv, read before argparse (and before torch is imported)."""
    for i, x in enumerate(argv):
        if x == name and i + 1 < len(argv):
            return int(argv[i + 1])
        if x.startswith(name + "="):
            return int(x.split("=", 1)[1])
    return default


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv, n: int, deadline_s: float, script: str | None = None) -> int:
    """`python bench.py --gpus N ...` run plainly (no torch.distributed.run, WORLD_SIZE unset): start
    the N rank processes of one node here and wait for them -- the broker bringing up its own
    server connections (broker/broker.go:191-205) instead of expecting them to exist.

    Runs before this process imports torch or loads libgolhip, so it never initialises the GPU and
    never exec()s: each rank is a fresh child (`sys.executable bench.py <same args>`) with the
    environment torch.distributed.run would give it (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free MASTER_PORT).  Rank 0's JSON line is relayed
    to stdout as this command's one line; everything else the ranks print goes to stderr.  Returns
    the exit code: 0 only if every rank exited 0; when a rank fails, the others get a grace period
    (their own collective deadlines fire first) and are then terminated; at the deadline every rank
    is killed; a rank never outlives the launcher (SIGTERM / SIGHUP are relayed, and each rank has
    a parent-death signal)."""
    import ctypes
    import signal
    import subprocess
    import threading

    script = script or os.path.abspath(__file__)
    port = _free_port()
    libc = ctypes.CDLL(None, use_errno=True)

    def die_with_launcher():  # in the child, before it starts Python: PR_SET_PDEATHSIG = 1
        libc.prctl(1, signal.SIGKILL, 0, 0, 0)

    class Stop(Exception):
        pass

    def on_signal(signum, _frame):  # SIGTERM / SIGHUP to the launcher: stop the ranks first
        raise Stop(f"signal {signum}")

    for sig in (signal.SIGTERM, signal.SIGHUP):
        signal.signal(sig, on_signal)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   GOLHIP_BENCH_LAUNCHER=str(os.getpid()))
        # a rank never outlives its launcher (killed by the driver's own deadline, say): the kernel
        # sends it SIGKILL when the launcher dies
        procs.append(subprocess.Popen([sys.executable, "-u", script, *argv], env=env, start_new_session=True,
                                      stdout=subprocess.PIPE, bufsize=0, preexec_fn=die_with_launcher))

    def relay(r, pipe):  # rank 0's JSON line -> stdout; everything else a rank prints -> stderr
        for raw in iter(pipe.readline, b""):
            to = sys.stdout if r == 0 and raw.lstrip().startswith(b"{") else sys.stderr
            to.buffer.write(raw)
            to.flush()

    relays = [threading.Thread(target=relay, args=(r, p.stdout), daemon=True) for r, p in enumerate(procs)]
    for t in relays:
        t.start()
    print(f"bench: launched {n} rank processes (pids {[p.pid for p in procs]}), master 127.0.0.1:{port}",
          file=sys.stderr, flush=True)
    t_end = time.monotonic() + deadline_s
    first_fail = None

    def stop(sig):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    try:
        while any(p.poll() is None for p in procs):
            now = time.monotonic()
            failed = [i for i, p in enumerate(procs) if p.returncode not in (None, 0)]
            if failed and first_fail is None:
                first_fail = now
                print(f"bench: rank(s) {failed} exited {[procs[i].returncode for i in failed]}; "
                      f"stopping the others in 15 s", file=sys.stderr, flush=True)
            if now > t_end or (first_fail is not None and now > first_fail + 15):
                stop(signal.SIGTERM)
                try:
                    for p in procs:
                        p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    stop(signal.SIGKILL)
                    for p in procs:
                        p.wait()
                break
            time.sleep(0.2)
    except BaseException as e:
        stop(signal.SIGTERM)
        time.sleep(2)
        stop(signal.SIGKILL)
        if isinstance(e, Stop):
            print(f"bench: launcher stopped by {e}; ranks stopped", file=sys.stderr, flush=True)
            return 143
        raise
    codes = [p.wait() for p in procs]
    for t in relays:
        t.join(timeout=5)
    if any(codes):
        print(f"bench: rank exit codes {codes}" + (" (deadline reached)" if time.monotonic() > t_end else ""),
              file=sys.stderr, flush=True)
        return 1
    return 0


# plain `python bench.py --gpus N` (N > 1) outside torch.distributed.run: become the launcher of the
# N ranks, before anything below imports torch or libgolhip
if __name__ == "__main__" and "WORLD_SIZE" not in os.environ and _argv_int(sys.argv[1:], "--gpus", 1) > 1:
    sys.exit(launch_ranks(sys.argv[1:], _argv_int(sys.argv[1:], "--gpus", 1),
                          float(_argv_int(sys.argv[1:], "--launch-deadline-s", 1500))))

import torch  # noqa: E402  (first: one HIP runtime per process, see golhip.py)
import torch.distributed as dist  # noqa: E402

import golhip  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BYTES_PER_CELL_UPDATE = 0.25  # 1 packed bit read + 1 packed bit written per cell per generation
# VALU roofline of the stencil (the bound for k >= 2): 12 wave64 VALU
# instructions per 32-cell word per generation with drifting row sums (9 v_bitop3, 2 v_alignbit,
# 1 DPP move).  Peak issue = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction
# (SIMD-32, MI355X_MICROARCH.md "Wave scheduling"): 1.2288 T wave64-instructions/s.  The half-rate
# ops (v_alignbit, DPP: 4 cycles, profiles/r01_ubench_valu2_clocked.txt) cap this mix at 24/30 of
# that peak ("mix_peak").
VALU_PER_WORD_GEN = 12
VALU_CYCLES_PER_WORD_GEN = 9 * 2 + 3 * 4
SIMDS, PEAK_CLOCK_GHZ, CYCLES_PER_WAVE_INSTR = 1024, 2.4, 2
VALU_PEAK_T = SIMDS * PEAK_CLOCK_GHZ * 1e9 / CYCLES_PER_WAVE_INSTR / 1e12
GOLDEN = ROOT / "tests" / "golden"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU). Under torch.distributed.run: must equal "
                         "WORLD_SIZE; run plainly with N > 1, bench.py starts the N rank processes "
                         "itself (launch_ranks)")
    ap.add_argument("--launch-deadline-s", type=int, default=1500,
                    help="plain --gpus N > 1 runs: the launcher kills every rank after this long")
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
    ap.add_argument("--cpu-size", type=int, default=65536, help="CPU baseline board (the bench board)")
    ap.add_argument("--cpu-turns", type=int, default=2, help="CPU baseline turns (~15 s of CPU work)")
    ap.add_argument("--cpu-threads-per-server", type=int, default=0,
                    help="goroutine-threads per reference server for the CPU baseline's bench-board "
                         "sample (0 = the best T of its sweep)")
    ap.add_argument("--no-timing", action="store_true",
                    help="no per-launch HIP events in the timed region (roofline from wall time)")
    ap.add_argument("--pmc-file", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the configs[3] leg (262144^2 board split over the N ranks)")
    ap.add_argument("--no-flips", action="store_true", help="skip the per-turn CellFlipped leg")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the configs[0]/[1]/[4] leg (512^2 PGM, 5120^2 and 4096^2 with every count)")
    ap.add_argument("--no-host", action="store_true",
                    help="skip the cfg5_host leg (configs[4] through the C++ host contract: ticker, keys)")
    ap.add_argument("--strong-size", type=int, default=262144)
    ap.add_argument("--strong-steps", type=int, default=160)
    ap.add_argument("--fixed-k", action="store_true",
                    help="every bulk launch exactly --k deep (PMC passes at one depth; the planner "
                         "otherwise runs its fastest measured depth <= k)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process (read before the HIP runtime starts; 0: "
                         "leave the environment's)")
    ap.add_argument("--pg-always", action="store_true",
                    help="rehearsal of a rank's process at N > 1 on one GPU: create the torch process "
                         "group (nccl, world 1) at N = 1 too; with GOLHIP_RING_SELF=1 the engine is the "
                         "RCCL ring of one, so the run has every stream and communicator a rank has")
    ap.add_argument("--rccl-barrier", action="store_true",
                    help="time the region between process-group (RCCL) barriers even when every rank "
                         "is on this node (default there: the shared-memory barrier)")
    ap.add_argument("--pg-timeout-s", type=float, default=120.0,
                    help="torch.distributed process-group timeout at N > 1 (well under a driver's "
                         "600 s bench limit: a stuck collective fails the run instead of hanging it)")
    ap.add_argument("--comm-timeout-ms", type=int, default=120000,
                    help="libgolhip's RCCL deadline (golhip_set_comm_timeout): a halo exchange, "
                         "all-reduce or communicator set-up that does not complete fails with "
                         "GOLHIP_ERR_RCCL naming the pending transfer")
    ap.add_argument("--preheat-ms", type=float, default=200.0,
                    help="after a cold-start pass of the same turns (reported as cold_start), "
                         "untimed K-deep launches for this long, then the board is re-initialised "
                         "from the seed and warmup + timed turns run on a chip at its loaded clock "
                         "(0 = off: the timed turns are the cold start)")
    return ap.parse_args()


class ShmBarrier:
    """The ranks' barrier when every rank runs on this node (the driver's one-node runs): one
    64-byte slot per rank in a shared-memory page, each rank writes only its own generation
    number and spins until every slot has reached it.  Same semantics as a collective barrier --
    no rank leaves before every rank has arrived -- at the cost of a few cache-line transfers
    instead of an RCCL all-reduce plus a device synchronisation (~55 us of a 20-turn region at
    world 1: profiles/r04/r04l_rank_rehearsal.log).  Set up and torn down outside the timed
    region; the file is unlinked as soon as every rank has mapped it."""

    def __init__(self, rank: int, world: int, timeout_s: float, path: str, mm, fd: int):
        import struct
        self.struct, self.rank, self.world, self.timeout_s, self.gen = struct, rank, world, timeout_s, 0
        self.path, self.mm, self.fd = path, mm, fd

    @classmethod
    def create(cls, rank: int, world: int, timeout_s: float, local_ok: bool = True) -> "ShmBarrier | None":
        """Collective (every rank calls it): every rank maps the page, or every rank gets None.  A
        rank whose own checks fail (local_ok False: not every rank on this node, no /dev/shm) or
        that cannot create or map the page votes no, and then every rank keeps the process group's
        barrier, so the ranks never disagree on which barrier they wait in."""
        import mmap
        name = [f"/dev/shm/golhip_bench_{os.getpid()}_{time.time_ns()}" if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(name, src=0)
        path, size, ok, mm, fd = name[0], 64 * world, bool(local_ok), None, -1
        if rank == 0 and ok:
            try:
                with open(path, "wb") as f:
                    f.write(b"\0" * size)
            except OSError:
                ok = False
        if world > 1:
            barrier()
        if ok:
            try:
                fd = os.open(path, os.O_RDWR)
                mm = mmap.mmap(fd, size)
            except (OSError, ValueError):
                ok = False
        oks = [ok]
        if world > 1:
            oks = [None] * world
            dist.all_gather_object(oks, ok)
        if rank == 0 and os.path.exists(path):
            os.unlink(path)  # every rank has mapped it (or given up): the page lives on in the maps
        if all(oks):
            return cls(rank, world, timeout_s, path, mm, fd)
        if mm is not None:
            mm.close()
        if fd >= 0:
            os.close(fd)
        return None

    def wait(self):
        self.gen += 1
        self.struct.pack_into("<q", self.mm, 64 * self.rank, self.gen)
        deadline = time.perf_counter() + self.timeout_s
        others = [r for r in range(self.world) if r != self.rank]
        spins = 0
        while others:
            others = [r for r in others if self.struct.unpack_from("<q", self.mm, 64 * r)[0] < self.gen]
            spins += 1
            if others and spins % 4096 == 0 and time.perf_counter() > deadline:
                raise RuntimeError(f"shared-memory barrier {self.gen}: ranks {others} did not arrive "
                                   f"within {self.timeout_s} s")

    def close(self):
        self.mm.close()
        os.close(self.fd)


SHM_BARRIER: "ShmBarrier | None" = None


def barrier():
    """The ranks' barrier: the shared-memory barrier when every rank is on this node, otherwise on
    the GPUs through the RCCL process group (a gloo TCP barrier inside a ~1 ms timed region would be
    a sizeable share of it)."""
    if SHM_BARRIER is not None:
        SHM_BARRIER.wait()
    elif dist.get_backend() == "nccl":
        dist.barrier(device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier()


RANK_TIMES: list = []  # every rank's seconds of the last timed_steps region (rank order)


def timed_steps(eng: golhip.Engine, steps: int, world: int) -> float:
    """Seconds of `steps` generations between barriers, the max over the ranks (RANK_TIMES keeps
    every rank's own)."""
    global RANK_TIMES
    if dist.is_initialized():  # N > 1, or the --pg-always rehearsal
        barrier()
    torch.cuda.synchronize()
    eng.sync()
    t0 = time.perf_counter()
    eng.step(steps)
    # torch.cuda.synchronize() is hipDeviceSynchronize: it waits for EVERY stream of the device,
    # the engine's own compute/edge/comm streams included (checked: the wall time never undercuts
    # the engine's HIP-event span, profiles/r02/r02am_timed_region_host.txt); a golhip_sync of the
    # three engine streams before it only added ~10 us of host round trips to a 20-turn region
    torch.cuda.synchronize()
    if dist.is_initialized():
        barrier()
    dt = time.perf_counter() - t0
    eng.sync()
    RANK_TIMES = [dt]
    if dist.is_initialized():
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        parts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, t)
        RANK_TIMES = [float(x.item()) for x in parts]
        dt = max(RANK_TIMES)
    return dt


def host_cpu() -> tuple[int, str]:
    """Logical CPUs of this host and its CPU model (lscpu's "Model name", from /proc/cpuinfo)."""
    model = "unknown"
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return os.cpu_count() or 0, model


def cpu_share() -> dict:
    """What this process may actually run on: its CPU affinity and the cgroup CPU quota (a GPU box
    shares the host: os.cpu_count() shows every CPU of the machine, the quota what this job gets)."""
    out = {"affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
           "cgroup_cpu_quota": None}
    try:
        quota, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            out["cgroup_cpu_quota"] = round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        pass
    return out


def cpu_baseline(size: int, turns: int, threads_per_server: int | None = None) -> dict:
    """The reference's algorithm (oracle/gol_oracle.c oracle_ref_*), timed on this host.

    The reference's cost structure: byte cells, branchy torus wrap + /255, fresh rows per turn,
    4 broker strips x T goroutine-threads (server/server.go:83-97, req.Threads per server), a
    private full-world copy per server per turn (the gob fan-out of broker/broker.go:51,64; each
    server copies its own, concurrently) and the controller's per-turn alive scan
    (gol/distributor.go:186).  The workers are a persistent pool handed each turn through
    barriers -- the goroutine analogue (round 3 created 4T OS threads per turn).  The RPC
    transport itself (gob encode/TCP) is not timed.

    Legs (sample sizes chosen to keep the whole leg ~30 s):
      sweep   : T = 1, 2, 4, 8, 16 (the reference's own thread matrix, gol_test.go:29), T = the
                cgroup CPU quota / 4 and T = every host CPU / 4: configs[0] in full (512^2 x 100,
                bit-exact vs check/images/512x512x100.pgm) and the first 20 turns of configs[1]
                (5120^2 seed 2, every count vs the golden CSV);
      value   : `turns` turns of the bench board itself (65536^2 random p=0.5 seed 3) at the best T
                of the configs[1] prefix (or threads_per_server when given);
      cfg5    : the first 100 turns of configs[4] (4096^2 gun + R-pentomino), every count checked;
      cfg4    : configs[3] (262144^2) is NOT run: its byte board needs 64 GiB per copy (world, next,
                4 fan-out copies: 384 GiB > the job's host-memory cap); one turn is extrapolated
                from the bench board's per-cell rate (labelled)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np

    import oracle

    nproc, model = host_cpu()
    share = cpu_share()
    quota = share.get("cgroup_cpu_quota")
    t_quota = max(1, round(quota / 4)) if quota else None
    t_cores = max(1, -(-nproc // 4))
    ref = GOLDEN / "reference"
    gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
    _, _, b512 = oracle.read_pgm(ref / "images" / "512x512.pgm")
    want512 = (ref / "check" / "images" / "512x512x100.pgm").read_bytes()
    lines = (GOLDEN / gold["cfg2"]["counts_csv"]).read_text().split()[1:21]
    want2 = [int(ln.split(",")[1]) for ln in lines]
    b2 = oracle.unpack(oracle.init_random(5120, 5120, seed=2), 5120)

    sweep = {}
    for T in sorted({1, 2, 4, 8, 16, t_cores} | ({t_quota} if t_quota else set())):
        t0 = time.perf_counter()
        out512, _ = oracle.ref_run(b512, 100, threads=T, servers=4, fanout_copy=True)
        dt512 = time.perf_counter() - t0
        t0 = time.perf_counter()
        _, c2 = oracle.ref_run(b2, 20, threads=T, servers=4, fanout_copy=True)
        dt2 = time.perf_counter() - t0
        labels = [x for x, v in (("quota", t_quota), ("host_cores", t_cores)) if v == T]
        sweep[str(T)] = {"os_threads": 4 * T, "label": labels or None,
                         "cfg1_512x100_s": round(dt512, 4),
                         "cfg1_gcups": round(512 * 512 * 100 / dt512 / 1e9, 4),
                         "cfg1_bit_exact": oracle.pgm_bytes(out512) == want512,
                         "cfg2_first20_s": round(dt2, 4),
                         "cfg2_gcups": round(5120 * 5120 * 20 / dt2 / 1e9, 4),
                         "cfg2_counts_match": [int(x) for x in c2] == want2}
    del b2
    # the job's CPUs: its affinity set and its cgroup quota, whichever is smaller (the GPU box
    # shares its host; os.cpu_count() shows the whole machine)
    effective = min(x for x in (share.get("affinity_cpus") or nproc, quota or nproc, nproc) if x)
    effective = max(1, int(effective))
    best_t = max(sweep, key=lambda t: sweep[t]["cfg2_gcups"])
    # the value's T: the fastest of the sweep among those whose 4T threads fit the job's CPUs
    # (oversubscribing the quota measures the scheduler, and would make `cores` exceed the CPUs)
    fitting = [t for t in sweep if 4 * int(t) <= effective]
    best_fit = max(fitting, key=lambda t: sweep[t]["cfg2_gcups"]) if fitting else "1"
    T = threads_per_server or int(best_fit)

    board = oracle.unpack(oracle.init_random(size, size, seed=3), size)
    t0 = time.perf_counter()
    oracle.ref_run(board, turns, threads=T, servers=4, fanout_copy=True)
    dt = time.perf_counter() - t0
    del board
    cups = size * size * turns / dt

    # configs[4]: the first 100 turns, every count vs the golden npz
    b5 = np.zeros((4096, 4096), dtype=np.uint8)
    golhip.place(b5, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
    golhip.place(b5, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
    deltas = np.load(GOLDEN / gold["cfg5"]["counts_1e6_npz"])["deltas"][:100]
    exp5 = (int((b5 == 255).sum()) + np.cumsum(deltas.astype(np.int64))).tolist()
    t0 = time.perf_counter()
    _, c5 = oracle.ref_run(b5, 100, threads=T, servers=4, fanout_copy=True)
    dt5 = time.perf_counter() - t0

    n4 = 262144
    return {
        "value": round(cups / 1e9, 4),
        "unit": "GCUPS",
        "cores": 4 * T,  # = threads used: 4 servers x T goroutine-threads, <= effective_cpus
        "threads": 4 * T,
        "threads_per_server": T,
        "effective_cpus": effective,
        "value_per_effective_cpu": round(cups / 1e9 / min(4 * T, effective), 4),
        "host_cores": nproc,
        **share,
        "cpu_model": model,
        "fanout_copy": True,
        "workers": "persistent pool (goroutine analogue): 4 servers x T threads created once per run",
        "kind": "port",
        "sample": (f"{size}x{size} random p=0.5 seed 3 (the bench board), {turns} turns of the "
                   f"reference algorithm at T = {T} goroutine-threads per server (the best T of the "
                   f"sweep on configs[1]'s first 20 turns with 4T <= the job's {effective} CPUs): "
                   f"byte cells, branchy torus wrap + /255, "
                   f"fresh rows per turn, 4 broker strips x {T} = {4 * T} worker threads (one pool "
                   f"per run), full-world copy per server per turn, per-turn alive scan; gob/TCP "
                   f"transport not timed; {dt:.1f} s"),
        "t_sweep": sweep,
        "best_threads_per_server": int(best_t),
        "best_threads_per_server_within_cpus": int(best_fit),
        "cfg5_4096_first100": {"s": round(dt5, 4), "gcups": round(4096 * 4096 * 100 / dt5 / 1e9, 4),
                               "us_per_turn": round(dt5 / 100 * 1e6, 1),
                               "counts_match_golden": [int(x) for x in c5] == exp5,
                               "sample": "first 100 of configs[4]'s 1e6 turns (labelled prefix)"},
        "cfg4_262144_extrapolated": {
            "s_per_turn": round(n4 * n4 / cups, 2), "gcups": round(cups / 1e9, 4),
            "note": ("not run: the byte board needs 64 GiB per copy (world, next and 4 fan-out "
                     "copies = 384 GiB, over the job's host-memory cap); extrapolated from the "
                     f"{size}^2 sample's per-cell rate (labelled extrapolation)")},
    }


DIGEST_CHUNK_ROWS = 4096  # = oracle.DIGEST_CHUNK_ROWS (tests/test_tools.py checks both)


def chunk_digests(words) -> list[bytes]:
    """SHA-256 of each 4096-row chunk of packed little-endian uint64 rows (a strip's share of the
    board digest; the oracle's definition, restated here so the bench's GPU path imports no oracle)."""
    import numpy as np

    w = np.ascontiguousarray(words, dtype="<u8")
    return [hashlib.sha256(w[y:y + DIGEST_CHUNK_ROWS].tobytes()).digest()
            for y in range(0, w.shape[0], DIGEST_CHUNK_ROWS)]


def strip_words(eng: golhip.Engine):
    """This rank's strip as packed uint64 rows (a host copy, ~15 ms for 512 MiB), or None when it
    cannot enter the board digest (width not a multiple of 64, strip not on a chunk boundary)."""
    info = eng.info
    if info.width % 64 == 0 and info.y0 % DIGEST_CHUNK_ROWS == 0:
        return eng.store_words()
    return None


def board_digest(words, world: int) -> str | None:
    """SHA-256 of the chunk digests of the whole board (every rank's strip_words, in row order), or
    None when a strip could not be hashed.  Collective at world > 1."""
    mine = chunk_digests(words) if words is not None else None
    if world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, mine)
    else:
        parts = [mine]
    if any(p is None for p in parts):
        return None
    return hashlib.sha256(b"".join(c for p in parts for c in p)).hexdigest()


def golden_digest(width: int, height: int, seed: int, turn: int) -> str | None:
    """The oracle's board digest of the width x height random board (p = 0.5, `seed`) after `turn`
    turns, if tests/golden/synthetic_golden.json pins it (scripts/make_golden.py digests)."""
    try:
        gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
    except OSError:
        return None
    for entry in gold.values():
        if (entry.get("width"), entry.get("height"), entry.get("seed")) == (width, height, seed):
            d = entry.get("board_digest", {}).get(str(turn))
            if d:
                return d
    return None


def golden_count(width: int, height: int, seed: int, turn: int) -> int | None:
    """The oracle's alive count of the width x height random board (p = 0.5, `seed`) after `turn`
    turns, if tests/golden/synthetic_golden.json registers a per-turn count CSV for that board
    (scripts/make_golden.py: configs[1..3], and the weak-scaling boards 65536 x 65536*N for
    N = 2, 4, 8 that bench --gpus N runs)."""
    if turn < 1:
        return None
    try:
        gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
    except OSError:
        return None
    for entry in gold.values():
        if (entry.get("width"), entry.get("height"), entry.get("seed")) != (width, height, seed):
            continue
        path = GOLDEN / entry.get("counts_csv", "")
        if not entry.get("counts_csv") or not path.exists():
            continue
        for line in path.read_text().splitlines()[1:]:
            t, c = line.split(",")
            if int(t) == turn:
                return int(c)
    return None


def read_pgm_body(path: Path) -> tuple[int, int, bytes]:
    """P5 header "P5\\n<w> <h>\\n255\\n" (gol/io.go:52-59) -> (width, height, pixel bytes)."""
    raw = path.read_bytes()
    fields, pos = [], 0
    while len(fields) < 4:
        while raw[pos:pos + 1].isspace():
            pos += 1
        end = pos
        while not raw[end:end + 1].isspace():
            end += 1
        fields.append(raw[pos:end])
        pos = end
    pos += 1  # the single whitespace byte after maxval
    w, h = int(fields[1]), int(fields[2])
    return w, h, raw[pos:pos + w * h]


def configs_leg() -> dict:
    """BASELINE.json configs[0], [1] and [4] on this GPU through the production path (automatic
    kernel choice, default planner), each checked against the reference fixture / oracle goldens:
      cfg1: images/512x512.pgm, 100 turns with every count -> check/images/512x512x100.pgm
            byte-exact and all 100 counts of check/alive/512x512.csv;
      cfg2: 5120^2 random seed 2, 10 000 turns with every count (tests/golden cfg2 CSV);
      cfg5: 4096^2 glider gun + R-pentomino, 1e6 turns with every count (tests/golden cfg5 npz).
    Wall time of the golhip_step call(s) incl. the per-turn count copy to the host."""
    import numpy as np

    gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
    ref = GOLDEN / "reference"
    res = {}
    # configs[0]
    w, h, px = read_pgm_body(ref / "images" / "512x512.pgm")
    board = np.frombuffer(px, dtype=np.uint8).reshape(h, w)
    _, _, want = read_pgm_body(ref / "check" / "images" / "512x512x100.pgm")
    csv = [ln.split(",") for ln in (ref / "check" / "alive" / "512x512.csv").read_text().split()]
    want_counts = {int(t): int(c) for t, c in (r for r in csv if r[0].strip().isdigit())}
    def cfg1_runs(board_kernel: int):  # -1: the automatic choice, 1: the whole-board kernel forced
        with golhip.Engine(w, h, k=16) as e:
            e.set_board_kernel(board_kernel)
            kind = e.launch_kind(16, counts=True)
            e.load(board)
            e.step(100, counts=True)  # warm (graphs, code paths)
            runs = []
            for _ in range(5):
                e.load(board)
                e.sync()
                t = time.perf_counter()
                c = e.step(100, counts=True)
                e.sync()
                runs.append(time.perf_counter() - t)
            out = e.store()
        ok = (out.tobytes() == want and [int(x) for x in c] == [want_counts[t] for t in range(1, 101)])
        return float(np.median(runs)), ok, f"{kind[0]}{kind[1] or ''}"

    dt, ok, kind = cfg1_runs(-1)
    dt_b, ok_b, kind_b = cfg1_runs(1)
    res["cfg1_512x100"] = {"us_per_turn": round(dt / 100 * 1e6, 3), "median_of": 5, "kernel": kind,
                           "bit_exact_vs_reference_fixture": bool(ok and ok_b),
                           # A/B: the single-workgroup whole-board kernel forced (automatic only up to
                           # 256 rows: one CU's VALU work per generation grows with the board)
                           "whole_board_kernel_forced": {"kernel": kind_b,
                                                         "us_per_turn": round(dt_b / 100 * 1e6, 3)}}
    # configs[1]
    lines = (GOLDEN / gold["cfg2"]["counts_csv"]).read_text().split()[1:]
    exp2 = np.array([int(ln.split(",")[1]) for ln in lines], dtype=np.uint64)
    def cfg2_runs(activity: int):  # -1: automatic (off: one slab per CU), 1: skipping forced
        with golhip.Engine(5120, 5120, k=16) as e:
            e.set_activity(activity)
            kind = e.launch_kind(16, counts=True)
            runs, ok = [], True
            for _ in range(5):
                e.init_random(2)
                e.sync()
                t = time.perf_counter()
                c = e.step(10000, counts=True)
                runs.append(time.perf_counter() - t)
                ok = ok and bool(np.array_equal(c.astype(np.uint64), exp2))
            stats = e.activity_stats()
        runs_sorted = sorted(runs[1:])  # the first run captures the count graphs
        return runs, runs_sorted, ok, kind, stats

    runs, runs_sorted, ok, kind, stats = cfg2_runs(-1)
    runs_d, runs_dsorted, ok_d, _, stats_d = cfg2_runs(1)

    def persistent_runs(setup, turns, exp, nruns, handoff=golhip.HANDOFF_FENCED):
        """golhip_step_persistent (opt-in) A/B, best of nruns with every count checked; a refused or
        failed call is recorded as {'skipped': reason} -- it never fails the production leg."""
        try:
            with golhip.Engine(setup[0], setup[0], k=16) as e:
                e.set_persistent_handoff(handoff)
                setup[1](e)
                e.step_persistent(4096)  # warm
                ts, okp = [], True
                for _ in range(nruns):
                    setup[1](e)
                    e.sync()
                    t = time.perf_counter()
                    c = e.step_persistent(turns)
                    ts.append(time.perf_counter() - t)
                    okp = okp and bool(np.array_equal(c.astype(np.uint64), exp))
        except golhip.GolHipError as err:
            return {"skipped": str(err)}
        return {"us_per_turn": round(min(ts) / turns * 1e6, 3), "best_of": nruns, "counts_match": okp}

    pers2 = persistent_runs((5120, lambda e: e.init_random(2)), 10000, exp2, 3)
    pers2s = persistent_runs((5120, lambda e: e.init_random(2)), 10000, exp2, 3, golhip.HANDOFF_SC1)
    dt = runs_sorted[len(runs_sorted) // 2]
    dt_d = runs_dsorted[len(runs_dsorted) // 2]
    res["cfg2_5120x10000"] = {"us_per_turn": round(dt / 10000 * 1e6, 3),
                              "best_us_per_turn": round(runs_sorted[0] / 10000 * 1e6, 3),
                              "runs_s": [round(r, 4) for r in runs],
                              "gcups": round(5120 * 5120 * 10000 / dt / 1e9, 1),
                              "counts_match_all_10000": bool(ok and ok_d), "kernel": f"{kind[0]}{kind[1] or ''}",
                              "stable_slab_skipping": {"slabs_computed": stats[0], "slabs_skipped": stats[1]},
                              "skipping_forced": {"us_per_turn": round(dt_d / 10000 * 1e6, 3),
                                                  "gcups": round(5120 * 5120 * 10000 / dt_d / 1e9, 1),
                                                  "slabs_computed": stats_d[0], "slabs_skipped": stats_d[1]},
                              # golhip_step_persistent: one launch per count window (opt-in: needs
                              # every slab resident), best of 3, every count checked; default
                              # release/acquire hand-off and the sc1-only measured form
                              "persistent_opt_in": pers2, "persistent_opt_in_sc1": pers2s}
    # configs[4]
    b = np.zeros((4096, 4096), dtype=np.uint8)
    golhip.place(b, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
    golhip.place(b, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
    deltas = np.load(GOLDEN / gold["cfg5"]["counts_1e6_npz"])["deltas"]
    exp5 = (int((b == 255).sum()) + np.cumsum(deltas.astype(np.int64))).astype(np.uint64)
    def cfg5_run(activity: int):  # -1: automatic (off: one slab per CU), 1: skipping forced
        with golhip.Engine(4096, 4096, k=16) as e:
            e.set_activity(activity)
            kind = e.launch_kind(16, counts=True)
            e.load(b)
            e.step(4096, counts=True)  # capture the count graphs
            e.load(b)
            e.sync()
            s0 = e.activity_stats()
            t = time.perf_counter()
            c = e.step(1000000, counts=True)
            dt = time.perf_counter() - t
            s1 = e.activity_stats()
        return dt, bool(np.array_equal(c.astype(np.uint64), exp5)), kind, (s1[0] - s0[0], s1[1] - s0[1])

    dt, ok5, kind, stats = cfg5_run(-1)
    dt_d, ok5_d, _, stats_d = cfg5_run(1)
    pers5 = persistent_runs((4096, lambda e: e.load(b)), 1000000, exp5, 1)
    pers5s = persistent_runs((4096, lambda e: e.load(b)), 1000000, exp5, 1, golhip.HANDOFF_SC1)
    res["cfg5_4096x1e6"] = {"us_per_turn": round(dt, 3), "gcups": round(4096 * 4096 * 1e6 / dt / 1e9, 1),
                            "counts_match_all_1e6": bool(ok5 and ok5_d),
                            "kernel": f"{kind[0]}{kind[1] or ''}",
                            "stable_slab_skipping": {"slabs_computed": stats[0], "slabs_skipped": stats[1]},
                            # A/B: skipping forced on (70 % of the slabs skip, yet a launch lasts as
                            # long as its slowest computed slab: 237 slabs, one per CU)
                            "skipping_forced": {"us_per_turn": round(dt_d, 3),
                                                "gcups": round(4096 * 4096 * 1e6 / dt_d / 1e9, 1),
                                                "slabs_computed": stats_d[0], "slabs_skipped": stats_d[1]},
                            "persistent_opt_in": pers5, "persistent_opt_in_sc1": pers5s}
    # the production (automatic) path decides ok; the opt-in persistent A/B reports its own match
    res["ok"] = bool(res["cfg1_512x100"]["bit_exact_vs_reference_fixture"]
                     and res["cfg2_5120x10000"]["counts_match_all_10000"]
                     and res["cfg5_4096x1e6"]["counts_match_all_1e6"])
    res["persistent_opt_in_ok"] = all(p.get("counts_match", True) for p in (pers2, pers5, pers2s, pers5s))
    return res


def cfg5_host_leg(turns: int = 1000000) -> dict:
    """configs[4]'s own metric ("ticker latency; throughput while
    servicing p/s"): the C++ host contract (gol::Run, distributed-gol_amd/host) driven by its
    consumer, lib/host_bench -- per-turn TurnComplete events, the AliveCellsCount ticker and keys
    pressed at set times (gol/distributor.go:105-151,168-191), on the 4096^2 gun + R-pentomino
    board for 1e6 turns.  Every tick's count, the final count and the 's' snapshot file are checked
    against the golden per-turn counts (tests/golden cfg5 npz).  Runs:
      reference : the reference's 2 s ticker, keys p (pause) @0.5 s, s (snapshot) @0.8 s, p @2.3 s
                  (the 2 s tick falls in the pause: it must report the paused turn's count);
      ticks     : a 20 ms ticker (many ticks: the tick-latency distribution), no keys;
      unpipelined: the 2 s ticker with no delivery thread (pipeline depth 0): device work and event
                  delivery alternate, as before round 6 -- the A/B of the pipelined turn loop."""
    import subprocess
    import tempfile

    import numpy as np

    exe = ROOT / "distributed-gol_amd" / "lib" / "host_bench"
    if not exe.exists():
        return {"skipped": f"{exe} not built"}
    if "ROCP_TOOL_LIBRARIES" in os.environ:
        # under rocprofv3 the child inherits the tool, and the tool's kernel tracing segfaults
        # inside hipGraphLaunch on the 1e6-turn run's large count graphs (profiles/r06/r06n_*,
        # r06r_*: the same crash with host_bench run directly under the tool; 20 000 turns, whose
        # graphs stay small, trace fine: r06o_*) -- the profiled run is for the kernels, the leg
        # runs in unprofiled bench runs
        return {"skipped": "running under rocprofv3 (the host-contract leg runs in unprofiled bench runs)"}
    gold = json.loads((GOLDEN / "synthetic_golden.json").read_text())
    b = np.zeros((4096, 4096), dtype=np.uint8)
    golhip.place(b, golhip.parse_rle((GOLDEN / "gosper_gun.rle").read_text()), 64, 64)
    golhip.place(b, golhip.parse_rle((GOLDEN / "r_pentomino.rle").read_text()), 2048, 2048)
    deltas = np.load(GOLDEN / gold["cfg5"]["counts_1e6_npz"])["deltas"][:turns]
    counts = np.concatenate([[int((b == 255).sum())], int((b == 255).sum()) + np.cumsum(deltas.astype(np.int64))])
    res = {}
    with tempfile.TemporaryDirectory(prefix="golhip_cfg5_") as d:
        dp = Path(d)
        (dp / "images").mkdir()
        (dp / "out").mkdir()
        (dp / "images" / "4096x4096.pgm").write_bytes(b"P5\n4096 4096\n255\n" + b.tobytes())
        counts.astype("<u4").tofile(dp / "expected.u32")
        runs = {"reference": ["-ticker_ms", "2000", "-keys", "p@0.5,s@0.8,p@2.3", "-depth", "2"],
                "ticks": ["-ticker_ms", "20", "-depth", "2"],
                "unpipelined": ["-ticker_ms", "2000", "-depth", "0"]}
        for name, extra in runs.items():
            cmd = [str(exe), "-w", "4096", "-h", "4096", "-turns", str(turns), "-images", str(dp / "images"),
                   "-out", str(dp / "out"), "-expected", str(dp / "expected.u32"), *extra]
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                res[name] = {"failed": p.returncode, "stderr": p.stderr[-2000:]}
                continue
            res[name] = json.loads(p.stdout.strip().splitlines()[-1])
    ok = True
    for name, r in res.items():
        if "failed" in r:
            ok = False
            continue
        ok = ok and r["turn_complete"]["in_order"] and r["final"]["match"] and (
            r["ticks"]["n"] == 0 or r["ticks"]["counts_match"])
        if r["snapshot"]["match"] is not None:
            ok = ok and r["snapshot"]["match"]
    res["ok"] = bool(ok)
    return res


def library_identity() -> dict:
    """The loaded libgolhip.so: path relative to the repo, golhip_version(), first 16 hex digits of
    the file's SHA-256."""
    p = Path(os.environ.get("GOLHIP_LIB", str(golhip.LIB_PATH))).resolve()
    try:
        rel = str(p.relative_to(ROOT))
    except ValueError:
        rel = str(p)
    try:
        return {"path": rel, "abi_version": int(golhip.load_library().golhip_version()),
                "sha256_16": hashlib.sha256(p.read_bytes()).hexdigest()[:16]}
    except (OSError, golhip.GolHipError, AttributeError) as e:  # a stand-in engine (CPU tests)
        return {"path": rel, "error": str(e)}


ENGINES: list = []  # the engines this process created (their last C ABI call names a failure)


def main():
    global SHM_BARRIER
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:  # bench.main() called in-process; `python bench.py` launches the ranks
            raise SystemExit("--gpus N > 1: run `python bench.py --gpus N` (it starts the N ranks) or "
                             "launch it with torch.distributed.run")
    # test hook (tests/test_gpu_rank_host.py): GOLHIP_HOST_COMM=1 runs the rank engines with the gloo
    # host transport instead of RCCL, so N ranks can share the one GPU of a test box (RCCL refuses
    # two ranks on one device); the engine, its launch plan and the timed region are unchanged
    host_comm = os.environ.get("GOLHIP_HOST_COMM", "0") == "1" and world > 1
    # test hook (tests/test_gpu_rccl_ranks.py): GOLHIP_RCCL_SHARED_GPU=1 runs N REAL RCCL ranks on
    # the one GPU of a test box: a distinct NCCL_HOSTID per rank makes RCCL treat the ranks as
    # separate hosts and connect them through its network transport (loopback) instead of refusing
    # "Duplicate GPU"; the engine, the process group, the timed region are the N > 1 code
    rccl_shared = os.environ.get("GOLHIP_RCCL_SHARED_GPU", "0") == "1" and world > 1 and not host_comm
    if rccl_shared:
        os.environ["NCCL_HOSTID"] = f"golhip-bench-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    if host_comm or rccl_shared:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1 or a.pg_always:
        # one process per GPU: the bench's own collectives (barriers, the max-over-ranks time, the
        # RCCL id broadcast) over RCCL; gloo where RCCL cannot run (the host-transport hook's
        # ranks share one GPU; CPU-only test runs)
        backend = "nccl" if torch.cuda.is_available() and not host_comm else "gloo"
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=a.pg_timeout_s))
        if world == 1:
            obj = [None]
            dist.broadcast_object_list(obj, src=0)  # the collective N > 1 runs before the engine
        # every rank on this node (torch.distributed.run's LOCAL_WORLD_SIZE): the timed region's
        # barriers go through shared memory (--rccl-barrier, the same flag on every rank, keeps the
        # process group's); every rank joins the set-up's vote whatever its local checks say
        if not a.rccl_barrier:
            local_ok = (int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world
                        and os.path.isdir("/dev/shm"))
            SHM_BARRIER = ShmBarrier.create(rank, world, a.pg_timeout_s, local_ok=local_ok)
    golhip.set_default_comm_timeout(a.comm_timeout_ms)

    width = a.size
    height = a.height or a.size * world
    nccl_id = None
    if world > 1 and not host_comm:
        obj = [golhip.nccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        nccl_id = obj[0]
    eng = golhip.Engine(width, height, k=a.k, rank=rank, world_size=world, device=local,
                        nccl_id=nccl_id, host_comm=golhip.GlooHostComm() if host_comm else None)
    ENGINES.append(eng)
    if a.band_rows:
        eng.set_band_rows(a.band_rows)
    if a.fixed_k:
        eng.set_fixed_k(True)
    eng.init_random(a.seed)
    local_rows = eng.info.rows
    cold = None
    if a.preheat_ms > 0:
        # cold start: the same warmup + timed turns on a chip that was idle until now (its clock
        # ramps up over the first tens of ms of load: profiles/r02/r02r_preheat.txt)
        eng.step(a.warmup)
        eng.sync()
        dtc = timed_steps(eng, a.steps, world)
        alive_c = eng.alive_count()  # collective
        cold = {"value": round(width * height * a.steps / dtc / 1e9, 2),
                "preheat_turns": None,
                "ms_per_step": round(dtc * 1e3 / a.steps, 4), "alive_after": int(alive_c)}
        # pre-heat: untimed K-deep launches for about preheat_ms, then the board starts from the
        # seed again, so warmup + the timed turns below are exactly those of a fresh run.  The
        # turn count comes from the cold pass's max-over-ranks time, so every rank runs the same
        # number of steps (each step call exchanges halos over RCCL when N > 1)
        pre_turns = max(a.k, int(a.preheat_ms / (dtc * 1e3 / a.steps)))
        pre_turns = -(-pre_turns // a.k) * a.k
        eng.step(pre_turns)
        eng.sync()
        cold["preheat_turns"] = pre_turns
        eng.init_random(a.seed)
    local_cells = local_rows * width

    eng.step(a.warmup)
    eng.sync()
    # the launch depths the engine runs for the timed region (golhip_launch_plan: the same planner
    # golhip_step uses): k is the maximum depth, the bulk runs the fastest measured depth <= k
    plan = golhip.launch_plan(width, height, a.k, a.steps, strips=world)
    depth_count = {}
    for d in plan:
        depth_count[d] = depth_count.get(d, 0) + 1
    dominant_k = max(depth_count, key=lambda d: (depth_count[d] * abs(d), d))

    # timed region: exactly a.steps generations, NOT instrumented -- the per-launch HIP event pairs
    # the roofline needs cost the region ~45 us per two launches (event records between the
    # kernels; scripts/host_submit.py, profiles/r03/r03af_host_submit.log), so `value` is measured
    # without them and the launch durations come from a second, identical pass below
    eng.timing(False)
    dt = timed_steps(eng, a.steps, world)
    timed_rank_s = list(RANK_TIMES)
    # regression canary: alive cells after exactly warmup + steps generations (deterministic for
    # the seed; compare across kernel versions)
    alive_timed = eng.alive_count()
    # the whole board after the timed pass, bit for bit: every rank copies its strip to the host
    # now (outside the timed region) and hashes it in 4096-row chunks after the instrumented pass
    # (a second of host hashing here would let the chip's clock drop before that pass)
    timed_words = strip_words(eng)
    instrumented = None
    if a.no_timing:
        launches = -(-a.steps // a.k)
        kern_ms, gens = dt * 1e3, a.steps
    else:
        # roofline pass: the same warmup + timed turns from the seed again, with per-launch HIP
        # events on the compute stream (every rank: the steps exchange halos when N > 1); a short
        # re-heat first (the host copy above idled the GPU), the same turn count on every rank
        if cold is not None:
            eng.step(max(a.k, cold["preheat_turns"] // 4 // a.k * a.k))
        eng.init_random(a.seed)
        eng.step(a.warmup)
        eng.sync()
        eng.timing(True)
        dti = timed_steps(eng, a.steps, world)
        inst_rank_s = list(RANK_TIMES)
        kern_ms, launches, gens = eng.kernel_time()
        edge_ms, edge_blocks = eng.edge_wait()
        eng.timing(False)
        alive_i = eng.alive_count()
        if alive_i != alive_timed:
            raise SystemExit(f"instrumented pass ended at {alive_i} alive cells, the timed one at {alive_timed}")
        if kern_ms > dti * 1e3 * 1.001:
            raise SystemExit(f"timed region {dti * 1e3:.3f} ms shorter than the engine's event span "
                             f"{kern_ms:.3f} ms: the end-of-region synchronisation missed engine work")
        instrumented = {"ms_per_step": round(dti * 1e3 / a.steps, 4),
                        "kernel_ms": round(kern_ms, 4), "launches": launches,
                        "note": "the same warmup + timed turns from the seed, with per-launch HIP "
                                "events (roofline.avg_launch_us); value is the uninstrumented pass"}
    digest = board_digest(timed_words, world)
    del timed_words
    # N > 1: what each rank's timed region was made of, so a scaling line explains its own
    # efficiency -- the rank's wall time in the timed pass, and in the instrumented pass its
    # HIP-event kernel span on the compute stream and the time that stream waited for the boundary
    # bands (which wait for the halo exchange) after each block's interior
    per_rank = None
    if dist.is_initialized():
        mine = {"rank": rank, "y0": int(eng.info.y0), "rows": int(local_rows),
                "timed_ms": round(timed_rank_s[rank] * 1e3, 4)}
        if not a.no_timing:
            mine.update({"instrumented_ms": round(inst_rank_s[rank] * 1e3, 4),
                         "kernel_span_ms": round(kern_ms, 4), "launches": launches,
                         "edge_wait_ms": round(edge_ms, 4), "split_blocks": edge_blocks})
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    total_updates = width * height * a.steps
    gcups = total_updates / dt / 1e9
    ms_per_step = dt * 1e3 / a.steps

    # roofline of the timed kernel (gol_stencil<k>, or gol_step1 at k = 1) on this rank, from the
    # HIP events around the timed launches on the engine's compute stream
    avg_launch_ms = kern_ms / max(launches, 1)
    gens_per_launch = gens / max(launches, 1)
    alg_bytes_per_launch = BYTES_PER_CELL_UPDATE * local_cells * gens_per_launch
    hbm_achieved = alg_bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9
    # algorithmic wave64 VALU instructions per launch: 12 per 32-cell word per generation over the
    # cells the launch updates (no band-halo trapezoid, pipeline fill, loop or store work)
    words_per_launch = local_cells / 32 * gens_per_launch
    valu_alg = words_per_launch / 64 * VALU_PER_WORD_GEN
    valu_achieved = valu_alg / (avg_launch_ms * 1e-3) / 1e12
    pmc_entry, pmc = {}, {}
    try:
        pmc = json.loads(Path(a.pmc_file).read_text())
        pmc_entry = pmc.get(f"{width}x{eng.info.rows}_k{dominant_k}", {})
    except Exception:
        pass
    # PMC-issued VALU instructions of the whole timed region, when every depth it ran has a PMC
    # entry for this board (profiles/pmc_traffic.json): sum over launches / the region's kernel time
    issued_all = None
    per_depth = [pmc.get(f"{width}x{eng.info.rows}_k{d}", {}).get("valu_instr_per_launch")
                 for d in depth_count]
    if depth_count and all(per_depth) and kern_ms > 0 and not a.no_timing:
        issued_all = sum(v * depth_count[d] for v, d in zip(per_depth, depth_count))
    traffic = pmc_entry.get("hbm_bytes_per_launch")
    uniform = len(depth_count) == 1  # every timed launch ran the same depth
    issued = pmc_entry.get("valu_instr_per_launch")
    # the launches the average covers: every depth of the timed region (e.g. 12 + 8 for 20 turns)
    kernel_name = " + ".join("gol_step1" if d == 1 else f"gol_stencil<{d}>"
                             for d in sorted(depth_count, key=lambda d: (-depth_count[d] * abs(d), d)))
    if dominant_k == 1:
        roof = {"bound": "hbm", "achieved": round(hbm_achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(hbm_achieved / HBM_PEAK_GBS, 4), "traffic": traffic}
    else:
        roof = {"bound": "valu", "achieved": round(valu_achieved, 4), "peak": round(VALU_PEAK_T, 4),
                "unit": "T wave64-VALU-instr/s", "frac": round(valu_achieved / VALU_PEAK_T, 4),
                "traffic": traffic,
                "mix": "12 per 32-cell word per generation: 9 v_bitop3 (2 cyc) + 2 v_alignbit "
                       "+ 1 DPP move (4 cyc): mix_peak = 24/30 of peak",
                "mix_peak": round(VALU_PEAK_T * 24 / VALU_CYCLES_PER_WORD_GEN, 4)}
        if issued:
            # PMC SQ_INSTS_VALU of one gol_stencil<dominant_k> launch (profiles/pmc_traffic.json);
            # the issue RATE needs every timed launch to be that kernel
            roof["issued_per_launch_pmc"] = issued
            if uniform:
                roof["issued_pmc"] = round(issued / (avg_launch_ms * 1e-3) / 1e12, 4)
                roof["issued_frac"] = round(issued / (avg_launch_ms * 1e-3) / 1e12 / VALU_PEAK_T, 4)
        if issued_all and not uniform:
            # mixed depths (e.g. 82 x K=12 + 1 x K=16): every launch's PMC count over the region
            roof["issued_pmc"] = round(issued_all / (kern_ms * 1e-3) / 1e12, 4)
            roof["issued_frac"] = round(issued_all / (kern_ms * 1e-3) / 1e12 / VALU_PEAK_T, 4)
        if pmc_entry.get("clock_ghz"):
            roof["clock_ghz_pmc"] = pmc_entry["clock_ghz"]
    roof.update({"kernel": kernel_name, "avg_launch_us": round(avg_launch_ms * 1e3, 2),
                 "launches": launches, "gens_per_launch": round(gens_per_launch, 3),
                 "launch_depths": {str(d): c for d, c in sorted(depth_count.items())}})
    hbm_roof = {"achieved": round(hbm_achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "algorithmic_over_peak": round(hbm_achieved / HBM_PEAK_GBS, 4),
                "measured_traffic_per_launch": traffic,
                "note": "0.25 B per cell-update; temporal blocking moves the board once per "
                        "launch, so this exceeds 1 for k > 1 and is not the binding bound"}
    # parity: the canary against the oracle's golden count of this board (every registered board:
    # configs[2] at N == 1, the weak-scaling boards 65536 x 65536*N at N = 2, 4, 8)
    parity = None
    if a.seed in (2, 3, 4):
        exp = golden_count(width, height, a.seed, a.warmup + a.steps)
        if exp is not None:
            parity = {"turn": a.warmup + a.steps, "alive": int(alive_timed), "golden": exp,
                      "ok": int(alive_timed) == exp}
            if cold is not None:
                parity["cold_start_ok"] = cold["alive_after"] == exp
                parity["ok"] = parity["ok"] and parity["cold_start_ok"]
    exp_digest = golden_digest(width, height, a.seed, a.warmup + a.steps)
    if exp_digest is not None:
        parity = parity or {"turn": a.warmup + a.steps, "ok": True}
        parity["digest"] = digest
        parity["golden_digest"] = exp_digest
        parity["digest_ok"] = digest == exp_digest
        parity["ok"] = parity["ok"] and parity["digest_ok"]

    sweep = None
    k1_launch_us = None
    if world == 1 and not a.no_sweep:
        sweep = {}
        eng.set_fixed_k(True)  # exactly kk deep per launch
        for kk in (1, 2, 4, 8, 10, 12, 14, 16, 32):
            eng.set_k(kk)
            # the first ~250 one-generation launches of a process run ~10 % slower (measured,
            # scripts/diag_k1.py), so k = 1 gets a longer untimed warmup
            eng.step(256 if kk == 1 else 2 * kk)
            n = max(4 * kk, 256)
            t = timed_steps(eng, n, 1)  # uninstrumented (events between launches cost time)
            if kk == 1:  # the k = 1 launch duration for hbm_roofline_k1: a separate evented run
                eng.timing(True)
                timed_steps(eng, n, 1)
                ms1, l1, _ = eng.kernel_time()
                k1_launch_us = ms1 * 1e3 / max(l1, 1)
                eng.timing(False)
            sweep[str(kk)] = round(width * height * n / t / 1e9, 1)
        eng.set_k(a.k)
        eng.set_fixed_k(False)

    checksum = eng.alive_count()  # collective
    eng.close()
    del eng

    # configs[3]: the 262144^2 board (seed 4) row-strip sharded over the N ranks (strong scaling
    # of a fixed board; per-GPU rate comparable across N), RCCL halos when N > 1
    strong = None
    if not a.no_strong:
        n = a.strong_size
        sid = None
        if world > 1 and not host_comm:  # a fresh RCCL unique id per communicator
            obj = [golhip.nccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            sid = obj[0]
        se = golhip.Engine(n, n, k=a.k, rank=rank, world_size=world, device=local, nccl_id=sid,
                           host_comm=golhip.GlooHostComm() if host_comm else None)
        ENGINES.append(se)
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
        exp = golden_count(n, n, 4, a.k + a.strong_steps)
        if exp is not None:
            strong["parity"] = {"turn": a.k + a.strong_steps, "golden": exp,
                                "ok": int(strong_alive) == exp}

    # per-turn CellFlipped path (gol/distributor.go:53-59; the TestSdl event stream): every turn's
    # flips through golhip_step_flips (device ring + one extraction per call) vs the one-turn
    # path (golhip_step(1) + golhip_flips per turn), wall time per turn incl. the host copy
    flips = None
    if world == 1 and not a.no_flips:
        flips = {}
        for n in (512, 5120):
            fe = golhip.Engine(n, n, k=a.k)
            fe.init_random(7)
            cap = fe.flips_ring_capacity()
            T = min(cap, 128)
            # warm each form on the turns it then times (the host lists are sized by the densest
            # call, the first: a list that outgrew its buffer inside the timed loop would be
            # re-allocated and fetched again there)
            fe.step_flips(T)  # allocate the ring, warm
            fe.init_random(7)
            fe.step_flips_rows(T)
            reps = max(1, 2048 // T)
            cells = 0
            fe.init_random(7)  # both forms time the same turns of the same board
            t0 = time.perf_counter()
            for _ in range(reps):
                per_turn, _ = fe.step_flips(T)
                cells += sum(len(x) for x in per_turn)
            dt = time.perf_counter() - t0
            # the compact form (golhip_step_flips_rows: uint16 x + per-turn-row offsets)
            fe.init_random(7)
            cells_r = 0
            t2 = time.perf_counter()
            for _ in range(reps):
                x, _, _ = fe.step_flips_rows(T)
                cells_r += len(x)
            dt2 = time.perf_counter() - t2
            t1 = time.perf_counter()
            for _ in range(64):
                fe.step(1)
                fe.flips()
            dt1 = time.perf_counter() - t1
            fe.close()
            flips[f"{n}x{n}"] = {"us_per_turn": round(dt / (reps * T) * 1e6, 2),
                                 "turns_per_call": T, "flips_per_turn": round(cells / (reps * T), 1),
                                 "us_per_turn_rows": round(dt2 / (reps * T) * 1e6, 2),
                                 "rows_same_cells": cells_r == cells,
                                 "us_per_turn_step1_then_flips": round(dt1 / 64 * 1e6, 2)}

    small = None
    if world == 1 and not a.no_configs:
        small = configs_leg()
    host5 = None
    if world == 1 and not a.no_host:
        host5 = cfg5_host_leg()

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(a.cpu_size, a.cpu_turns, threads_per_server=a.cpu_threads_per_server or None)

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
                             f"{world} row strip(s) of {local_rows} rows, up to k={a.k} gens/launch "
                             f"(timed launches: " + " + ".join(f"{c}x{d}" for d, c in sorted(depth_count.items())) + ")"),
                "width": width, "height": height, "k": a.k, "parallelism": f"rows{world}",
            },
            "parity": parity,
            "preheat_ms": a.preheat_ms,
            # every generation this process computed on the bench board before the timed region
            # (the cold-start pass's warmup + steps, the pre-heat turns, then this pass's warmup;
            # the board is re-initialised from the seed before the last warmup): a plain
            # --steps 20 --warmup 5 line is measured on a warmed chip, its idle-clock figure is
            # cold_start
            "untimed_generations_before_value": (
                a.warmup + (a.warmup + a.steps + cold["preheat_turns"] if cold else 0)),
            "transport": "gloo host transport (test hook GOLHIP_HOST_COMM=1)" if host_comm else
                         ("rccl, every rank on one GPU (test hook GOLHIP_RCCL_SHARED_GPU=1: RCCL's "
                          "network transport over loopback)" if rccl_shared else
                          "rccl" if world > 1 else
                          "rccl ring of one (GOLHIP_RING_SELF=1)" if os.environ.get("GOLHIP_RING_SELF") == "1" else None),
            # the library the line was measured with: its C ABI version and a hash of the file
            "library": library_identity(),
            "process": {"gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                        "process_group": dist.get_backend() if dist.is_initialized() else None,
                        "barrier": ("shared memory" if SHM_BARRIER is not None else
                                    dist.get_backend() if dist.is_initialized() else None)},
            # the same warmup + timed turns measured first, on the chip as the process found it
            # (idle clock): what a 20-turn run pays before the clock has ramped
            "cold_start": cold,
            # the roofline's launch durations: an identical pass after the timed one, with events
            "instrumented_pass": instrumented,
            "per_rank": per_rank,
            "roofline": roof,
            "hbm_roofline": hbm_roof,
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
            "flips_path": flips,
            "configs": small,
            # configs[4]'s own metric: the host contract's throughput with per-turn TurnComplete,
            # tick and key latency, every tick / the snapshot / the final count vs the goldens
            "cfg5_host": host5,
            "alive_after_timed": int(alive_timed),
            "alive_after": int(checksum),
        }
        print(json.dumps(line), flush=True)
    if SHM_BARRIER is not None:
        SHM_BARRIER.close()
    if dist.is_initialized():
        dist.destroy_process_group()
    # a wrong board is not a result: the line above is printed for the record, then the run fails
    bad = [name for name, failed in (
        ("the timed board (alive count or digest)", parity and not parity["ok"]),
        ("strong_262144", strong and strong.get("parity") and not strong["parity"]["ok"]),
        ("configs", small and not small["ok"]),
        ("cfg5_host (a run failed, or a count / snapshot differs)", host5 and "ok" in host5 and not host5["ok"]),
    ) if failed]
    if bad:
        raise SystemExit("bench FAILED against the oracle / goldens: " + "; ".join(bad))


if __name__ == "__main__":
    try:
        main()
    except SystemExit:
        raise
    except BaseException as e:  # a failed engine call or collective: say where, exit non-zero
        rank = os.environ.get("RANK", "0")
        calls = ", ".join(f"{getattr(x, 'last_call', '?')}" for x in ENGINES) or "none"
        print(f"bench: rank {rank} failed: {e!r}; last engine call(s): {calls}", file=sys.stderr,
              flush=True)
        sys.stdout.flush()
        # after an RCCL failure: abort every engine's failed communicator (ncclCommAbort makes the
        # RCCL kernels spinning on the stuck transfer exit: profiles/r05/r05d_stuck_rccl_receive_abort.log),
        # then leave without the interpreter's teardown
        for x in ENGINES:
            try:
                x.comm_abort()
            except Exception:
                pass
        os._exit(3)
