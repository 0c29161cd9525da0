"""bench.py's N > 1 control flow on CPU: two, three and eight gloo ranks run bench.main() exactly as
`torch.distributed.run --nproc-per-node N bench.py --gpus N ...` would, with the GPU engine replaced
by a host stand-in.  The driver's 8-GPU scaling run is the only place the RCCL rank path meets
hardware, so this checks what can break there without a GPU: every rank makes the same collective
calls in the same order (barriers, the max-over-ranks timing, the pre-heat turn count taken from
the cold pass), no N == 1-only leg runs, rank 0 prints one well-formed JSON line with the whole-job
value, and that line's `parity` is set and true: the N > 1 weak-scaling boards have committed
oracle goldens (tests/golden/weak_*), and bench.py checks its alive count against them.

The stand-in holds its own row strip (+ k halo rows each side) and really advances it: each
k-block exchanges halos over gloo in golhip_halo_plan's order (the order the engine issues its
RCCL send/recv in) and steps the halo'd strip with the CPU oracle; alive_count is the strip's
popcount summed over the ranks (the engine's count all-reduce).  The GPU engine itself runs at
world 2 and 3 in tests/test_gpu_rank_host.py (host transport instead of RCCL on one GPU).
"""
import json
import os
import socket
import sys
from pathlib import Path

import pytest
import torch.multiprocessing as mp

from conftest import PKG, ROOT
from fake_engine import FakeEngine


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, extra=()):
    for p in (str(ROOT), str(ROOT / "oracle"), str(PKG)):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch

    torch.cuda.set_device = lambda d: None
    torch.cuda.synchronize = lambda *a, **k: None
    import golhip

    golhip.Engine = FakeEngine
    golhip.nccl_unique_id = lambda: b"x" * 128
    import bench

    sys.argv = ["bench.py", "--gpus", str(world), "--steps", "20", "--warmup", "5",
                "--size", "4096", "--strong-size", "2048", "--strong-steps", "32",
                "--preheat-ms", "50", *extra]
    out = os.path.join(out_dir, f"rank{rank}.out")
    with open(out, "w") as f:
        so = sys.stdout
        sys.stdout = f
        try:
            bench.main()
        finally:
            sys.stdout = so
    with open(os.path.join(out_dir, f"rank{rank}.log"), "w") as f:
        json.dump(FakeEngine.log, f)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_rank_path_cpu(tmp_path, world):
    shm_before = set(Path("/dev/shm").glob("golhip_bench_*"))
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    logs = [json.loads((tmp_path / f"rank{r}.log").read_text()) for r in range(world)]
    # every rank issued the same sequence of engine calls (step sizes included): the pre-heat
    # turn count is the same everywhere, so the RCCL exchanges of the real engine would pair up
    steps = [[e for e in log if e[0] in ("step", "init", "close")] for log in logs]
    assert all(s == steps[0] for s in steps[1:])
    creates = [[e for e in log if e[0] == "create"] for log in logs]
    assert [c[0][3] for c in creates] == list(range(world))  # one engine per rank, its own strip
    assert all(len(c) == 2 for c in creates)  # the weak-scaling board and the 262144^2-style leg
    # rank 0 prints exactly one JSON line, the others nothing
    out0 = (tmp_path / "rank0.out").read_text().strip().splitlines()
    assert len(out0) == 1
    for r in range(1, world):
        assert (tmp_path / f"rank{r}.out").read_text().strip() == ""
    line = json.loads(out0[0])
    assert line["n_gpus"] == world and line["steps"] == 20 and line["warmup"] == 5
    assert line["config"]["height"] == 4096 * world and line["config"]["parallelism"] == f"rows{world}"
    assert line["scaling"] == "weak" and line["value"] > 0
    # N > 1: no k sweep, configs leg, flips leg or CPU baseline; pre-heat ran after a cold pass
    assert line["k_sweep_gcups"] is None and line["configs"] is None
    assert line["flips_path"] is None and line["cpu_baseline"] is None
    assert line["cold_start"]["preheat_turns"] >= 16
    assert line["strong_262144"]["rows_per_gpu"] == -(-2048 // world)
    # the weak-scaling board (4096 x 4096*N, seed 3) is pinned: parity against the oracle golden
    # at turn warmup + steps, in both the pre-heated and the cold-start pass; and bit for bit:
    # every rank hashed its strip, rank 0 the gathered chunk digests == the oracle's board digest
    assert line["parity"] is not None and line["parity"]["turn"] == 25
    assert line["parity"]["ok"] and line["parity"]["cold_start_ok"], line["parity"]
    assert line["parity"]["digest_ok"] is True, line["parity"]
    # every rank on this node: the timed region's barriers through shared memory, file removed
    assert line["process"]["barrier"] == "shared memory", line["process"]
    assert set(Path("/dev/shm").glob("golhip_bench_*")) <= shm_before
    assert line["untimed_generations_before_value"] == 5 + 25 + line["cold_start"]["preheat_turns"]
    # per-rank data: every rank's timed-region and instrumented wall time, kernel span, edge wait
    pr = line["per_rank"]
    assert [r["rank"] for r in pr] == list(range(world)), pr
    assert sum(r["rows"] for r in pr) == 4096 * world and [r["y0"] for r in pr] == sorted(r["y0"] for r in pr)
    for r in pr:
        assert r["timed_ms"] > 0 and r["instrumented_ms"] > 0 and r["kernel_span_ms"] > 0, r
        assert r["launches"] >= 1 and r["edge_wait_ms"] >= 0 and r["split_blocks"] >= 1, r
    # the line's value is the max over the ranks' timed regions
    assert abs(line["ms_per_step"] * 20 - max(r["timed_ms"] for r in pr)) < 1e-3 * 20 + 1e-6, (line["ms_per_step"], pr)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_plain_launch_cpu(tmp_path, world):
    """`python bench.py --gpus N` run plainly, as the driver runs the 1-GPU bench (no
    torch.distributed.run, WORLD_SIZE unset): bench.py starts the N rank processes itself
    (launch_ranks, before importing torch) and exits with their status; rank 0's line is the
    command's one stdout line.  tests/fake_site/sitecustomize.py swaps in the CPU engine stand-in
    in every process the command starts (gloo halos)."""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYTHONPATH=os.pathsep.join([str(ROOT / "tests" / "fake_site"), env.get("PYTHONPATH", "")]),
               GOLHIP_TEST_FAKE_ENGINE="1", GOLHIP_TEST_FAKE_LOG_DIR=str(tmp_path), OMP_NUM_THREADS="1")
    shm_before = set(Path("/dev/shm").glob("golhip_bench_*"))
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--steps", "20",
                        "--warmup", "5", "--size", "4096", "--strong-size", "1024", "--strong-steps", "16",
                        "--preheat-ms", "20"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert f"launched {world} rank processes" in r.stderr
    out = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(out) == 1, r.stdout
    line = json.loads(out[0])
    assert line["n_gpus"] == world and line["config"]["height"] == 4096 * world
    assert [p["rank"] for p in line["per_rank"]] == list(range(world))
    assert line["process"]["barrier"] == "shared memory"
    assert line["parity"] is not None and line["parity"]["ok"] and line["parity"]["digest_ok"] is True, line["parity"]
    logs = [json.loads((tmp_path / f"rank{rank}.log").read_text()) for rank in range(world)]
    assert [[e for e in lg if e[0] == "create"][0][3] for lg in logs] == list(range(world))
    assert set(Path("/dev/shm").glob("golhip_bench_*")) <= shm_before


def test_bench_plain_launch_rank_failure(tmp_path):
    """A rank that fails makes the plain launch fail: the launcher stops the other ranks and exits
    non-zero (no line is taken for a result)."""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYTHONPATH=os.pathsep.join([str(ROOT / "tests" / "fake_site"), env.get("PYTHONPATH", "")]),
               GOLHIP_TEST_FAKE_ENGINE="1", GOLHIP_TEST_FAKE_FAIL_RANK="1", OMP_NUM_THREADS="1")
    t = __import__("time").perf_counter()
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5",
                        "--size", "2048", "--preheat-ms", "20", "--k", "8", "--pg-timeout-s", "20"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert "rank exit codes" in r.stderr, r.stderr[-3000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert __import__("time").perf_counter() - t < 120


def test_bench_rank_path_cpu_process_group_barrier(tmp_path):
    """--rccl-barrier: the timed region between the process group's barriers (here gloo) even when
    every rank is on this node; the same line otherwise."""
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path), ("--rccl-barrier",)), nprocs=2,
                       join=True, start_method="spawn")
    line = json.loads((tmp_path / "rank0.out").read_text().strip().splitlines()[0])
    assert line["process"]["barrier"] == "gloo", line["process"]
    assert line["parity"]["ok"] and line["parity"]["digest_ok"] is True, line["parity"]


def _barrier_worker(rank, world, port, out_dir):
    for p in (str(ROOT), str(PKG)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import time

    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import bench

    b = bench.ShmBarrier.create(rank, world, timeout_s=2.0)
    assert b is not None
    order = []
    for i in range(3):  # a barrier holds every rank until all have arrived
        if rank == world - 1:
            time.sleep(0.2)
        b.wait()
        order.append(time.time())
    result = {"ok_waits": 3, "times": order}
    if rank == 0:  # the other ranks never arrive at a 4th barrier: rank 0 fails at the deadline
        t = time.perf_counter()
        try:
            b.wait()
            result["timeout"] = None
        except RuntimeError as e:
            result["timeout"] = str(e)
        result["waited"] = time.perf_counter() - t
    dist.barrier()
    b.close()
    with open(os.path.join(out_dir, f"b{rank}.json"), "w") as f:
        json.dump(result, f)
    dist.destroy_process_group()


def test_shm_barrier_holds_ranks_and_times_out(tmp_path):
    """bench.ShmBarrier: no rank leaves a barrier before every rank has arrived (the late rank's
    0.2 s delay shows in every rank's exit time), and a rank whose peer never arrives fails at the
    deadline naming the missing ranks."""
    world = 3
    shm_before = set(Path("/dev/shm").glob("golhip_bench_*"))
    mp.start_processes(_barrier_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    res = [json.loads((tmp_path / f"b{r}.json").read_text()) for r in range(world)]
    for i in range(3):
        exits = [r["times"][i] for r in res]
        assert max(exits) - min(exits) < 0.15, exits  # released together, after the late rank
    assert res[0]["timeout"] and "ranks [1, 2] did not arrive" in res[0]["timeout"], res[0]
    assert 1.9 <= res[0]["waited"] < 10, res[0]
    assert set(Path("/dev/shm").glob("golhip_bench_*")) <= shm_before


def _fallback_worker(rank, world, port, out_dir):
    for p in (str(ROOT), str(PKG)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import bench

    if rank == 1:  # this rank cannot map the page
        real_open = os.open

        def failing_open(path, *a, **k):
            if "golhip_bench_" in str(path):
                raise OSError("no shared memory here")
            return real_open(path, *a, **k)

        os.open = failing_open
    b = bench.ShmBarrier.create(rank, world, timeout_s=2.0)
    with open(os.path.join(out_dir, f"f{rank}.json"), "w") as f:
        json.dump({"barrier": b is not None}, f)
    dist.destroy_process_group()


def test_shm_barrier_all_or_none(tmp_path):
    """One rank that cannot map the page makes EVERY rank keep the process group's barrier (the
    ranks must not wait in different barriers), and no file is left behind."""
    world = 3
    shm_before = set(Path("/dev/shm").glob("golhip_bench_*"))
    mp.start_processes(_fallback_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    res = [json.loads((tmp_path / f"f{r}.json").read_text()) for r in range(world)]
    assert [r["barrier"] for r in res] == [False] * world, res
    assert set(Path("/dev/shm").glob("golhip_bench_*")) <= shm_before


def test_bench_plain_launch_ranks_die_with_launcher(tmp_path):
    """The launcher's ranks never outlive it: SIGTERM to the launcher stops every rank (it relays the
    stop, then exits 143), and a rank's parent-death signal covers a launcher that is killed outright."""
    import signal
    import subprocess
    import time

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYTHONPATH=os.pathsep.join([str(ROOT / "tests" / "fake_site"), env.get("PYTHONPATH", "")]),
               GOLHIP_TEST_FAKE_ENGINE="1", OMP_NUM_THREADS="1")
    for sig in (signal.SIGTERM, signal.SIGKILL):
        # a long run (many steps of a big board) that the signal interrupts
        p = subprocess.Popen([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "100000",
                              "--warmup", "5", "--size", "4096", "--preheat-ms", "20"],
                             cwd=str(tmp_path), env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        pids = []
        t_end = time.time() + 120
        while time.time() < t_end and len(pids) < 2:  # the launcher names its ranks on stderr
            line = p.stderr.readline()
            if "launched 2 rank processes" in line:
                pids = [int(x) for x in line.split("pids [")[1].split("]")[0].split(",")]
        assert len(pids) == 2
        time.sleep(3)
        p.send_signal(sig)
        p.wait(timeout=60)
        if sig == signal.SIGTERM:
            assert p.returncode == 143, p.returncode
        deadline = time.time() + 30
        alive = pids
        while alive and time.time() < deadline:
            alive = [q for q in pids if os.path.exists(f"/proc/{q}") and
                     open(f"/proc/{q}/stat").read().split()[2] != "Z"]
            time.sleep(0.2)
        assert not alive, (sig, alive)
