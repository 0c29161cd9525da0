"""The rank-mode ENGINE at world 2 and 3 on one GPU, over both of its transports:
  * "rccl": REAL RCCL ranks sharing this GPU -- a distinct NCCL_HOSTID per rank makes RCCL treat the
    ranks as separate hosts (it refuses two ranks on one device otherwise: "Duplicate GPU") and
    connect them through its network transport over loopback.  So ncclCommInitRankConfig with
    several ranks, the grouped ncclSend/ncclRecv between ranks and the count ncclAllReduce run for
    real -- what the driver's 8-GPU node runs, minus xGMI;
  * "host": golhip_create_rank_host, the same engine with the halos and count sums carried by a
    gloo host transport.
Either way: per-rank strips, the rank-independent launch plan, golhip_halo_plan's transfer order,
the interior launch overlapped with the two boundary bands, the per-turn count reduction.  Every
rank's strip, every per-turn count, the alive-cell list and the per-turn flips must equal the
single-board oracle.

Reference analogue: broker/broker.go:37-56 (strip fan-out), :168-174 (stitch),
gol/distributor.go:53-59,153-166 (flips, alive cells); the reference broadcasts the whole world to
every server instead of exchanging halos.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SCHEDULE = [1, 7, 20, 33, 16, 3]  # K = 1 launches, tail plans, bulk depths, a short call


def _worker(rank, world, port, width, height, k, out_dir, transport="host"):
    for p in (str(ROOT / "oracle"), str(PKG)):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if transport == "rccl":  # before anything initialises RCCL in this process
        os.environ["NCCL_HOSTID"] = f"golhip-test-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    import torch.distributed as dist

    import golhip
    import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm, nid = None, None
    if transport == "host":
        comm = golhip.GlooHostComm()
    else:
        obj = [golhip.nccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        nid = obj[0]
    res = {}
    with golhip.Engine(width, height, k=k, rank=rank, world_size=world, device=0,
                       host_comm=comm, nccl_id=nid) as e:
        y0, rows = e.info.y0, e.info.rows
        assert (y0, rows) == golhip.strip_bounds(height, world, rank)
        e.load_words(oracle.init_random(width, height, seed=11)[y0:y0 + rows])
        counts = [e.step(n, counts=True) for n in SCHEDULE]
        res["counts"] = np.concatenate(counts)
        res["alive"] = np.array([e.alive_count()])
        res["words"] = e.store_words()
        res["cells"] = e.alive_cells()
        # fixed-depth launches (every launch exactly 4 deep, then a 2-deep tail)
        e.set_fixed_k(True)
        e.set_k(4)
        res["counts_fixed"] = e.step(10, counts=True)
        e.set_fixed_k(False)
        e.set_k(k)
        # per-turn flips ring (one K = 1 launch and one exchange per turn)
        per_turn, alive = e.step_flips(5, counts=True)
        res["flips_n"] = np.array([len(x) for x in per_turn])
        res["flips"] = np.concatenate([x for x in per_turn]) if any(len(x) for x in per_turn) \
            else np.zeros((0, 2), np.int32)
        res["flips_alive"] = alive
        res["words_end"] = e.store_words()
    if comm is not None:
        res["exchanges"] = np.array([comm.exchanges])
        res["reduced"] = np.array(comm.reduced)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("transport", ["rccl", "host"])
@pytest.mark.parametrize("world,width,height,k", [
    (2, 1024, 1001, 16),   # uneven strips (500 / 501 rows)
    (3, 1024, 1000, 16),   # 333 / 333 / 334
    (2, 2048, 40, 16),     # strips shorter than 3k: the boundary launch waits for the halos
    (3, 576, 197, 8),      # width not a multiple of 128 (the torus is replicated horizontally)
    (4, 1024, 403, 12),    # four ranks
])
def test_rank_engine_matches_oracle(tmp_path, oracle, world, width, height, k, transport):
    mp.start_processes(_worker, args=(world, _free_port(), width, height, k, str(tmp_path), transport),
                       nprocs=world, join=True, start_method="spawn")
    r = [dict(np.load(tmp_path / f"rank{i}.npz")) for i in range(world)]
    ref = oracle.init_random(width, height, seed=11)
    turns = sum(SCHEDULE)
    exp_counts = oracle.packed_run_words(ref, turns)
    for i in range(world):  # the count reduction hands every rank the whole board's counts
        assert np.array_equal(r[i]["counts"].astype(np.int64), exp_counts), i
        assert int(r[i]["alive"][0]) == int(exp_counts[-1])
    assert np.array_equal(np.concatenate([x["words"] for x in r]), ref)
    # alive cells: each rank lists its own strip's cells (global y), row-major
    cells = np.concatenate([x["cells"] for x in r])
    ys, xs = np.nonzero(oracle.unpack(ref, width) == 255)
    assert np.array_equal(cells, np.stack([xs, ys], axis=1).astype(np.int32))
    exp_fixed = oracle.packed_run_words(ref, 10)
    for i in range(world):
        assert np.array_equal(r[i]["counts_fixed"].astype(np.int64), exp_fixed)
    # per-turn flips: per rank its strip's flips of each turn; together the board's
    prev = oracle.unpack(ref, width)
    off = [0] * world
    for t in range(5):
        c = oracle.packed_run_words(ref, 1)
        cur = oracle.unpack(ref, width)
        ys, xs = np.nonzero(prev != cur)
        want = np.stack([xs, ys], axis=1).astype(np.int32)
        got = []
        for i in range(world):
            n = int(r[i]["flips_n"][t])
            got.append(r[i]["flips"][off[i]:off[i] + n])
            off[i] += n
            assert int(r[i]["flips_alive"][t]) == int(c[0])
        assert np.array_equal(np.concatenate(got), want), t
        prev = cur
    assert np.array_equal(np.concatenate([x["words_end"] for x in r]), ref)
    if transport == "host":
        # the transport really carried the exchanges: one per launch; count sums of every call
        ex = [int(x["exchanges"][0]) for x in r]
        assert len(set(ex)) == 1 and ex[0] >= len(SCHEDULE) + 5
        assert all(np.array_equal(x["reduced"], r[0]["reduced"]) for x in r)


@pytest.mark.timeout(700)
def test_bench_rank_path_host_transport(tmp_path):
    """bench.py --gpus 2 and 3 as torch.distributed.run launches it, the ranks sharing this GPU
    through the host transport (GOLHIP_HOST_COMM=1): the real engine, launch plan and timed region
    at N > 1; the line's parity (8192 x 8192*N board, seed 3, oracle golden CSV) must hold."""
    for world in (2, 3):
        env = dict(os.environ, GOLHIP_HOST_COMM="1", PYTHONUNBUFFERED="1")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), str(ROOT / "bench.py"), "--gpus", str(world),
               "--size", "8192", "--steps", "40", "--warmup", "5", "--no-strong",
               "--preheat-ms", "20"]
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, p.stdout
        line = json.loads(lines[0])
        (tmp_path / f"bench_world{world}.json").write_text(lines[0])
        assert line["n_gpus"] == world and line["config"]["height"] == 8192 * world
        assert line["parity"] is not None and line["parity"]["ok"], line["parity"]
        assert line["parity"]["cold_start_ok"]
        assert line["transport"].startswith("gloo host transport")


@pytest.mark.timeout(400)
def test_bench_rank_path_real_rccl_shared_gpu(tmp_path):
    """bench.py --gpus 2 and 3 as torch.distributed.run launches it, every rank a REAL RCCL rank on
    this one GPU (GOLHIP_RCCL_SHARED_GPU=1: distinct NCCL_HOSTIDs, RCCL's network transport): the
    torch process group over RCCL, the engine's RCCL halo exchange and count all-reduce, the
    shared-memory barrier and the per-rank block of the line.  The line's parity and board digest
    (8192 x 8192*N, seed 3, oracle goldens at turn 25) must hold."""
    for world in (2, 3):
        env = dict(os.environ, GOLHIP_RCCL_SHARED_GPU="1", PYTHONUNBUFFERED="1")
        env.pop("GOLHIP_HOST_COMM", None)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), str(ROOT / "bench.py"), "--gpus", str(world),
               "--size", "8192", "--steps", "20", "--warmup", "5", "--no-strong",
               "--preheat-ms", "20", "--comm-timeout-ms", "60000"]
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, p.stdout
        line = json.loads(lines[0])
        (tmp_path / f"bench_rccl_world{world}.json").write_text(lines[0])
        print(lines[0][:2000])
        assert line["n_gpus"] == world and line["config"]["height"] == 8192 * world
        assert line["transport"].startswith("rccl, every rank on one GPU"), line["transport"]
        assert line["process"]["process_group"] == "nccl", line["process"]
        assert line["parity"] is not None and line["parity"]["ok"], line["parity"]
        assert line["parity"]["cold_start_ok"] and line["parity"]["digest_ok"] is True, line["parity"]
        pr = line["per_rank"]
        assert [x["rank"] for x in pr] == list(range(world)), pr
        assert all(x["split_blocks"] >= 1 and x["kernel_span_ms"] > 0 for x in pr), pr


@pytest.mark.timeout(300)
def test_bench_plain_launch_real_rccl_shared_gpu(tmp_path):
    """`python bench.py --gpus 2` run PLAINLY, as the driver runs the bench (no torch.distributed.run):
    bench.py starts its two rank processes itself before touching the GPU (launch_ranks), each a
    real RCCL rank on this one GPU (GOLHIP_RCCL_SHARED_GPU=1).  One JSON line on stdout, exit 0,
    and the line's parity and board digest (8192 x 16384, seed 3, oracle goldens) must hold."""
    env = dict(os.environ, GOLHIP_RCCL_SHARED_GPU="1", PYTHONUNBUFFERED="1")
    for v in ("GOLHIP_HOST_COMM", "WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(v, None)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--size", "8192", "--steps", "20",
           "--warmup", "5", "--no-strong", "--preheat-ms", "20", "--comm-timeout-ms", "60000",
           "--launch-deadline-s", "240"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "launched 2 rank processes" in p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout
    line = json.loads(lines[0])
    (tmp_path / "bench_plain_world2.json").write_text(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["height"] == 16384
    assert line["transport"].startswith("rccl, every rank on one GPU"), line["transport"]
    assert line["parity"]["ok"] and line["parity"]["digest_ok"] is True, line["parity"]
    assert [x["rank"] for x in line["per_rank"]] == [0, 1]


@pytest.mark.timeout(300)
def test_bench_rank_process_rehearsal_ring_of_one(tmp_path):
    """What one rank of the driver's N > 1 run does, on this GPU: bench.py --pg-always creates the
    torch process group over RCCL and runs its collectives at world 1, and GOLHIP_RING_SELF=1 makes
    the engine the RCCL ring of one (the rank-mode split step, RCCL send/recv, the count
    all-reduce); the timed region between shared-memory barriers.  The line's parity and the board
    digest (8192 x 16384, seed 3, oracle goldens) must hold."""
    env = dict(os.environ, GOLHIP_RING_SELF="1", PYTHONUNBUFFERED="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    cmd = [sys.executable, str(ROOT / "bench.py"), "--pg-always", "--size", "8192", "--height", "16384",
           "--steps", "20", "--warmup", "5", "--no-cpu", "--no-sweep", "--no-strong", "--no-configs",
           "--no-flips", "--preheat-ms", "20"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    (tmp_path / "rehearsal.json").write_text(lines[0])
    assert line["transport"] == "rccl ring of one (GOLHIP_RING_SELF=1)", line["transport"]
    assert line["process"]["process_group"] == "nccl" and line["process"]["barrier"] == "shared memory"
    assert line["process"]["gpu_max_hw_queues"] == "8"
    assert line["parity"]["ok"] and line["parity"]["cold_start_ok"], line["parity"]
    assert line["parity"]["digest_ok"] is True, line["parity"]
