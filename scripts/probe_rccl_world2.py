"""Probe: two RCCL ranks on ONE GPU.

RCCL refuses two ranks of a communicator on the same device ("Duplicate GPU detected"): its check
compares (host hash, bus id).  A distinct NCCL_HOSTID per rank gives each rank its own host hash,
so RCCL builds a real 2-rank communicator whose transfers go through its network transport
(NET/Socket over loopback) -- the RCCL calls of the rank engine (ncclCommInitRankConfig with
several ranks, the grouped send/recv between ranks, ncclAllReduce) then run for real on a one-GPU
box.  Each rank checks its strip and every count against the oracle.

usage: python scripts/probe_rccl_world2.py [world] [width] [height] [k]
"""
import json
import os
import socket
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, width, height, k, out):
    os.environ["NCCL_HOSTID"] = f"golhip-probe-rank{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for p in (str(ROOT / "oracle"), str(ROOT / "distributed-gol_amd")):
        sys.path.insert(0, p)
    import numpy as np
    import torch.distributed as dist

    import golhip
    import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    obj = [golhip.nccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    golhip.set_default_comm_timeout(60000)
    res = {"rank": rank}
    t0 = time.perf_counter()
    try:
        with golhip.Engine(width, height, k=k, rank=rank, world_size=world, device=0, nccl_id=obj[0]) as e:
            res["create_s"] = round(time.perf_counter() - t0, 3)
            y0, rows = e.info.y0, e.info.rows
            ref = oracle.init_random(width, height, seed=11)
            e.load_words(ref[y0:y0 + rows])
            sched = [1, 7, 20, 33, 16, 3]
            t1 = time.perf_counter()
            counts = np.concatenate([e.step(n, counts=True) for n in sched])
            res["steps_s"] = round(time.perf_counter() - t1, 3)
            got = e.store_words()
            exp = oracle.packed_run_words(ref, sum(sched))
            res["counts_ok"] = bool(np.array_equal(counts.astype(np.int64), exp))
            res["strip_ok"] = bool(np.array_equal(got, ref[y0:y0 + rows]))
            res["alive_ok"] = e.alive_count() == int(exp[-1])
    except golhip.GolHipError as err:
        res["error"] = str(err)
    res["total_s"] = round(time.perf_counter() - t0, 3)
    Path(out, f"rank{rank}.json").write_text(json.dumps(res))
    print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    import tempfile

    import torch.multiprocessing as mp

    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    height = int(sys.argv[3]) if len(sys.argv) > 3 else 1001
    k = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    out = tempfile.mkdtemp()
    mp.start_processes(worker, args=(world, _free_port(), width, height, k, out), nprocs=world,
                       join=True, start_method="spawn")
    res = [json.loads(Path(out, f"rank{r}.json").read_text()) for r in range(world)]
    ok = all(r.get("counts_ok") and r.get("strip_ok") and r.get("alive_ok") for r in res)
    print(json.dumps({"world": world, "width": width, "height": height, "k": k, "ok": ok, "ranks": res}))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
