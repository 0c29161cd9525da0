"""The N>1 decomposition on CPU: world_size 2 and 3 gloo process groups run the engine's OWN strip
split (golhip_strip_bounds) and halo plan (golhip_halo_plan, the order the engine issues its RCCL
send/recv in) with the transfers carried by gloo, and the oracle stepping each halo'd strip.
The stitched board must equal the single-board oracle bit for bit.

Reference analogue: broker/broker.go:37-56 (strip split), :168-174 (stitch) -- which broadcasts the
whole world instead of exchanging halos."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, width, height, k, rounds, result_dir):
    import sys

    for p in (str(ROOT / "oracle"), str(PKG)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import golhip
    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    y0, rows = golhip.strip_bounds(height, world, rank)
    wpr = width // 64
    full = oracle.init_random(width, height, seed=11)
    buf = np.zeros((rows + 2 * k, wpr), dtype=np.uint64)  # [k halo | strip | k halo]
    buf[k:k + rows] = full[y0:y0 + rows]
    for _ in range(rounds):
        plan = golhip.halo_plan(height, world, rank, k)
        # RCCL semantics: the i-th send from A to B matches the i-th recv on B from A
        sent, recvd, reqs, landing = {}, {}, [], []
        for kind, peer, row, n in plan:
            if kind == "send":
                tag = sent.get(peer, 0)
                sent[peer] = tag + 1
                t = torch.from_numpy(buf[k + row:k + row + n].view(np.int64).copy())
                reqs.append(dist.isend(t, dst=peer, tag=tag))
            else:
                tag = recvd.get(peer, 0)
                recvd[peer] = tag + 1
                t = torch.empty((n, wpr), dtype=torch.int64)
                reqs.append(dist.irecv(t, src=peer, tag=tag))
                landing.append((row, n, t))
        for r in reqs:
            r.wait()
        for row, n, t in landing:
            buf[k + row:k + row + n] = t.numpy().view(np.uint64)
        # k generations of the halo'd strip: garbage from its open edges travels 1 row per
        # generation, so after k generations the strip's own rows are exact
        ext = np.ascontiguousarray(buf)
        oracle.packed_run_words(ext, k, threads=1)
        buf[k:k + rows] = ext[k:k + rows]
    np.save(os.path.join(result_dir, f"strip{rank}.npy"), buf[k:k + rows])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,width,height,k,rounds", [
    (2, 128, 64, 1, 5), (2, 256, 90, 4, 3), (3, 192, 61, 2, 4), (2, 128, 40, 8, 2),
])
def test_strips_with_halo_exchange_match_single_board(tmp_path, oracle, world, width, height, k,
                                                      rounds):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, width, height, k, rounds, str(tmp_path)), nprocs=world,
             join=True)
    got = np.concatenate([np.load(tmp_path / f"strip{r}.npy") for r in range(world)])
    ref = oracle.init_random(width, height, seed=11)
    oracle.packed_run_words(ref, k * rounds)
    assert np.array_equal(got, ref)
