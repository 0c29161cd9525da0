#!/usr/bin/env python3
"""Rank-mode (one process per GPU, RCCL halos) self-test: launch with
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
      scripts/rank_selftest.py [width height k turns]
Every rank builds its strip with golhip_create_rank, steps with per-turn counts (collective), and
rank 0 checks the gathered board and counts against one single-strip engine of the whole board.
Ranks share GPUs round-robin when there are fewer devices than ranks (RCCL may refuse that)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import golhip  # noqa: E402

w, h, k, turns = (int(x) for x in (sys.argv[1:5] if len(sys.argv) >= 5 else (4096, 1030, 8, 37)))
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
local = int(os.environ.get("LOCAL_RANK", rank))
dist.init_process_group("gloo", rank=rank, world_size=world)
ndev = torch.cuda.device_count()
obj = [golhip.nccl_unique_id() if rank == 0 else None]
dist.broadcast_object_list(obj, src=0)
e = golhip.Engine(w, h, k=k, rank=rank, world_size=world, device=local % ndev, nccl_id=obj[0])
e.init_random(7)
counts = e.step(turns, counts=True)
mine = e.store_words()
total = e.alive_count()
parts = [None] * world
dist.all_gather_object(parts, mine)
e.close()
if rank == 0:
    got = np.concatenate(parts)
    with golhip.Engine(w, h, k=k, device=0) as ref:
        ref.init_random(7)
        rc = ref.step(turns, counts=True)
        want = ref.store_words()
    ok = np.array_equal(got, want) and np.array_equal(counts, rc) and total == int(rc[-1])
    print(f"rank_selftest world={world} devices={ndev} {w}x{h} k={k} turns={turns}: "
          f"{'OK' if ok else 'MISMATCH'}", flush=True)
    if not ok:
        sys.exit(1)
dist.barrier()
dist.destroy_process_group()
