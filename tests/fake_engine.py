"""Host stand-in for golhip.Engine in rank mode (the calls bench.py makes), used by the CPU tests of
bench.py's N > 1 path (tests/test_bench_multirank_cpu.py).  Test infrastructure: it steps its strip
with the oracle, as the checker, and exchanges k-row halos with its ring neighbours over gloo in
golhip_halo_plan's order (the order the engine issues its RCCL send/recv in)."""
import numpy as np


class _Info:
    def __init__(self, rows, y0, width):
        self.rows, self.y0, self.width = rows, y0, width


class FakeEngine:
    """Host stand-in for golhip.Engine in rank mode (the calls bench.py makes), stepping its strip
    with the oracle and exchanging k-row halos with its ring neighbours over gloo."""

    log = []

    def __init__(self, width, height, ngpus=1, k=1, *, rank=None, world_size=None, device=0,
                 nccl_id=None, host_comm=None):
        import golhip

        assert world_size and world_size > 1 and nccl_id is not None and len(nccl_id) > 0
        assert host_comm is None
        self.y0, rows = golhip.strip_bounds(height, world_size, rank)
        self.width, self.height, self.rows, self.k = width, height, rows, k
        self.rank, self.world = rank, world_size
        self.buf = np.zeros((rows + 2 * k, width // 64), dtype=np.uint64)
        self.info = _Info(rows, self.y0, width)
        self.last_call = "golhip_create_rank"
        self.turn = 0
        self.timed = False
        self.t_ms = 0.0
        self.launches = 0
        self.gens = 0
        FakeEngine.log.append(("create", width, height, rank, world_size))

    def init_random(self, seed):
        import oracle

        k = self.k
        self.buf[k:k + self.rows] = oracle.init_random(self.width, self.height, seed,
                                                       y0=self.y0, y1=self.y0 + self.rows)
        self.turn = 0
        FakeEngine.log.append(("init", seed))

    def set_band_rows(self, n):
        pass

    def set_fixed_k(self, fixed):
        pass

    def store_words(self):
        FakeEngine.log.append(("store_words",))
        return self.buf[self.k:self.k + self.rows].copy()

    def _block(self, K):
        import golhip
        import oracle
        import torch
        import torch.distributed as dist

        k, buf = self.k, self.buf
        sent, recvd, reqs, landing = {}, {}, [], []
        for kind, peer, row, n in golhip.halo_plan(self.height, self.world, self.rank, K):
            if kind == "send":
                tag = sent.get(peer, 0)
                sent[peer] = tag + 1
                t = torch.from_numpy(buf[k + row:k + row + n].view(np.int64).copy())
                reqs.append(dist.isend(t, dst=peer, tag=tag))
            else:
                tag = recvd.get(peer, 0)
                recvd[peer] = tag + 1
                t = torch.empty((n, buf.shape[1]), dtype=torch.int64)
                reqs.append(dist.irecv(t, src=peer, tag=tag))
                landing.append((row, n, t))
        for r in reqs:
            r.wait()
        for row, n, t in landing:
            buf[k + row:k + row + n] = t.numpy().view(np.uint64)
        # K generations of the strip with K halo rows each side: the rows past the halos are
        # garbage that reaches the strip's own rows only after K generations
        ext = np.ascontiguousarray(buf[k - K:k + self.rows + K])
        oracle.packed_run_words(ext, K, threads=2)
        buf[k:k + self.rows] = ext[K:K + self.rows]

    def step(self, turns, counts=False):
        import time

        assert not counts
        t0 = time.perf_counter()
        left = turns
        while left > 0:
            K = min(self.k, left)
            self._block(K)
            left -= K
            if self.timed:
                self.launches += 1
        if self.timed:
            self.t_ms += (time.perf_counter() - t0) * 1e3
            self.gens += turns
        self.turn += turns
        FakeEngine.log.append(("step", turns))

    def sync(self):
        pass

    def timing(self, enable):
        self.timed = bool(enable)

    def kernel_time(self):
        return self.t_ms, self.launches, self.gens

    def edge_wait(self):
        return 0.0, self.launches

    def alive_count(self):
        import torch
        import torch.distributed as dist

        own = self.buf[self.k:self.k + self.rows]
        c = int(np.unpackbits(own.view(np.uint8)).sum())
        t = torch.tensor([c], dtype=torch.int64)  # collective, like the engine's count all-reduce
        dist.all_reduce(t)
        return int(t.item())

    def close(self):
        FakeEngine.log.append(("close",))
