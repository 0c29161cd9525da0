import sys
sys.path.insert(0, "distributed-gol_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np, golhip
from test_gpu_activity import sparse_board
for (h, w, graphs) in [(1000, 600, 0), (1152, 2048, 0), (4096, 4096, 0), (4096, 4096, -1)]:
    b = sparse_board(h, w, seed=h + w, **({} if w % 128 == 0 else dict(n_gliders=1, n_osc=1, n_still=1)))
    with golhip.Engine(w, h, k=16) as e:
        e.set_graphs(graphs)
        e.load(b)
        print(h, w, graphs, e.launch_kind(16, counts=True), e.launch_kind(16), golhip.launch_plan(w, h, 16, 64))
        for n in (64, 64, 64):
            e.step(n, counts=True)
            print("  counts", e.activity_stats())
        for n in (64, 64):
            e.step(n)
            print("  plain", e.activity_stats())
