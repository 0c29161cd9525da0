"""Test hook for plain `python bench.py --gpus N` runs on CPU (tests/test_bench_multirank_cpu.py).

A test puts this directory first on PYTHONPATH and sets GOLHIP_TEST_FAKE_ENGINE=1.  Every Python
process started that way -- the launcher bench.py becomes and the N rank processes it starts --
then runs with golhip.Engine replaced by tests/fake_engine.FakeEngine (gloo halos, oracle steps) and
no-op torch.cuda.set_device / synchronize, so the launcher and the ranks' control flow run exactly
as on a GPU node.  Each rank writes its engine-call log to $GOLHIP_TEST_FAKE_LOG_DIR/rank<R>.log at
exit; GOLHIP_TEST_FAKE_FAIL_RANK=R makes rank R's first step raise.  Without GOLHIP_TEST_FAKE_ENGINE=1 this module does nothing."""
import os

if os.environ.get("GOLHIP_TEST_FAKE_ENGINE") == "1":
    import atexit
    import json
    import sys
    from pathlib import Path

    _tests = Path(__file__).resolve().parents[1]
    _root = _tests.parent
    for _p in (str(_tests), str(_root / "oracle"), str(_root / "distributed-gol_amd"), str(_root)):
        if _p not in sys.path:
            sys.path.insert(0, _p)
    import torch

    torch.cuda.set_device = lambda d: None
    torch.cuda.synchronize = lambda *a, **k: None
    import golhip
    from fake_engine import FakeEngine

    if os.environ.get("GOLHIP_TEST_FAKE_FAIL_RANK") == os.environ.get("RANK", "-"):
        class _FailingEngine(FakeEngine):  # GOLHIP_TEST_FAKE_FAIL_RANK=R: rank R's first step fails
            def step(self, turns, counts=False):
                raise RuntimeError("injected engine failure (GOLHIP_TEST_FAKE_FAIL_RANK)")

        golhip.Engine = _FailingEngine
    else:
        golhip.Engine = FakeEngine
    golhip.nccl_unique_id = lambda: b"x" * 128

    def _dump():
        d, rank = os.environ.get("GOLHIP_TEST_FAKE_LOG_DIR"), os.environ.get("RANK")
        if d and rank is not None:
            with open(os.path.join(d, f"rank{rank}.log"), "w") as f:
                json.dump(FakeEngine.log, f)

    atexit.register(_dump)
