"""RCCL fail-fast on one GPU: a rank-mode engine whose RCCL work cannot complete returns
GOLHIP_ERR_RCCL within its deadline (golhip_set_comm_timeout), naming the pending transfer,
instead of hanging the run (the reference has no such bound: a dead server stalls
Broker.Publish forever, broker/broker.go:58-84).

Each case runs in a FRESH process under its own time limit, so a failure of the deadline itself
ends in a killed child, not a hung test session:
  * stalled rank: the ring-of-one hook GOLHIP_RING_SELF=2 ends every step in a 20 s stall of the
    compute stream, so the sync waits past its deadline;
  * init: rank 0 of a 2-rank communicator whose rank 1 never joins -- ncclCommInitRankConfig
    (non-blocking) never finishes its set-up, and is aborted (nothing of it runs on the device).
"""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu

CHILD = r"""
import json, os, sys, time
sys.path.insert(0, sys.argv[1])
import torch  # one HIP runtime per process (golhip.py)
import golhip
case, timeout_ms = sys.argv[2], int(sys.argv[3])
out = {"case": case}
e = None
try:
    if case == "stall":
        # created under the default deadline (a first RCCL set-up in a fresh process can take
        # seconds), then the handle's own deadline
        e = golhip.Engine(640, 64, k=4, rank=0, world_size=1, device=0)
        e.set_comm_timeout(timeout_ms)
        out["halo_rows"] = e.info.halo_rows
        e.init_random(5)
        t0 = time.perf_counter()
        e.step(9)
        e.sync()
        out["completed"] = True
    else:
        golhip.set_default_comm_timeout(timeout_ms)
        t0 = time.perf_counter()
        golhip.Engine(640, 64, k=4, rank=0, world_size=2, device=0, nccl_id=golhip.nccl_unique_id())
        out["completed"] = True
except golhip.GolHipError as err:
    out["code"] = err.code
    out["msg"] = str(err)
out["seconds"] = time.perf_counter() - t0
t1 = time.perf_counter()
if case == "stall" and "code" in out and e is not None:
    # the handle refuses further device work with the same error, and destroys without waiting
    # for the stalled stream
    try:
        e.step(1)
        e.sync()
        out["after"] = "ok"
    except golhip.GolHipError as err:
        out["after"] = err.code
    e.close()
out["teardown_seconds"] = time.perf_counter() - t1
print(json.dumps(out), flush=True)
os._exit(0)  # as bench.py after an RCCL failure: no interpreter teardown behind a stalled stream
"""


def run_child(case, timeout_ms, ring_self=None):
    env = dict(os.environ)
    env.pop("GOLHIP_RING_SELF", None)
    if ring_self:
        env["GOLHIP_RING_SELF"] = ring_self
    p = subprocess.run(["timeout", "-k", "10", "150", sys.executable, "-c", CHILD, str(PKG), case,
                        str(timeout_ms)], env=env, capture_output=True, text=True, timeout=200)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    return json.loads(lines[-1])


def test_stalled_rank_fails_at_the_deadline(golhip):
    """GOLHIP_RING_SELF=2: every step's work ends in a 20 s stall of the compute stream (a rank
    whose device work does not finish in time).  The sync polls against the 3 s deadline and
    returns ERR_RCCL at the deadline -- not after the stall -- naming the last exchange; the handle
    refuses further work; destroy does not wait for the stalled stream.  Nothing RCCL is queued
    behind the stall, and the communicator is not aborted after its set-up (an abort with RCCL
    work queued behind a stall faulted the GPU: profiles/r04/r04d_failfast_abort_hooks.log)."""
    timeout_ms = 3000
    out = run_child("stall", timeout_ms, ring_self="2")
    print(json.dumps(out))
    assert out.get("halo_rows") == 4, out
    assert not out.get("completed"), out
    assert out["code"] == golhip.ERR_RCCL, out
    assert timeout_ms / 1e3 * 0.9 <= out["seconds"] < timeout_ms / 1e3 + 10, out
    msg = out["msg"]
    # golhip_last_error names the rank, the pending exchange, its peers, K and the byte count
    assert "rank 0 of 1" in msg and "did not complete within 3000 ms" in msg, msg
    assert "K = 1" in msg and "bytes" in msg and "<- rank 0" in msg and "-> rank 0" in msg, msg
    assert "end the process" in msg, msg
    assert out["after"] == golhip.ERR_RCCL, out
    assert out["teardown_seconds"] < timeout_ms / 1e3 + 10, out


def test_peer_that_never_joins_fails_fast_at_create(golhip):
    timeout_ms = 3000
    out = run_child("init", timeout_ms)
    print(json.dumps(out))
    assert not out.get("completed"), out
    assert out["code"] == golhip.ERR_RCCL, out
    assert out["seconds"] < timeout_ms / 1e3 + 30, out
    assert "rank 0 of 2" in out["msg"] and "ncclCommInitRankConfig" in out["msg"], out["msg"]


def test_ring_of_one_still_exchanges_with_a_deadline(golhip, oracle, monkeypatch):
    """The non-blocking communicator and the polled waits leave the working path bit-exact: the
    ring of one under a short deadline, every count and the board equal to the oracle."""
    monkeypatch.setenv("GOLHIP_RING_SELF", "1")
    w, h, k = 640, 77, 8
    words = oracle.init_random(w, h, seed=77)
    with golhip.Engine(w, h, k=k, rank=0, world_size=1, device=0) as e:
        e.set_comm_timeout(5000)
        e.load_words(words)
        counts = e.step(3 * k + 5, counts=True)
        got = e.store_words()
    ref = words.copy()
    ref_counts = oracle.packed_run_words(ref, 3 * k + 5)
    assert (got == ref).all()
    assert (counts.astype("int64") == ref_counts).all()
