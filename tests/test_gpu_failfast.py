"""RCCL fail-fast on one GPU: a rank-mode engine whose RCCL work cannot complete returns
GOLHIP_ERR_RCCL within its deadline (golhip_set_comm_timeout), naming the pending transfer,
instead of hanging the run (the reference has no such bound: a dead server stalls
Broker.Publish forever, broker/broker.go:58-84).

Each case runs in FRESH processes under their own time limits, so a failure of the deadline itself
ends in a killed child, not a hung test session.  Fault injection is in the tuning library's engine
hooks only (csrc/tuning/engine_tuning.hip, GOLHIP_FAULT), loaded here from lib_faults (the
production objects + those hooks); the engine code under test is the production code.
  * stuck receive: TWO real RCCL ranks on this one GPU (a distinct NCCL_HOSTID per rank makes RCCL
    build a 2-rank communicator over its network transport instead of refusing "Duplicate GPU");
    rank 1 leaves the first send of every halo exchange out of its RCCL group (GOLHIP_FAULT=
    skip_send), so rank 0's receive never completes -- the path a real multi-GPU hang takes: an
    RCCL kernel spinning on an unmatched receive.  Both ranks must fail at the deadline with the
    first incomplete exchange named, golhip_comm_abort (rank 0) / golhip_destroy (rank 1) must
    release the spinning RCCL kernels (ncclCommAbort), the streams must drain and both processes
    exit 0 (round 4 claimed an abort with RCCL work queued faults the GPU; measured here, it does
    not: profiles/r05/r05d_stuck_rccl_receive_abort.log);
  * stalled rank: the ring of one (GOLHIP_RING_SELF=1) whose every step ends in a 20 s stall of the
    compute stream (GOLHIP_FAULT=stall), so the sync waits past its deadline;
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
        e = golhip.Engine(640, 64, k=4, rank=0, world_size=1, device=0, lib=golhip.fault_library())
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

# One rank of a real 2-rank RCCL communicator on this GPU (argv: pkg rank timeout_ms idfile).
CHILD_RANK = r"""
import faulthandler, json, os, sys, time
pkg, rank, timeout_ms, idfile = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
sys.path.insert(0, pkg)
T0 = time.perf_counter()
def log(msg):  # progress on stderr: where a killed child was
    print(f"[rank {rank} +{time.perf_counter() - T0:.2f}s] {msg}", file=sys.stderr, flush=True)
faulthandler.dump_traceback_later(75, exit=False)  # the Python stack of a child about to be killed
import torch  # one HIP runtime per process (golhip.py)
import golhip
out = {"rank": rank}
L = golhip.fault_library()
if rank == 0:
    nid = golhip.nccl_unique_id()  # rank 0 hosts the bootstrap root
    with open(idfile + ".tmp", "wb") as f:
        f.write(nid)
    os.rename(idfile + ".tmp", idfile)
else:
    t = time.time()
    while not os.path.exists(idfile) and time.time() - t < 60:
        time.sleep(0.05)
    nid = open(idfile, "rb").read()
t0 = time.perf_counter()
# created under the default deadline (the set-up of a fresh communicator can take seconds), then
# the handle's own deadline
log("creating")
e = golhip.Engine(640, 128, k=4, rank=rank, world_size=2, device=0, nccl_id=nid, lib=L)
out["create_seconds"] = time.perf_counter() - t0
e.set_comm_timeout(timeout_ms)
e.init_random(5)
log("stepping")
t0 = time.perf_counter()
try:
    out["counts"] = [int(c) for c in e.step(9, counts=True)]
    e.sync()
    out["completed"] = True
except golhip.GolHipError as err:
    out["code"] = err.code
    out["msg"] = str(err)
    out["last_call"] = e.last_call
out["seconds"] = time.perf_counter() - t0
log(f"step returned: {out.get('code', 'ok')}: {out.get('msg', '')}")
print(json.dumps(out), flush=True)  # the result so far, in case the teardown below is killed
if "code" in out and os.environ.get("GOLHIP_TEST_ABORT", "1") == "1":
    t1 = time.perf_counter()
    if rank == 0:  # explicitly; rank 1 leaves it to golhip_destroy, which aborts a failed communicator
        log("golhip_comm_abort")
        e.comm_abort()  # ncclCommAbort: RCCL aborts its operations still running on the device
    log("golhip_destroy")
    e.close()  # aborts a failed communicator, drains the streams (bounded by the deadline), frees
    log("closed")
    out["abort_close_seconds"] = time.perf_counter() - t1
    out["drained"] = True
    print(json.dumps(out), flush=True)
os._exit(0)
"""


def run_child(case, timeout_ms, fault=None):
    env = dict(os.environ)
    env.pop("GOLHIP_RING_SELF", None)
    env.pop("GOLHIP_FAULT", None)
    if fault:
        env["GOLHIP_RING_SELF"] = "1"
        env["GOLHIP_FAULT"] = fault
    p = subprocess.run(["timeout", "-k", "10", "150", sys.executable, "-c", CHILD, str(PKG), case,
                        str(timeout_ms)], env=env, capture_output=True, text=True, timeout=200)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    return json.loads(lines[-1])


def rccl_shared_gpu_env(rank: int) -> dict:
    """Environment of one rank of a multi-rank RCCL communicator on this single GPU: a distinct
    NCCL_HOSTID per rank (RCCL then treats the ranks as separate hosts and connects them through
    its network transport, over loopback)."""
    env = dict(os.environ)
    for k in ("GOLHIP_RING_SELF", "GOLHIP_FAULT"):
        env.pop(k, None)
    env["NCCL_HOSTID"] = f"golhip-test-rank{rank}"
    env.setdefault("NCCL_SOCKET_IFNAME", "lo")
    return env


@pytest.mark.timeout(240)
def test_stuck_rccl_receive_fails_at_the_deadline_and_aborts(golhip, tmp_path):
    timeout_ms = 3000
    idfile = str(tmp_path / "nccl.id")
    procs = []
    for rank in (0, 1):
        env = rccl_shared_gpu_env(rank)
        if rank == 1:
            env["GOLHIP_FAULT"] = "skip_send"
        procs.append(subprocess.Popen(["timeout", "-k", "10", "90", sys.executable, "-c", CHILD_RANK, str(PKG),
                                       str(rank), str(timeout_ms), idfile], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    res, outs = [], []
    for p in procs:
        so, se = p.communicate(timeout=200)
        outs.append((p.returncode, so, se))
    for rc, so, se in outs:  # both ranks' logs in any failure message
        print(f"rc={rc}\n{so[-3000:]}\n{se[-6000:]}")
    for rc, so, se in outs:
        lines = [ln for ln in so.splitlines() if ln.startswith("{")]
        assert rc == 0 and lines, (rc, so[-2000:], se[-3000:])
        res.append(json.loads(lines[-1]))
    print(json.dumps(res))
    for r in res:
        # every rank fails at its deadline (with the modelled allowance for its queued work) --
        # not after the 150 s child limit, and without completing the call
        assert not r.get("completed"), r
        assert r["code"] == golhip.ERR_RCCL, r
        assert r["seconds"] < timeout_ms / 1e3 + 15, r
        msg = r["msg"]
        assert f"rank {r['rank']} of 2" in msg and "end the process" in msg, msg
        assert "golhip_comm_abort" in msg, msg
        # the abort released the spinning RCCL kernels: the streams drained and the strips were
        # freed within the deadline
        assert r["drained"] and r["abort_close_seconds"] < timeout_ms / 1e3 + 10, r
    # rank 0 waits for a halo that never comes: its error names the first incomplete RCCL
    # operation -- an exchange, not merely the last operation queued (the count all-reduce)
    assert "the first incomplete of" in res[0]["msg"], res[0]["msg"]
    assert "halo exchange #" in res[0]["msg"] and "<- rank 1" in res[0]["msg"], res[0]["msg"]


def test_stalled_rank_fails_at_the_deadline(golhip):
    """GOLHIP_FAULT=stall: every step's work ends in a 20 s stall of the compute stream (a rank
    whose device work does not finish in time).  The sync polls against the 3 s deadline and
    returns ERR_RCCL at the deadline -- not after the stall -- naming the last exchange; the handle
    refuses further work; destroy does not wait for the stalled stream."""
    timeout_ms = 3000
    out = run_child("stall", timeout_ms, fault="stall")
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


CHILD_SLAB = r"""
import hashlib, json, os, sys, time
sys.path.insert(0, sys.argv[1])
import torch  # one HIP runtime per process (golhip.py)
import numpy as np
import golhip
out = {}
with golhip.Engine(4096, 4096, k=16, lib=golhip.fault_library()) as e:  # GOLHIP_FAULT=slab_stall
    e.init_random(11)
    e.step(32)
    before = hashlib.sha256(e.store_words().tobytes()).hexdigest()
    t0 = time.perf_counter()
    try:
        e.step_persistent(600)
        out["raised"] = False
    except golhip.GolHipError as err:
        out["raised"], out["code"], out["msg"] = True, err.code, str(err)
    out["seconds"] = time.perf_counter() - t0
    out["turn"] = e.turn
    out["board_unchanged"] = hashlib.sha256(e.store_words().tobytes()).hexdigest() == before
    # the handle keeps working: golhip_step from the restored board
    c = e.step(48, counts=True)
    out["after_counts"] = [int(x) for x in c[-3:]]
    out["after_turn"] = e.turn
    out["after_digest"] = hashlib.sha256(e.store_words().tobytes()).hexdigest()
with golhip.Engine(4096, 4096, k=16) as e:  # the production library, same board, no fault
    e.init_random(11)
    e.step(32 + 48)
    out["ref_digest"] = hashlib.sha256(e.store_words().tobytes()).hexdigest()
print(json.dumps(out), flush=True)
"""


def test_persistent_slab_timeout_restores_board():
    """golhip_step_persistent when a slab never signals (GOLHIP_FAULT=slab_stall, tuning library:
    slab 0 skips its first block counter, as a slab that is not resident would): its neighbours give
    up after 200 ms, every later window leaves at entry, and the call returns GOLHIP_ERR_STATE with
    the board and turn restored to where the call started -- never a half-advanced board (the
    reference's Publish gate never leaves the world half-written, broker/broker.go:109-120).  The
    handle keeps working: golhip_step from the restored board ends where an untouched run does."""
    env = dict(os.environ, GOLHIP_FAULT="slab_stall")
    p = subprocess.run(["timeout", "-k", "10", "120", sys.executable, "-c", CHILD_SLAB, str(PKG)],
                       env=env, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["raised"] and out["code"] == -7, out
    assert "restored to turn 32" in out["msg"], out
    assert out["turn"] == 32 and out["board_unchanged"], out
    assert out["seconds"] < 30, out
    assert out["after_turn"] == 80 and out["after_digest"] == out["ref_digest"], out


def test_fault_library_selectors_smoke(golhip, oracle, monkeypatch):
    """The round-end suite's tuning smoke: the engine hooks (csrc/tuning/engine_tuning.hip) over the
    production kernels, from lib_faults -- GOLHIP_SLAB forces another production slab shape and
    GOLHIP_FIXED_K the launch depth, read at create -- bit-exact against the oracle and against the
    production library's automatic choice."""
    import numpy as np

    words = oracle.init_random(2048, 2048, seed=13)
    L = golhip.fault_library()
    monkeypatch.setenv("GOLHIP_SLAB", "91207")  # gol_slab2 12 x 7 (NC 9)
    monkeypatch.setenv("GOLHIP_FIXED_K", "1")
    with golhip.Engine(2048, 2048, k=16, lib=L) as e:
        assert e.launch_kind(16) == ("slab", 91207), e.launch_kind(16)
        e.load_words(words)
        c = e.step(100, counts=True)
        forced = e.store_words()
    monkeypatch.delenv("GOLHIP_SLAB")
    monkeypatch.delenv("GOLHIP_FIXED_K")
    with golhip.Engine(2048, 2048, k=16) as e:
        assert e.launch_kind(16) != ("slab", 91207)
        e.load_words(words)
        c2 = e.step(100, counts=True)
        auto = e.store_words()
    ref = words.copy()
    exp = oracle.packed_run_words(ref, 100)
    assert np.array_equal(forced, ref) and np.array_equal(auto, ref)
    assert np.array_equal(c.astype(np.int64), exp) and np.array_equal(c2.astype(np.int64), exp)
