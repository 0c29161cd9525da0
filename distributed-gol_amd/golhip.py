"""ctypes binding of libgolhip (include/golhip.h) -- the Python side of the drop-in boundary.

This is plumbing: every call goes straight to the C ABI of ``lib/libgolhip.so``, the gfx950
engine that replaces the reference's ``Broker.Publish`` -> ``GolOP.Work`` path
(broker/broker.go:157-180, server/server.go:77-107).  There is no CPU fallback: if the
library or a gfx950 device is missing, calls raise ``GolHipError``.

``import torch`` (when installed) happens before the library is loaded so that one process
never holds two HIP runtimes: torch's bundled ``libamdhip64.so`` and ``librccl.so`` carry the
same SONAMEs as /opt/rocm's, so loading torch first makes libgolhip bind to torch's copies.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

try:  # single HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the binding itself
    torch = None

HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("GOLHIP_LIB", HERE / "lib" / "libgolhip.so"))
# The tuning build of the same sources (-DGOLHIP_TUNING, distributed-gol_amd/Makefile): the
# production kernels plus the measured-and-rejected variants, the level-split / register-tile
# kernels and the A/B environment selectors.  Only tests of those kernels and tuning scripts load it.
TUNING_LIB_PATH = HERE / "lib_tuning" / "libgolhip.so"
FAULTS_LIB_PATH = HERE / "lib_faults" / "libgolhip.so"

OK = 0
ERR_ARG, ERR_HIP, ERR_OOM, ERR_CAP, ERR_RCCL, ERR_NODEV, ERR_STATE = -1, -2, -3, -4, -5, -6, -7
NCCL_ID_BYTES = 128
DENSITY_HALF = 0x80000000
HANDOFF_FENCED, HANDOFF_SC1 = 0, 1  # golhip_set_persistent_handoff

# Every symbol include/golhip.h declares (tests/test_boundary.py checks the .so exports them).
EXPORTS = [
    "golhip_version", "golhip_strerror", "golhip_device_count", "golhip_strip_bounds",
    "golhip_halo_plan",
    "golhip_create", "golhip_create_strips", "golhip_nccl_unique_id", "golhip_create_rank",
    "golhip_comm_abort", "golhip_edge_wait", "golhip_set_activity", "golhip_activity_stats",
    "golhip_set_board_kernel", "golhip_step_persistent", "golhip_set_persistent_limit", "golhip_set_persistent_handoff",
    "golhip_create_rank_host", "golhip_destroy",
    "golhip_last_error", "golhip_get_info", "golhip_load_bytes", "golhip_init_random",
    "golhip_store_bytes", "golhip_store_words", "golhip_load_words", "golhip_step",
    "golhip_alive_count", "golhip_alive_cells", "golhip_flips", "golhip_turn",
    "golhip_set_turn", "golhip_set_k", "golhip_set_band_rows", "golhip_set_tail_bands", "golhip_sync", "golhip_timing",
    "golhip_set_graphs", "golhip_set_count_window", "golhip_set_comm_timeout",
    "golhip_kernel_time", "golhip_launch_plan", "golhip_launch_kind", "golhip_launch_kind_counts", "golhip_set_fixed_k", "golhip_track_flips",
    "golhip_step_flips", "golhip_flips_ring_capacity", "golhip_flips_fetch",
    "golhip_step_flips_rows", "golhip_flips_fetch_rows",
    "golhip_checkpoint_save", "golhip_checkpoint_load", "golhip_checkpoint_info",
]


class GolHipError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"golhip error {code}: {msg}")
        self.code = code


class Xfer(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("peer", ctypes.c_int32), ("row", ctypes.c_int64),
                ("nrows", ctypes.c_int64)]


EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(Xfer), ctypes.c_int,
                               ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                ctypes.c_size_t)


class HostCommStruct(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("exchange", EXCHANGE_FN), ("allreduce_u64", ALLREDUCE_FN)]


class GlooHostComm:
    """golhip_host_comm over a torch.distributed (gloo) process group: the halo exchange as
    isend/irecv of the engine's pinned host buffers in the plan's order (gloo matches the i-th send
    to a peer with that peer's i-th receive, as RCCL does inside a group), the count reduction as
    one all_reduce.  The transport for ranks that cannot use RCCL peers (several ranks on one GPU
    in the rank-mode tests: RCCL refuses a duplicate GPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self._dist, self._group = dist, group
        self._exchange = EXCHANGE_FN(self._do_exchange)
        self._allreduce = ALLREDUCE_FN(self._do_allreduce)
        self.struct = HostCommStruct(None, self._exchange, self._allreduce)
        self.exchanges = 0  # exchange calls seen (tests count them)
        self.reduced = []   # sizes of the count reductions seen

    def _do_exchange(self, _ctx, xfers, n, bufs, nbytes):
        try:
            reqs = []
            for i in range(n):
                x = xfers[i]
                arr = np.ctypeslib.as_array(ctypes.cast(bufs[i], ctypes.POINTER(ctypes.c_uint8)),
                                            shape=(nbytes,))
                t = torch.from_numpy(arr)
                op = self._dist.isend if x.kind == 0 else self._dist.irecv
                reqs.append(op(t, x.peer, group=self._group))
            for r in reqs:
                r.wait()
            self.exchanges += 1
            return 0
        except Exception as e:  # pragma: no cover - reported through the C ABI's error path
            print(f"golhip host transport: exchange failed: {e!r}", flush=True)
            return -1

    def _do_allreduce(self, _ctx, vals, n):
        try:
            arr = np.ctypeslib.as_array(vals, shape=(n,)).view(np.int64)
            t = torch.from_numpy(arr.copy())
            self._dist.all_reduce(t, group=self._group)  # sum; uint64 wraps like int64
            arr[:] = t.numpy()
            self.reduced.append(int(n))
            return 0
        except Exception as e:  # pragma: no cover
            print(f"golhip host transport: all_reduce failed: {e!r}", flush=True)
            return -1


class Info(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int64), ("height", ctypes.c_int64), ("torus_width", ctypes.c_int64),
        ("y0", ctypes.c_int64), ("rows", ctypes.c_int64), ("rank", ctypes.c_int32),
        ("world_size", ctypes.c_int32), ("nshards", ctypes.c_int32), ("k", ctypes.c_int32),
        ("halo_rows", ctypes.c_int32), ("band_rows", ctypes.c_int32),
    ]


_lib = None
_libs: dict[str, ctypes.CDLL] = {}


def load_library(path: Path | str | None = None) -> ctypes.CDLL:
    """Load libgolhip.so (raises if it was not built: no fallback).  path=None: the default library
    (GOLHIP_LIB, an alternative build for A/B experiments, else the in-tree production build);
    another path loads that build beside it (its own handle namespace, RTLD_LOCAL)."""
    global _lib
    if path is None and _lib is not None:
        return _lib
    # GOLHIP_LIB: an alternative build of the same library (A/B experiments); default in-tree
    p = Path(path) if path else Path(os.environ.get("GOLHIP_LIB", str(LIB_PATH)))
    key = str(p.resolve()) if p.exists() else str(p)
    if key in _libs:
        if path is None:
            _lib = _libs[key]
        return _libs[key]
    if not p.exists():
        raise GolHipError(ERR_NODEV, f"{p} not built (run __graft_entry__.build())")
    L = ctypes.CDLL(str(p))
    H = ctypes.c_void_p
    i64, i32, u64p = ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)
    i64p = ctypes.POINTER(ctypes.c_int64)
    sig = {
        "golhip_version": ([], i32),
        "golhip_strerror": ([i32], ctypes.c_char_p),
        "golhip_device_count": ([ctypes.POINTER(i32)], i32),
        "golhip_strip_bounds": ([i64, i32, i32, i64p, i64p], i32),
        "golhip_halo_plan": ([i64, i32, i32, i32, ctypes.POINTER(Xfer)], i32),
        "golhip_create": ([i32, i32, i32, i32, ctypes.POINTER(H)], i32),
        "golhip_create_strips": ([i32, i32, i32, i32, i32, ctypes.POINTER(H)], i32),
        "golhip_nccl_unique_id": ([ctypes.c_char_p], i32),
        "golhip_create_rank": ([i32, i32, i32, i32, i32, i32, ctypes.c_char_p, ctypes.POINTER(H)], i32),
        "golhip_create_rank_host": ([i32, i32, i32, i32, i32, i32, ctypes.POINTER(HostCommStruct),
                                     ctypes.POINTER(H)], i32),
        "golhip_destroy": ([H], i32),
        "golhip_last_error": ([H], ctypes.c_char_p),
        "golhip_get_info": ([H, ctypes.POINTER(Info)], i32),
        "golhip_load_bytes": ([H, ctypes.c_void_p, ctypes.c_size_t], i32),
        "golhip_init_random": ([H, ctypes.c_uint64, ctypes.c_uint32], i32),
        "golhip_store_bytes": ([H, ctypes.c_void_p, ctypes.c_size_t], i32),
        "golhip_store_words": ([H, ctypes.c_void_p], i32),
        "golhip_load_words": ([H, ctypes.c_void_p], i32),
        "golhip_step": ([H, i64, ctypes.c_void_p], i32),
        "golhip_step_persistent": ([H, i64, ctypes.c_void_p], i32),
        "golhip_set_persistent_limit": ([H, i32], i32),
        "golhip_set_persistent_handoff": ([H, i32], i32),
        "golhip_alive_count": ([H, u64p], i32),
        "golhip_alive_cells": ([H, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)], i32),
        "golhip_flips": ([H, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)], i32),
        "golhip_turn": ([H, i64p], i32),
        "golhip_set_turn": ([H, i64], i32),
        "golhip_set_k": ([H, i32], i32),
        "golhip_set_band_rows": ([H, i32], i32),
        "golhip_set_tail_bands": ([H, i32, i32], i32),
        "golhip_set_fixed_k": ([H, i32], i32),
        "golhip_track_flips": ([H, i32], i32),
        "golhip_checkpoint_save": ([H, ctypes.c_char_p], i32),
        "golhip_checkpoint_load": ([H, ctypes.c_char_p], i32),
        "golhip_checkpoint_info": ([ctypes.c_char_p, i64p, i64p, i64p], i32),
        "golhip_step_flips": ([H, i64, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                               ctypes.c_void_p, ctypes.c_void_p], i32),
        "golhip_flips_ring_capacity": ([H, i64p], i32),
        "golhip_flips_fetch": ([H, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                ctypes.c_void_p], i32),
        "golhip_step_flips_rows": ([H, i64, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p, ctypes.c_void_p], i32),
        "golhip_flips_fetch_rows": ([H, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.c_void_p], i32),
        "golhip_sync": ([H], i32),
        "golhip_set_graphs": ([H, i32], i32),
        "golhip_set_count_window": ([H, i32], i32),
        "golhip_set_comm_timeout": ([H, i64], i32),
        "golhip_comm_abort": ([H], i32),
        "golhip_timing": ([H, i32], i32),
        "golhip_kernel_time": ([H, ctypes.POINTER(ctypes.c_double), i64p, i64p], i32),
        "golhip_edge_wait": ([H, ctypes.POINTER(ctypes.c_double), i64p], i32),
        "golhip_set_activity": ([H, i32], i32),
        "golhip_set_board_kernel": ([H, i32], i32),
        "golhip_activity_stats": ([H, i64p, i64p], i32),
        "golhip_launch_plan": ([i64, i64, i32, i32, i64, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.POINTER(ctypes.c_size_t)], i32),
        "golhip_launch_kind": ([H, i32, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], i32),
        "golhip_launch_kind_counts": ([H, i32, i32, ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_int)], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _libs[key] = L
    if path is None:
        _lib = L
    if _default_comm_timeout_ms is not None:  # set_default_comm_timeout reaches every library
        L.golhip_set_comm_timeout(None, _default_comm_timeout_ms)
    return L


def tuning_library() -> ctypes.CDLL:
    """The tuning build (lib_tuning/libgolhip.so): pass it as Engine(..., lib=tuning_library()) to
    run a non-production kernel (GOLHIP_VARIANT / GOLHIP_SPLIT / GOLHIP_TILE / GOLHIP_SLAB ...).
    Built here; pushed to a GPU box only for the runs that load it (.gpurunignore)."""
    return load_library(TUNING_LIB_PATH)


def fault_library() -> ctypes.CDLL:
    """The production kernels + the tuning library's engine hooks (lib_faults/libgolhip.so): fault
    injection (GOLHIP_FAULT) and the A/B selectors over the production kernels -- what the fail-fast
    tests load."""
    return load_library(FAULTS_LIB_PATH)


_default_comm_timeout_ms: int | None = None


def set_default_comm_timeout(ms: int, lib: ctypes.CDLL | None = None) -> None:
    """golhip_set_comm_timeout(NULL, ms): the RCCL deadline of engines created from now on, in every
    library loaded now or later (an Engine(..., lib=tuning_library()) in rank mode included), or
    only in `lib` when given."""
    global _default_comm_timeout_ms
    if int(ms) <= 0:
        raise GolHipError(ERR_ARG, "set_comm_timeout: invalid argument")
    if lib is not None:
        libs = [lib]
    else:
        _default_comm_timeout_ms = int(ms)
        libs = list(_libs.values()) or [load_library()]
    for L in libs:
        rc = L.golhip_set_comm_timeout(None, int(ms))
        if rc != OK:
            raise GolHipError(rc, "set_comm_timeout: invalid argument")


class _CallLog:
    """The library seen through an engine: records the name of the last C ABI function called
    (Engine.last_call), so a failed or stuck multi-rank run can say where it was."""

    def __init__(self, lib: ctypes.CDLL, owner: "Engine"):
        self._lib, self._owner = lib, owner

    _QUIET = ("golhip_last_error", "golhip_strerror", "golhip_get_info")

    def __getattr__(self, name):
        if name not in self._QUIET:
            self._owner.last_call = name
        return getattr(self._lib, name)


def parse_rle(text: str) -> np.ndarray:
    """Run-length-encoded Life pattern (the standard .rle format) -> 0/255 uint8 (h, w)."""
    lines = [ln.strip() for ln in text.splitlines() if ln.strip() and not ln.startswith("#")]
    header, body = lines[0], "".join(lines[1:])
    dims = dict(kv.split("=") for kv in header.replace(" ", "").split(",")[:2])
    w, h = int(dims["x"]), int(dims["y"])
    out = np.zeros((h, w), dtype=np.uint8)
    x = y = 0
    run = ""
    for ch in body:
        if ch.isdigit():
            run += ch
            continue
        n = int(run) if run else 1
        run = ""
        if ch == "b":
            x += n
        elif ch == "o":
            out[y, x:x + n] = 255
            x += n
        elif ch == "$":
            y += n
            x = 0
        elif ch == "!":
            break
    return out


def place(board: np.ndarray, pattern: np.ndarray, x: int, y: int) -> None:
    """Stamp a pattern at (x, y) on a torus board (in place)."""
    h, w = pattern.shape
    H, W = board.shape
    ys = (np.arange(h) + y) % H
    xs = (np.arange(w) + x) % W
    board[np.ix_(ys, xs)] |= pattern


def pinned_empty(shape, dtype) -> np.ndarray:
    """A page-locked host array when a GPU is present (device -> host copies into it are one DMA at
    the full PCIe rate instead of going through the runtime's pageable staging), else a plain one.
    The array keeps its torch storage alive."""
    if torch is not None and torch.cuda.is_available():
        n = int(np.prod(shape)) * np.dtype(dtype).itemsize
        t = torch.empty(max(n, 1), dtype=torch.uint8, pin_memory=True)
        a = t.numpy()[:n].view(dtype).reshape(shape)
        return a
    return np.zeros(shape, dtype=dtype)


def device_count() -> int:
    n = ctypes.c_int(0)
    load_library().golhip_device_count(ctypes.byref(n))
    return n.value


def strip_bounds(height: int, world_size: int, rank: int) -> tuple[int, int]:
    """Rows [y0, y0+rows) of `rank` (pure host arithmetic, no device)."""
    y0, rows = ctypes.c_int64(), ctypes.c_int64()
    rc = load_library().golhip_strip_bounds(height, world_size, rank, ctypes.byref(y0), ctypes.byref(rows))
    if rc != OK:
        raise GolHipError(rc, "strip_bounds: invalid arguments")
    return y0.value, rows.value


def halo_plan(height: int, world_size: int, rank: int, k: int) -> list[tuple[str, int, int, int]]:
    """The engine's 4 halo transfers for `rank`, in issue order: (send|recv, peer, row, nrows)."""
    arr = (Xfer * 4)()
    rc = load_library().golhip_halo_plan(height, world_size, rank, k, arr)
    if rc != OK:
        raise GolHipError(rc, "halo_plan: invalid arguments")
    return [("send" if x.kind == 0 else "recv", x.peer, x.row, x.nrows) for x in arr]


def launch_plan(width: int, height: int, k: int, turns: int, strips: int = 1) -> list[int]:
    """The launch depths golhip_step(turns) runs (pure host arithmetic, no device): > 0 one
    stencil launch of that depth, < 0 one graph replay of that many generations."""
    L = load_library()
    n = ctypes.c_size_t(0)
    rc = L.golhip_launch_plan(width, height, strips, k, turns, None, 0, ctypes.byref(n))
    if rc != OK:
        raise GolHipError(rc, "launch_plan: invalid arguments")
    out = np.zeros(max(n.value, 1), dtype=np.int32)
    rc = L.golhip_launch_plan(width, height, strips, k, turns, out.ctypes.data, n.value, ctypes.byref(n))
    if rc != OK:
        raise GolHipError(rc, "launch_plan failed")
    return [int(x) for x in out[: n.value]]


def checkpoint_info(path) -> tuple[int, int, int]:
    """(width, height, turn) of a checkpoint file (pure host, no device)."""
    w, h, t = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    rc = load_library().golhip_checkpoint_info(str(path).encode(), ctypes.byref(w), ctypes.byref(h),
                                               ctypes.byref(t))
    if rc != OK:
        raise GolHipError(rc, f"{path}: not a golhip checkpoint")
    return w.value, h.value, t.value


def nccl_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(NCCL_ID_BYTES)
    rc = load_library().golhip_nccl_unique_id(buf)
    if rc != OK:
        raise GolHipError(rc, "ncclGetUniqueId failed")
    return buf.raw


class Engine:
    """One libgolhip handle.  Mirrors the broker's role: the board lives on the GPU(s)."""

    def __init__(self, width: int, height: int, ngpus: int = 1, k: int = 1, *, rank: int | None = None,
                 world_size: int = 1, device: int = 0, nccl_id: bytes | None = None,
                 strips: int | None = None, host_comm: GlooHostComm | None = None,
                 lib: ctypes.CDLL | None = None):
        self.last_call = "golhip_create"
        L = _CallLog(lib if lib is not None else load_library(), self)
        self._L = L
        self._h = ctypes.c_void_p()
        self.host_comm = host_comm  # keeps the ctypes callbacks alive with the handle
        if host_comm is not None:
            rc = L.golhip_create_rank_host(width, height, rank or 0, world_size, device, k,
                                           ctypes.byref(host_comm.struct), ctypes.byref(self._h))
        elif strips is not None:
            rc = L.golhip_create_strips(width, height, strips, ngpus, k, ctypes.byref(self._h))
        elif rank is None:
            rc = L.golhip_create(width, height, ngpus, k, ctypes.byref(self._h))
        else:
            rc = L.golhip_create_rank(width, height, rank, world_size, device, k, nccl_id,
                                      ctypes.byref(self._h))
        if rc != OK:
            why = L.golhip_last_error(None).decode() or L.golhip_strerror(rc).decode()
            raise GolHipError(rc, why)
        self.info = self.get_info()

    # -- plumbing
    def _check(self, rc: int) -> int:
        if rc != OK:
            raise GolHipError(rc, self._L.golhip_last_error(self._h).decode() or
                              self._L.golhip_strerror(rc).decode())
        return rc

    def close(self):
        if self._h:
            self._L.golhip_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def get_info(self) -> Info:
        info = Info()
        self._check(self._L.golhip_get_info(self._h, ctypes.byref(info)))
        return info

    # -- board in/out
    def load(self, cells: np.ndarray):
        cells = np.ascontiguousarray(cells, dtype=np.uint8)
        assert cells.shape == (self.info.rows, self.info.width), cells.shape
        self._check(self._L.golhip_load_bytes(self._h, cells.ctypes.data, cells.strides[0]))

    def init_random(self, seed: int, density_q32: int = DENSITY_HALF):
        self._check(self._L.golhip_init_random(self._h, seed, density_q32))

    def store(self) -> np.ndarray:
        out = np.empty((self.info.rows, self.info.width), dtype=np.uint8)
        self._check(self._L.golhip_store_bytes(self._h, out.ctypes.data, out.strides[0]))
        return out

    def store_words(self) -> np.ndarray:
        out = np.empty((self.info.rows, self.info.width // 64), dtype=np.uint64)
        self._check(self._L.golhip_store_words(self._h, out.ctypes.data))
        return out

    def load_words(self, words: np.ndarray):
        words = np.ascontiguousarray(words, dtype=np.uint64)
        assert words.shape == (self.info.rows, self.info.width // 64)
        self._check(self._L.golhip_load_words(self._h, words.ctypes.data))

    # -- hot path
    def step(self, turns: int, counts: bool = False) -> np.ndarray | None:
        if counts:
            out = np.zeros(max(turns, 1), dtype=np.uint64)
            self._check(self._L.golhip_step(self._h, turns, out.ctypes.data))
            return out[:turns]
        self._check(self._L.golhip_step(self._h, turns, None))
        return None

    def step_persistent(self, turns: int) -> np.ndarray:
        """golhip_step_persistent: `turns` turns with every count, one persistent-slab launch per
        count window (opt-in; configs[1] / configs[4]-like boards).  Refuses (GOLHIP_ERR_STATE,
        board unchanged) when the slabs cannot all be resident; restores the board on a timeout."""
        out = np.zeros(max(turns, 1), dtype=np.uint64)
        self._check(self._L.golhip_step_persistent(self._h, turns, out.ctypes.data))
        return out[:turns]

    def set_persistent_handoff(self, mode: int) -> None:
        """golhip_set_persistent_handoff: HANDOFF_FENCED (default) or HANDOFF_SC1 (measured form)."""
        self._check(self._L.golhip_set_persistent_handoff(self._h, mode))

    def set_persistent_limit(self, max_groups: int) -> None:
        """golhip_set_persistent_limit: slabs the caller owns CUs for (0 = the whole device)."""
        self._check(self._L.golhip_set_persistent_limit(self._h, max_groups))

    def alive_count(self) -> int:
        v = ctypes.c_uint64()
        self._check(self._L.golhip_alive_count(self._h, ctypes.byref(v)))
        return v.value

    def _cells(self, fn) -> np.ndarray:
        n = ctypes.c_size_t(0)
        rc = fn(self._h, None, 0, ctypes.byref(n))
        if rc not in (OK, ERR_CAP):
            self._check(rc)
        out = np.empty((max(n.value, 1), 2), dtype=np.int32)
        self._check(fn(self._h, out.ctypes.data, n.value, ctypes.byref(n)))
        return out[: n.value]

    def alive_cells(self) -> np.ndarray:
        """(n, 2) int32 array of (x, y), row-major (gol/distributor.go:153-166)."""
        return self._cells(self._L.golhip_alive_cells)

    def flips(self) -> np.ndarray:
        """(n, 2) int32 array of (x, y) that changed in the last generation."""
        return self._cells(self._L.golhip_flips)

    def checkpoint_save(self, path):
        self._check(self._L.golhip_checkpoint_save(self._h, str(path).encode()))

    def checkpoint_load(self, path):
        self._check(self._L.golhip_checkpoint_load(self._h, str(path).encode()))

    def track_flips(self, enable: bool = True):
        """Keep the last generation's flips on every step (golhip_flips valid after a K-deep step)."""
        self._check(self._L.golhip_track_flips(self._h, int(enable)))

    def flips_ring_capacity(self) -> int:
        v = ctypes.c_int64()
        self._check(self._L.golhip_flips_ring_capacity(self._h, ctypes.byref(v)))
        return v.value

    def step_flips(self, turns: int, counts: bool = False):
        """Advance `turns` keeping every turn's flips: returns (list of per-turn (n_t, 2) views of
        a host buffer reused by the next call, alive counts per turn or None)."""
        n = ctypes.c_size_t(0)
        per = np.zeros(max(turns, 1), dtype=np.uint64)
        alive = np.zeros(max(turns, 1), dtype=np.uint64) if counts else None
        # one page-locked host list reused across calls (a fresh multi-100-MB array per call would
        # spend its time in page faults; pageable memory halves the copy rate): filled directly
        # when it fits, else grown and fetched
        buf = getattr(self, "_flip_buf", None)
        if buf is None:
            buf = self._flip_buf = pinned_empty((1 << 16, 2), np.int32)
        rc = self._L.golhip_step_flips(self._h, turns, buf.ctypes.data, len(buf), ctypes.byref(n),
                                       per.ctypes.data, alive.ctypes.data if counts else None)
        if rc == ERR_CAP:
            buf = self._flip_buf = pinned_empty((max(n.value, 2 * len(buf)), 2), np.int32)
            self._check(self._L.golhip_flips_fetch(self._h, buf.ctypes.data, len(buf),
                                                   ctypes.byref(n), per.ctypes.data))
        else:
            self._check(rc)
        xy = buf
        bounds = np.concatenate([[0], np.cumsum(per[:turns])]).astype(np.int64)
        out = [xy[bounds[t]:bounds[t + 1]] for t in range(turns)]
        return out, (alive[:turns] if counts else None)

    def step_flips_rows(self, turns: int, counts: bool = False):
        """golhip_step_flips_rows: (x, row_offsets, alive counts or None), views of page-locked
        buffers reused by the next call.  x[row_offsets[t*rows + y] : row_offsets[t*rows + y + 1]]
        are the x of the cells turn t flipped on row y of this handle's strip."""
        n = ctypes.c_size_t(0)
        rows = self.info.rows
        alive = np.zeros(max(turns, 1), dtype=np.uint64) if counts else None
        offs = getattr(self, "_rows_offs", None)
        if offs is None or len(offs) < turns * rows + 1:
            offs = self._rows_offs = pinned_empty((turns * rows + 1,), np.uint64)
        x = getattr(self, "_rows_x", None)
        if x is None:
            x = self._rows_x = pinned_empty((1 << 17,), np.uint16)
        rc = self._L.golhip_step_flips_rows(self._h, turns, x.ctypes.data, len(x), ctypes.byref(n),
                                            offs.ctypes.data, alive.ctypes.data if counts else None)
        if rc == ERR_CAP:
            x = self._rows_x = pinned_empty((max(n.value, 2 * len(x)),), np.uint16)
            self._check(self._L.golhip_flips_fetch_rows(self._h, x.ctypes.data, len(x), ctypes.byref(n),
                                                        offs.ctypes.data))
        else:
            self._check(rc)
        return x[:n.value], offs[:turns * rows + 1], (alive[:turns] if counts else None)

    @staticmethod
    def rows_to_cells(x, offs, rows: int, turns: int, y0: int = 0):
        """Expand golhip_step_flips_rows output to per-turn (n_t, 2) int32 (x, y) arrays (tests)."""
        out = []
        for t in range(turns):
            o = offs[t * rows:(t + 1) * rows + 1].astype(np.int64)
            ys = np.repeat(np.arange(rows, dtype=np.int32) + y0, np.diff(o))
            xs = x[o[0]:o[-1]].astype(np.int32)
            out.append(np.stack([xs, ys], axis=1) if len(xs) else np.zeros((0, 2), np.int32))
        return out

    @property
    def turn(self) -> int:
        t = ctypes.c_int64()
        self._check(self._L.golhip_turn(self._h, ctypes.byref(t)))
        return t.value

    @turn.setter
    def turn(self, value: int):
        self._check(self._L.golhip_set_turn(self._h, value))

    # -- tuning / measurement
    def set_k(self, k: int):
        self._check(self._L.golhip_set_k(self._h, k))
        self.info = self.get_info()

    def set_fixed_k(self, fixed: bool):
        """Every bulk launch exactly k deep (depth sweeps); default: fastest measured depth <= k."""
        self._check(self._L.golhip_set_fixed_k(self._h, int(fixed)))

    def set_band_rows(self, rows: int):
        self._check(self._L.golhip_set_band_rows(self._h, rows))
        self.info = self.get_info()

    def set_tail_bands(self, bands: int, rows: int):
        self._check(self._L.golhip_set_tail_bands(self._h, bands, rows))

    def set_graphs(self, mode: int):
        """Graph replay of step blocks: -1 automatic, 0 never, 1 whenever the plan allows."""
        self._check(self._L.golhip_set_graphs(self._h, mode))

    def set_count_window(self, generations: int):
        self._check(self._L.golhip_set_count_window(self._h, generations))

    def set_comm_timeout(self, ms: int):
        """Deadline of waits on RCCL-dependent work (rank mode): ERR_RCCL when it passes."""
        self._check(self._L.golhip_set_comm_timeout(self._h, int(ms)))

    def comm_abort(self):
        """After GOLHIP_ERR_RCCL: ncclCommAbort the handle's communicator (RCCL aborts its operations
        still running on the device), so the streams can drain before close()."""
        self._check(self._L.golhip_comm_abort(self._h))

    def launch_kind(self, k: int, counts: bool = False) -> tuple[str, int]:
        """The kernel a k-deep launch runs (with / without per-generation counts): ("stream", 0),
        ("split", S), ("tile", T), ("slab", [10000 NC +] 100 W + S) or ("board", 100 W + R)."""
        kind, param = ctypes.c_int(), ctypes.c_int()
        self._check(self._L.golhip_launch_kind_counts(self._h, k, int(counts), ctypes.byref(kind),
                                                      ctypes.byref(param)))
        return ("stream", "split", "tile", "slab", "board")[kind.value], param.value

    def sync(self):
        self._check(self._L.golhip_sync(self._h))

    def timing(self, enable: bool):
        self._check(self._L.golhip_timing(self._h, int(enable)))

    def set_activity(self, enable: int):
        """Stable-slab skipping of the slab launches (golhip_set_activity): -1 automatic (the
        default: boards with more slabs than CUs), 0 / False off, 1 / True on."""
        self._check(self._L.golhip_set_activity(self._h, int(enable)))

    def set_board_kernel(self, enable: int):
        """The whole-board kernel for boards that fit one workgroup (golhip_set_board_kernel): -1
        automatic (the default: boards of at most 256 rows), 0 / False off, 1 / True every board
        it fits."""
        self._check(self._L.golhip_set_board_kernel(self._h, int(enable)))

    def activity_stats(self) -> tuple[int, int]:
        """(slabs computed, slabs skipped) since create (golhip_activity_stats)."""
        c, k = ctypes.c_int64(), ctypes.c_int64()
        self._check(self._L.golhip_activity_stats(self._h, ctypes.byref(c), ctypes.byref(k)))
        return c.value, k.value

    def edge_wait(self) -> tuple[float, int]:
        """With timing on (split boards): ms the compute stream waited for the boundary bands after
        each block's interior, summed, and the number of blocks (golhip_edge_wait)."""
        ms, blocks = ctypes.c_double(), ctypes.c_int64()
        self._check(self._L.golhip_edge_wait(self._h, ctypes.byref(ms), ctypes.byref(blocks)))
        return ms.value, blocks.value

    def kernel_time(self) -> tuple[float, int, int]:
        ms, launches, gens = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        self._check(self._L.golhip_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(launches),
                                               ctypes.byref(gens)))
        return ms.value, launches.value, gens.value
