"""CPU ORACLE for the Game-of-Life hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker (or the timed CPU baseline).  The product
path (``distributed-gol_amd/`` -> ``libgolhip.so``) never imports it.

Thin numpy/ctypes layer over ``oracle/build/liboracle.so`` (``gol_oracle.c``):

* ``ref_run``     -- restatement of the reference's byte-per-cell broker+server turn
                     (server/server.go:21-107, broker/broker.go:37-56,157-180).
* ``packed_run``  -- independent bit-sliced stepper (pinned against ``ref_run`` and the
                     reference fixtures by tests/test_oracle.py).
* PGM codec       -- gol/io.go:42-128 (header ``P5\\n<W> <H>\\n255\\n`` + W*H bytes).
* ``alive_cells`` -- gol/distributor.go:153-166 (row-major y, then x; value == 255).
* ``flips``       -- gol/distributor.go:53-59 (cells whose byte differs between turns).
"""
from __future__ import annotations

import ctypes
import hashlib
import math
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "liboracle.so"
_lib = None


def build() -> Path:
    """Compile liboracle.so (gcc) if missing or stale."""
    src = HERE / "gol_oracle.c"
    if not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < src.stat().st_mtime:
        import subprocess

        subprocess.check_call(["make", "-s", "-C", str(HERE)])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(str(LIB_PATH))
        i64p = ctypes.POINTER(ctypes.c_int64)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_ref_step.argtypes = [ctypes.c_int, u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_ref_step.restype = ctypes.c_int
        L.oracle_ref_run.argtypes = [ctypes.c_int, u8p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, i64p]
        L.oracle_ref_run.restype = ctypes.c_int
        L.oracle_packed_run.argtypes = [ctypes.c_int, ctypes.c_int, u64p, ctypes.c_long, ctypes.c_int, i64p]
        L.oracle_packed_run.restype = ctypes.c_int
        L.oracle_init_random.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                         ctypes.c_uint64, u64p]
        L.oracle_init_random.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


# ----------------------------------------------------------------------------- PGM codec
def parse_pgm(data: bytes) -> tuple[int, int, np.ndarray]:
    """P5 reader, gol/io.go:90-128 (fields split on whitespace; maxval must be 255)."""
    fields = data.split(maxsplit=4)
    if fields[0] != b"P5":
        raise ValueError("Not a pgm file")
    w, h, maxval = int(fields[1]), int(fields[2]), int(fields[3])
    if maxval != 255:
        raise ValueError("Incorrect maxval/bit depth")
    body = fields[4] if len(fields) > 4 else b""
    if len(body) < w * h:
        raise ValueError("truncated pgm body")
    return w, h, np.frombuffer(body[: w * h], dtype=np.uint8).reshape(h, w).copy()


def read_pgm(path) -> tuple[int, int, np.ndarray]:
    return parse_pgm(Path(path).read_bytes())


def pgm_bytes(board: np.ndarray) -> bytes:
    """P5 writer, gol/io.go:42-87: header then one byte per cell."""
    h, w = board.shape
    return b"P5\n%d %d\n255\n" % (w, h) + np.ascontiguousarray(board, dtype=np.uint8).tobytes()


def to_cells(board: np.ndarray) -> np.ndarray:
    """0/nonzero -> 0/255 (the reference's tests treat any nonzero pixel as alive, gol_test.go:119)."""
    return np.where(board != 0, 255, 0).astype(np.uint8)


# ------------------------------------------------------------------ reference restatement
def ref_run(board: np.ndarray, turns: int, threads: int = 8, servers: int = 4,
            fanout_copy: bool = False) -> tuple[np.ndarray, np.ndarray]:
    """Run the reference broker+server algorithm; returns (final board, counts[turns])."""
    h, w = board.shape
    if h != w:
        raise ValueError("the reference only supports square boards (server/server.go:27)")
    world = np.ascontiguousarray(board, dtype=np.uint8).copy()
    counts = np.zeros(max(turns, 1), dtype=np.int64)
    rc = lib().oracle_ref_run(w, _ptr(world, ctypes.c_uint8), turns, threads, servers,
                              int(fanout_copy), _ptr(counts, ctypes.c_int64))
    if rc != 0:
        raise ValueError("reference split arithmetic drops rows for this size (n % servers != 0)")
    return world, counts[:turns]


# --------------------------------------------------------------------- bit-packed oracle
def torus_width(width: int, align: int = 64) -> int:
    """Width of the horizontally replicated torus the packed layout uses (lcm(width, align))."""
    return width * align // math.gcd(width, align)


def pack(board: np.ndarray, align: int = 64) -> np.ndarray:
    """0/nonzero bytes (h, w) -> uint64 words (h, L/64), LSB-first, replicated to L = lcm(w, align)."""
    h, w = board.shape
    L = torus_width(w, align)
    rep = np.tile((board != 0).astype(np.uint8), (1, L // w))
    return np.packbits(rep, axis=1, bitorder="little").view("<u8").reshape(h, L // 64).copy()


def unpack(words: np.ndarray, width: int) -> np.ndarray:
    """uint64 words -> 0/255 bytes of the first `width` columns."""
    h = words.shape[0]
    bits = np.unpackbits(np.ascontiguousarray(words).view(np.uint8).reshape(h, -1), axis=1,
                         bitorder="little")
    return (bits[:, :width] * 255).astype(np.uint8)


def packed_run_words(words: np.ndarray, turns: int, threads: int = 8) -> np.ndarray:
    """In-place `turns` generations of a packed torus; returns per-turn counts of the
    whole (replicated) torus."""
    assert words.dtype == np.uint64 and words.flags.c_contiguous
    h, wpr = words.shape
    counts = np.zeros(max(turns, 1), dtype=np.int64)
    rc = lib().oracle_packed_run(wpr, h, _ptr(words, ctypes.c_uint64), turns, threads,
                                 _ptr(counts, ctypes.c_int64))
    assert rc == 0
    return counts[:turns]


def packed_run(board: np.ndarray, turns: int, threads: int = 8) -> tuple[np.ndarray, np.ndarray]:
    """Bit-sliced run of a 0/255 byte board of any shape; returns (final board, counts)."""
    h, w = board.shape
    words = pack(board)
    rep = words.shape[1] * 64 // w
    counts = packed_run_words(words, turns, threads) // rep
    return unpack(words, w), counts


# ------------------------------------------------------------------------ synthetic input
DENSITY_HALF = 1 << 31


def init_random(width: int, height: int, seed: int, density_q32: int = DENSITY_HALF,
                y0: int = 0, y1: int | None = None) -> np.ndarray:
    """Counter-based random board (rows y0..y1), packed uint64 (width % 64 == 0)."""
    y1 = height if y1 is None else y1
    out = np.zeros((y1 - y0, width // 64), dtype=np.uint64)
    rc = lib().oracle_init_random(width, y0, y1, seed, density_q32, _ptr(out, ctypes.c_uint64))
    if rc != 0:
        raise ValueError("width must be a multiple of 64")
    return out


# --------------------------------------------------------------------- host-side helpers
def alive_cells(board: np.ndarray) -> list[tuple[int, int]]:
    """gol/distributor.go:153-166: (x, y) of every 255 cell, row-major."""
    ys, xs = np.nonzero(board == 255)
    return list(zip(xs.tolist(), ys.tolist()))


def flips(prev: np.ndarray, cur: np.ndarray) -> list[tuple[int, int]]:
    """gol/distributor.go:53-59: (x, y) of every cell that differs, row-major."""
    ys, xs = np.nonzero(prev != cur)
    return list(zip(xs.tolist(), ys.tolist()))


def digest_words(words: np.ndarray) -> str:
    """SHA-256 of a packed board's little-endian uint64 rows."""
    return hashlib.sha256(np.ascontiguousarray(words, dtype="<u8").tobytes()).hexdigest()


# Board digest that row strips can compute apart ("checksum of checksums"): SHA-256 of the
# concatenated SHA-256s of consecutive DIGEST_CHUNK_ROWS-row chunks of the packed little-endian
# uint64 rows.  A rank whose strip starts on a chunk boundary hashes its own chunks; rank 0 hashes
# the gathered list (bench.py's parity.digest).  4096 divides every strip height the benches use.
DIGEST_CHUNK_ROWS = 4096


def chunk_digests(words: np.ndarray, chunk_rows: int = DIGEST_CHUNK_ROWS) -> list[bytes]:
    w = np.ascontiguousarray(words, dtype="<u8")
    return [hashlib.sha256(w[y:y + chunk_rows].tobytes()).digest() for y in range(0, w.shape[0], chunk_rows)]


def board_digest(chunks: list[bytes]) -> str:
    return hashlib.sha256(b"".join(chunks)).hexdigest()


def read_alive_csv(path) -> dict[int, int]:
    """check/alive/*.csv: header completed_turns,alive_cells (count_test.go:78-89)."""
    out = {}
    for i, line in enumerate(Path(path).read_text().splitlines()):
        if i == 0 or not line.strip():
            continue
        t, c = line.split(",")
        out[int(t)] = int(c)
    return out


if __name__ == "__main__":  # pragma: no cover
    print(build())
    os.sys.exit(0)
