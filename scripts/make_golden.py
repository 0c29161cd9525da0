#!/usr/bin/env python3
"""Generate the golden vectors of the synthetic configs with the (pinned) CPU oracle.

  cfg2: 5120x5120 random p=0.5 seed 2, per-turn alive counts for 10000 turns + final digest
  cfg3: 65536x65536 random p=0.5 seed 3, per-turn counts for 1000 turns (CSV) + digests at 8/1000
  cfg4: 262144x262144 random p=0.5 seed 4, per-turn counts for 176 turns (CSV) + digests at 16/176
  cfg5: 4096x4096 Gosper gun at (64,64) + R-pentomino at (2048,2048), all 1e6 per-turn counts
        (SHA-256 of the uint32 array; the array itself as a compressed delta npz) + digests
Digests = SHA-256 of the packed little-endian uint64 rows (oracle.digest_words).
Run from the repo root: python scripts/make_golden.py [cfg2|cfg3|cfg5 ...]
"""
import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "distributed-gol_amd"))
import oracle  # noqa: E402

OUT = ROOT / "tests" / "golden"


def cfg2():
    w = oracle.init_random(5120, 5120, seed=2)
    t = time.time()
    counts = oracle.packed_run_words(w, 10000, threads=8)
    (OUT / "cfg2_5120_seed2_counts.csv").write_text(
        "completed_turns,alive_cells\n" + "".join(f"{i + 1},{c}\n" for i, c in enumerate(counts)))
    return {"cfg2": {"width": 5120, "height": 5120, "seed": 2, "turns": 10000,
                     "final_digest": oracle.digest_words(w), "counts_csv": "cfg2_5120_seed2_counts.csv",
                     "oracle_seconds": round(time.time() - t, 1)}}


def write_counts_csv(name, counts):
    (OUT / name).write_text(
        "completed_turns,alive_cells\n" + "".join(f"{i + 1},{c}\n" for i, c in enumerate(counts)))


def cfg3():
    w = oracle.init_random(65536, 65536, seed=3)
    t = time.time()
    c8 = oracle.packed_run_words(w, 8, threads=8)
    d8 = oracle.digest_words(w)
    rest = oracle.packed_run_words(w, 992, threads=8)
    counts = np.concatenate([c8, rest])
    d1000 = oracle.digest_words(w)
    # every per-turn count up to 1200 (bench.py checks its alive_after_timed canary against these:
    # the default run ends at turn 8 + 1000, the driver's at 5 + 20)
    more = oracle.packed_run_words(w, 200, threads=8)
    write_counts_csv("cfg3_65536_seed3_counts.csv", np.concatenate([counts, more]))
    return {"cfg3": {"width": 65536, "height": 65536, "seed": 3, "turns": 1000, "csv_turns": 1200,
                     "digest_after_8": d8, "digest_after_1000": d1000,
                     "counts_sha256": hashlib.sha256(counts.astype("<u8").tobytes()).hexdigest(),
                     "counts_csv": "cfg3_65536_seed3_counts.csv",
                     "counts_every_50": {str(i + 1): int(counts[i]) for i in range(49, 1000, 50)},
                     "count_after_1": int(counts[0]), "oracle_seconds": round(time.time() - t, 1)}}


def cfg4():
    """configs[3]: 262144^2 random p=0.5 seed 4 (8 GiB packed; 2 x 8.6 GB of RAM).  Digests after
    16 turns (the bench leg's warm-up launch) and 176 (+ its 160 timed turns) and every count."""
    n = 262144
    w = oracle.init_random(n, n, seed=4)
    t = time.time()
    c16 = oracle.packed_run_words(w, 16, threads=8)
    d16 = oracle.digest_words(w)
    rest = oracle.packed_run_words(w, 160, threads=8)
    counts = np.concatenate([c16, rest])
    write_counts_csv("cfg4_262144_seed4_counts.csv", counts)
    return {"cfg4": {"width": n, "height": n, "seed": 4, "turns": 176,
                     "digest_after_16": d16, "digest_after_176": oracle.digest_words(w),
                     "counts_sha256": hashlib.sha256(counts.astype("<u8").tobytes()).hexdigest(),
                     "counts_csv": "cfg4_262144_seed4_counts.csv",
                     "oracle_seconds": round(time.time() - t, 1)}}


def weak():
    """bench.py --gpus N (weak scaling): the 65536 x 65536*N board, random p=0.5 seed 3, split
    into N row strips.  init_random numbers words over the WHOLE board, so the N-rank board is
    this one global board.  Every per-turn count up to 1200 for N = 2, 4, 8 (the driver's run ends
    at turn 5 + 20, the default one at 8 + 1000); N = 1 is cfg3_65536_seed3_counts.csv."""
    out = {}
    for n in (2, 4, 8):
        w = oracle.init_random(65536, 65536 * n, seed=3)
        t = time.time()
        counts = oracle.packed_run_words(w, 1200, threads=8)
        name = f"weak_65536x{65536 * n}_seed3_counts.csv"
        write_counts_csv(name, counts)
        out[f"weak{n}"] = {"width": 65536, "height": 65536 * n, "seed": 3, "csv_turns": 1200,
                           "counts_csv": name, "digest_after_1200": oracle.digest_words(w),
                           "oracle_seconds": round(time.time() - t, 1)}
        del w
        print("weak", n, out[f"weak{n}"]["oracle_seconds"], "s", flush=True)
    return out


def weak_small():
    """Small weak-scaling boards for the rank-path tests (per-turn counts up to 1200, seed 3):
    4096 x 4096*N (N = 2, 3, 4, 8; tests/test_bench_multirank_cpu.py, the plain-launch rehearsals) and 8192 x 8192*N (N = 2, 3;
    bench.py --gpus N --size 8192 on one GPU with the host transport, tests/test_gpu_rank_host.py)."""
    out = {}
    for w, n in ((4096, 2), (4096, 3), (4096, 4), (4096, 8), (8192, 2), (8192, 3)):
        b = oracle.init_random(w, w * n, seed=3)
        counts = oracle.packed_run_words(b, 1200, threads=8)
        name = f"weak_{w}x{w * n}_seed3_counts.csv"
        write_counts_csv(name, counts)
        out[f"weak_{w}x{w * n}"] = {"width": w, "height": w * n, "seed": 3, "csv_turns": 1200,
                                     "counts_csv": name, "digest_after_1200": oracle.digest_words(b)}
    return out


def digests():
    """Whole-board digests of the bench boards (bench.py parity.digest_ok): the 65536 x 65536*N
    board, random p=0.5 seed 3, for N = 1 (configs[2]) and the weak-scaling N = 2, 4, 8, after
    25 turns (the driver's --warmup 5 --steps 20) and 1008 (the default --warmup 8 --steps 1000).
    oracle.board_digest of 4096-row chunk digests, so each rank hashes its own strip."""
    out = {}
    for n in (1, 2, 4, 8):
        w = oracle.init_random(65536, 65536 * n, seed=3)
        t = time.time()
        oracle.packed_run_words(w, 25, threads=8)
        d25 = oracle.board_digest(oracle.chunk_digests(w))
        oracle.packed_run_words(w, 1008 - 25, threads=8)
        d1008 = oracle.board_digest(oracle.chunk_digests(w))
        out[f"digest_65536x{65536 * n}"] = {
            "width": 65536, "height": 65536 * n, "seed": 3, "chunk_rows": oracle.DIGEST_CHUNK_ROWS,
            "board_digest": {"25": d25, "1008": d1008}, "oracle_seconds": round(time.time() - t, 1)}
        del w
        print("digests", n, out[f"digest_65536x{65536 * n}"]["oracle_seconds"], "s", flush=True)
    return out


def digests_small():
    """Board digests of the small weak-scaling boards the rank-path tests run bench.main() on
    (4096 x 4096*N, N = 2, 3, 8, and 8192 x 8192*N, N = 2, 3, seed 3) after 25 turns (--warmup 5
    --steps 20)."""
    out = {}
    for w, n in ((4096, 2), (4096, 3), (4096, 4), (4096, 8), (8192, 2), (8192, 3)):
        b = oracle.init_random(w, w * n, seed=3)
        oracle.packed_run_words(b, 25, threads=8)
        out[f"digest_{w}x{w * n}"] = {"width": w, "height": w * n, "seed": 3,
                                      "chunk_rows": oracle.DIGEST_CHUNK_ROWS,
                                      "board_digest": {"25": oracle.board_digest(oracle.chunk_digests(b))}}
    return out


def cfg5_board():
    import golhip

    b = np.zeros((4096, 4096), dtype=np.uint8)
    golhip.place(b, golhip.parse_rle((OUT / "gosper_gun.rle").read_text()), 64, 64)
    golhip.place(b, golhip.parse_rle((OUT / "r_pentomino.rle").read_text()), 2048, 2048)
    return b


def cfg5():
    """configs[4]: 4096^2 gun + R-pentomino, all 1e6 per-turn counts.  The counts are committed
    as a delta-encoded, zlib-compressed int32 array (cfg5_4096_counts_1e6.npz) so tests compare
    every tick with the golden count, not with the engine's own."""
    b = cfg5_board()
    w = oracle.pack(b)
    t = time.time()
    counts = oracle.packed_run_words(w, 100000, threads=8)
    d100k = oracle.digest_words(w)
    rest = oracle.packed_run_words(w, 900000, threads=8)
    allc = np.concatenate([counts, rest])
    deltas = np.diff(np.concatenate([[int((b == 255).sum())], allc])).astype("<i4")
    np.savez_compressed(OUT / "cfg5_4096_counts_1e6.npz", deltas=deltas)
    return {"cfg5": {"width": 4096, "height": 4096, "turns": 100000,
                     "initial_alive": int((b == 255).sum()),
                     "counts_u32_sha256": hashlib.sha256(counts.astype("<u4").tobytes()).hexdigest(),
                     "counts_every_1000": {str(i + 1): int(counts[i]) for i in range(999, 100000, 1000)},
                     "digest_after_100000": d100k,
                     "turns_full": 1000000,
                     "counts_1e6_u32_sha256": hashlib.sha256(allc.astype("<u4").tobytes()).hexdigest(),
                     "counts_1e6_npz": "cfg5_4096_counts_1e6.npz",
                     "digest_after_1000000": oracle.digest_words(w),
                     "oracle_seconds": round(time.time() - t, 1)}}


if __name__ == "__main__":
    which = sys.argv[1:] or ["cfg2", "cfg3", "cfg4", "cfg5"]
    path = OUT / "synthetic_golden.json"
    data = json.loads(path.read_text()) if path.exists() else {}
    for name in which:
        data.update(globals()[name]())
        path.write_text(json.dumps(data, indent=1) + "\n")
        print(name, "done", flush=True)
