/*
 * golhip.h -- C ABI of libgolhip, the MI355X (gfx950) Game-of-Life engine.
 *
 * libgolhip replaces the reference's per-turn compute path (Oliver-Cairns/distributed-gol):
 *
 *   reference (Go, net/rpc)                                   replaced by
 *   -------------------------------------------------------   ----------------------------------
 *   Broker.Publish(req, res)        broker/broker.go:157-180  golhip_step()  (res.World = next gen)
 *     publish: 4-strip fan-out      broker/broker.go:37-56    row strips over GPUs (golhip_create*)
 *     strip stitch + worldSave      broker/broker.go:168-175  device-resident board, halos by RCCL
 *   GolOP.Work(req, res)            server/server.go:77-107   gfx950 stencil kernel (k gens/launch)
 *     calculateNextState/updateCell server/server.go:21-75    bit-sliced B3/S23 (64 cells per uint64)
 *   calculateAliveCells             gol/distributor.go:153-166 golhip_alive_count / golhip_alive_cells
 *   CellFlipped diff                gol/distributor.go:53-59  golhip_flips
 *   readPgmImage / writePgmImage    gol/io.go:42-128          golhip_load_bytes / golhip_store_bytes
 *   Broker.CheckStates/Pause state  broker/broker.go:124-155  golhip_turn + the resident board
 *
 * Conventions (all functions):
 *   - return 0 (GOLHIP_OK) or a negative GOLHIP_ERR_* code; golhip_last_error(h) describes the
 *     last failure on that handle (the reference only prints RPC errors, gol/distributor.go:50-52;
 *     here every failure is reported, never silently ignored).
 *   - a handle is owned by ONE host thread; caller-owned host buffers are never retained.
 *   - cells are bytes: 0 = dead, any nonzero = alive on input (gol_test.go:119), 255 on output
 *     (server/server.go:37,46).  The board is a torus (server/server.go:58-69).
 *   - "the handle's rows" are [y0, y0+rows) of the global board (golhip_get_info): the whole board
 *     for golhip_create(), this rank's row strip for golhip_create_rank().
 *   - functions marked COLLECTIVE must be called by every rank of a golhip_create_rank() group.
 */
#ifndef GOLHIP_H
#define GOLHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct golhip_engine *golhip_t;

#define GOLHIP_OK 0
#define GOLHIP_ERR_ARG (-1)   /* invalid argument (sizes, null pointers, k range) */
#define GOLHIP_ERR_HIP (-2)   /* HIP runtime error */
#define GOLHIP_ERR_OOM (-3)   /* device allocation failed */
#define GOLHIP_ERR_CAP (-4)   /* output capacity too small: *n holds the required count */
#define GOLHIP_ERR_RCCL (-5)  /* RCCL error */
#define GOLHIP_ERR_NODEV (-6) /* no gfx950 device / not enough devices */
#define GOLHIP_ERR_STATE (-7) /* call not valid in the current state (e.g. flips after k>1) */

#define GOLHIP_NCCL_ID_BYTES 128
#define GOLHIP_DENSITY_HALF 0x80000000u /* density_q32 for p = 0.5 (raw random bits) */

typedef struct {
    int64_t width;        /* logical board width  (Params.ImageWidth,  gol/gol.go:6-11) */
    int64_t height;       /* logical board height (Params.ImageHeight) */
    int64_t torus_width;  /* device torus width L = lcm(width, 128) (horizontal replication) */
    int64_t y0;           /* first global row held by this handle */
    int64_t rows;         /* rows held by this handle */
    int32_t rank;         /* first rank of this handle */
    int32_t world_size;   /* number of row strips (GPUs) the board is split over */
    int32_t nshards;      /* strips owned by this handle (ngpus for golhip_create) */
    int32_t k;            /* generations per stencil launch (temporal blocking depth) */
    int32_t halo_rows;    /* halo rows allocated per strip edge (>= k when world_size > 1) */
    int32_t band_rows;    /* rows per wave band in the stencil launch (0 = automatic) */
} golhip_info;

/* ---- library / devices ------------------------------------------------------------------ */
int golhip_version(void);                 /* e.g. 100 for 0.1.0 */
const char *golhip_strerror(int code);
int golhip_device_count(int *out);        /* visible HIP devices */
/* Pure host helper: the row strip of `rank` when `height` rows are split over world_size GPUs. */
int golhip_strip_bounds(int64_t height, int world_size, int rank, int64_t *y0, int64_t *rows);

/* One transfer of the halo exchange, in the order the engine issues it inside one RCCL group
 * (kind 0 = send, 1 = receive; rows relative to the strip's row 0, negative = top halo).
 * With world_size == 2 both neighbours are the same peer: RCCL matches the i-th send of a rank
 * to a peer with the i-th receive of that peer, which this order keeps consistent. */
typedef struct {
    int32_t kind;
    int32_t peer;
    int64_t row;
    int64_t nrows;
} golhip_xfer;
/* Pure host helper: the 4 transfers of `rank` for a k-row exchange (out[4]). */
int golhip_halo_plan(int64_t height, int world_size, int rank, int k, golhip_xfer *out);

/* ---- lifetime --------------------------------------------------------------------------- */
/* One process, `ngpus` devices (0..ngpus-1), one row strip each
 * (the on-node replacement of the broker + 4 servers, broker/broker.go:191-205), halos moved by
 * peer copies over xGMI. k = max generations per temporal-blocking stencil launch (1..32; the
 * whole-board kernel of golhip_set_board_kernel is not bounded by it). */
int golhip_create(int width, int height, int ngpus, int k, golhip_t *out);
/* One process, `nstrips` row strips placed on devices 0..ndevices-1 (strip s on device
 * s*ndevices/nstrips), halos by peer copies.  golhip_create(w, h, n, k) == create_strips(w, h, n, n, k);
 * nstrips > ndevices exercises the multi-strip path on fewer GPUs. */
int golhip_create_strips(int width, int height, int nstrips, int ndevices, int k, golhip_t *out);
/* One process per GPU: rank `rank` of `world_size`, on HIP device `device`. nccl_id: the
 * GOLHIP_NCCL_ID_BYTES produced by golhip_nccl_unique_id() on rank 0 (NULL if world_size == 1).
 * Test hook: with world_size == 1 and the environment variable GOLHIP_RING_SELF set (nonzero) the
 * board is a ring of ONE halo'd strip whose halos go through RCCL send/recv to itself (the
 * rank-mode path on a single GPU).
 * The communicator is non-blocking: a rank whose peers never join fails after the comm timeout.
 * GOLHIP_RING_SELF and GOLHIP_STAGE_BYTES (the transfer stage's size in bytes, read at create;
 * tests shrink it to force many row chunks) are the only environment variables the production
 * library reads (fault injection for the fail-fast tests is in the tuning library only). */
int golhip_nccl_unique_id(uint8_t *out /* GOLHIP_NCCL_ID_BYTES */);
int golhip_create_rank(int width, int height, int rank, int world_size, int device, int k,
                       const uint8_t *nccl_id, golhip_t *out);
/* The rank-mode engine with the caller's host transport in place of RCCL (the same strips,
 * launch plan, halo plan, interior/boundary overlap and count reduction; only the transport
 * differs).  Each K-block the engine copies its two send blocks of K rows to pinned host
 * buffers and calls exchange() with the 4 transfers of golhip_halo_plan in issue order
 * (bufs[i]: K * torus_width/8 bytes, a send's payload or a receive's destination; the i-th
 * send to a peer must match that peer's i-th receive from this rank); allreduce_u64 sums n
 * values over the ranks in place (per-turn counts, golhip_alive_count).  Both return 0 on
 * success; anything else fails the call with GOLHIP_ERR_RCCL.  For hosts whose ranks cannot
 * use RCCL peers -- e.g. several ranks sharing one GPU in a test, which RCCL refuses
 * ("Duplicate GPU"); the cgo host would hand its own transport here the same way.  `comm` is
 * copied; ctx must outlive the handle. */
typedef struct {
    void *ctx;
    int (*exchange)(void *ctx, const golhip_xfer *xfers, int n, void *const *bufs, size_t bytes);
    int (*allreduce_u64)(void *ctx, uint64_t *vals, size_t n);
} golhip_host_comm;
int golhip_create_rank_host(int width, int height, int rank, int world_size, int device, int k,
                            const golhip_host_comm *comm, golhip_t *out);
int golhip_destroy(golhip_t h);
const char *golhip_last_error(golhip_t h);  /* h == NULL: why the last create failed (this thread) */
int golhip_get_info(golhip_t h, golhip_info *out);

/* ---- board in / out (gol/io.go:42-128, util/cell.go) ------------------------------------- */
/* Load the handle's rows from 0/nonzero bytes (row y at cells + (y - y0) * row_stride). */
int golhip_load_bytes(golhip_t h, const uint8_t *cells, size_t row_stride);
/* Counter-based random board, regenerated on device (identical for any world_size):
 * width % 64 == 0; logical uint64 word i = y * width/64 + j:
 *   density_q32 == GOLHIP_DENSITY_HALF : word = splitmix64(seed + (i+1) * 0x9E3779B97F4A7C15)
 *   otherwise : cell c = y*width + x alive iff (uint32)splitmix64(seed + (c+1)*0x9E37..) < density_q32 */
int golhip_init_random(golhip_t h, uint64_t seed, uint32_t density_q32);
/* Store the handle's rows as 0/255 bytes (the PGM body, gol/io.go:76-81). */
int golhip_store_bytes(golhip_t h, uint8_t *out, size_t row_stride);
/* Packed little-endian uint64 rows of the handle's rows (width % 64 == 0): rows * width/64 words. */
int golhip_store_words(golhip_t h, uint64_t *out);
int golhip_load_words(golhip_t h, const uint64_t *in);

/* ---- checkpoint: the broker's paused state (broker/broker.go:124-155) ---------------------
 * The reference keeps worldSave/turn/size in the broker process between controller runs ('q'
 * sends Pause{P: true, Turn, Dimension}; the next controller's CheckStates resumes when the size
 * matches, gol/distributor.go:69-91).  Here that state is a file: the handle's rows as packed
 * bits (64-byte header: "GOLCKPT1", version 1, width, height, y0, rows, turn, row bytes; then
 * rows x ceil(width/8) bytes, LSB-first) and the completed turn, written atomically (tmp +
 * rename).  A rank-mode handle writes/loads its own strip (one file per rank). */
int golhip_checkpoint_save(golhip_t h, const char *path);
/* Restores the board and turn; GOLHIP_ERR_STATE if the file holds another board or strip. */
int golhip_checkpoint_load(golhip_t h, const char *path);
/* Pure host helper: the board size and turn a checkpoint holds (CheckStates' SameSize test). */
int golhip_checkpoint_info(const char *path, int64_t *width, int64_t *height, int64_t *turn);

/* ---- the hot path ------------------------------------------------------------------------ */
/* Advance `turns` generations (Broker.Publish called `turns` times, gol/distributor.go:48-49).
 * alive_per_turn (nullable, len turns): alive cells after each completed turn, counted inside the
 * stencil launch (the AliveCellsCount/TurnComplete source, gol/distributor.go:168-191).
 * COLLECTIVE when alive_per_turn != NULL or world_size > 1.  Asynchronous when alive_per_turn
 * is NULL (use golhip_sync to wait). */
int golhip_step(golhip_t h, int64_t turns, uint64_t *alive_per_turn);
/* Pure host helper: the launch depths golhip_step(turns) runs on a width x height board held as
 * `strips` row strips with maximum depth k (the reference has no such split: it runs one turn per
 * Broker.Publish, gol/distributor.go:48-49).  depths[i] > 0: one stencil launch of that many
 * generations; < 0: one captured graph replay of -depths[i] generations (small boards).  Large
 * boards run the depth <= k with the highest measured rate in bulk and split the last ones by a
 * modelled-time plan (e.g. 20 turns at 65536^2 -> 12 + 8, not 16 + 4).  Row strips are planned
 * from the largest strip, ceil(height / strips) rows, so every rank of a rank-mode board runs this
 * same sequence (each launch exchanges K-row halos) even when the strips differ by a row.
 * *n = number of entries; depths may be NULL to size the array; GOLHIP_ERR_CAP if cap is too
 * small. */
int golhip_launch_plan(int64_t width, int64_t height, int strips, int k, int64_t turns,
                       int32_t *depths, size_t cap, size_t *n);
/* Alive cells of the whole board (COLLECTIVE: sums over ranks). */
int golhip_alive_count(golhip_t h, uint64_t *out);
/* Alive cells of the handle's rows as (x, y) int32 pairs, row-major (gol/distributor.go:153-166).
 * If the count exceeds cap, returns GOLHIP_ERR_CAP with *n = required count. */
int golhip_alive_cells(golhip_t h, int32_t *xy, size_t cap, size_t *n);
/* Cells that changed in the last generation (gol/distributor.go:53-59), (x, y) pairs, row-major.
 * Valid after any golhip_step when flips tracking is on (the step's last launch writes them
 * beside its output), or after a step whose last launch advanced 1 generation; GOLHIP_ERR_STATE
 * otherwise. */
int golhip_flips(golhip_t h, int32_t *xy, size_t cap, size_t *n);
/* Flips tracking: every golhip_step keeps the flips of its last generation (one extra store per
 * row in its last launch), so golhip_flips is valid after a K-deep step. */
int golhip_track_flips(golhip_t h, int enable);
/* Per-turn CellFlipped for event consumers (the reference's per-turn diff, gol/distributor.go:
 * 53-59, and TurnComplete, :180-184): advance `turns` generations (<= golhip_flips_ring_capacity)
 * keeping each turn's flips in a device ring, then return them in ONE extraction: xy = every
 * turn's flipped cells, turn by turn, row-major within a turn; flips_per_turn[t] (nullable, len
 * turns) = cells flipped by turn t; alive_per_turn as in golhip_step.  If cap is too small the
 * turns are still advanced, GOLHIP_ERR_CAP is returned with *n = the required count and
 * golhip_flips_fetch returns them.  COLLECTIVE like golhip_step. */
int golhip_step_flips(golhip_t h, int64_t turns, int32_t *xy, size_t cap, size_t *n,
                      uint64_t *flips_per_turn, uint64_t *alive_per_turn);
int golhip_flips_ring_capacity(golhip_t h, int64_t *out);
int golhip_flips_fetch(golhip_t h, int32_t *xy, size_t cap, size_t *n, uint64_t *flips_per_turn);
/* The same per-turn flips (gol/distributor.go:53-59) in a compact form for consumers that take
 * rows: x[i] (uint16, width <= 65536) in the same turn-major, row-major order, and
 * row_offsets[t * rows + y] = the index in x of the first flip of turn t on row y of this
 * handle's strip (rows = golhip_info.rows; row y is board row golhip_info.y0 + y),
 * row_offsets[turns * rows] = *n (turns * rows + 1 entries, always written).  2 bytes per flip
 * instead of an 8-byte (x, y) pair: the list's transfer is what bounds golhip_step_flips on boards
 * with many flips.  One strip per handle (GOLHIP_ERR_STATE otherwise).  A too-small cap returns
 * GOLHIP_ERR_CAP with *n and row_offsets set; golhip_flips_fetch_rows returns the cells then.
 * COLLECTIVE like golhip_step. */
int golhip_step_flips_rows(golhip_t h, int64_t turns, uint16_t *x, size_t cap, size_t *n,
                           uint64_t *row_offsets, uint64_t *alive_per_turn);
int golhip_flips_fetch_rows(golhip_t h, uint16_t *x, size_t cap, size_t *n, uint64_t *row_offsets);
/* Completed turns since the last load (the broker's `turn`, broker/broker.go:140). */
int golhip_turn(golhip_t h, int64_t *out);
int golhip_set_turn(golhip_t h, int64_t turn);

/* ---- tuning / measurement ---------------------------------------------------------------- */
int golhip_set_k(golhip_t h, int k);                 /* 1..32, <= halo_rows when world_size > 1 */
/* k is the MAXIMUM launch depth: long runs use the depth <= k with the highest measured rate
 * (golhip_launch_plan).  fixed != 0: every bulk launch is exactly k deep (depth sweeps). */
int golhip_set_fixed_k(golhip_t h, int fixed);
int golhip_set_band_rows(golhip_t h, int band_rows); /* 0 = automatic */
/* Graded bands (tuning): the streaming launch's rows end in `bands` bands of `rows` rows each
 * instead of full-height ones (0, 0 = uniform bands). */
int golhip_set_tail_bands(golhip_t h, int bands, int rows);
/* Which kernel a k-deep launch on this handle's first strip runs: *kind = 0 the streaming kernel
 * (gol_stencil, gol_step1 at k = 1), 1 the level-split kernel (*param = waves per band), 2 the
 * register-tile kernel gol_tile (*param = tile height T), 3 the register-slab kernel gol_slab
 * (*param = [10000 * row chains +] 100 * waves + rows per wave), 4 the whole-board kernel gol_board
 * (*param = 100 * waves + rows per segment; golhip_set_board_kernel).  Introspection for tests and the
 * bench line.  golhip_launch_kind describes a launch without per-generation counts,
 * golhip_launch_kind_counts one with (counting != 0) or without them: small boards pick a
 * different slab shape when counting. */
int golhip_launch_kind(golhip_t h, int k, int *kind, int *param);
int golhip_launch_kind_counts(golhip_t h, int k, int counting, int *kind, int *param);
/* Captured-graph replay of step blocks on single-strip small boards: -1 automatic (boards whose
 * launches are short), 0 never, 1 whenever the launch plan allows (tests, tuning). */
int golhip_set_graphs(golhip_t h, int mode);
/* Generations of per-turn counts summed per finalize launch (default 4096, minimum 128; tests
 * shrink it to exercise the flushes).  Synchronises the handle. */
int golhip_set_count_window(golhip_t h, int generations);
/* Deadline (ms) of every host wait on work behind an RCCL transfer in rank mode -- the
 * communicator's set-up at create, a halo exchange, the count all-reduce, a sync -- plus 10x the
 * modelled time of the stencil work queued since the last sync.  When it passes (or RCCL reports an
 * asynchronous error) the call returns GOLHIP_ERR_RCCL, with golhip_last_error naming the rank,
 * the pending operation, its peers, K and its byte count; the handle then only accepts
 * golhip_comm_abort / golhip_destroy.  A communicator whose set-up failed is aborted (nothing of
 * it is on the device); after set-up it is left in place until golhip_comm_abort or golhip_destroy
 * (which aborts a failed communicator, then drains the streams within the timeout) or the end of
 * the process.  h == NULL sets the default of later creates (120000).
 * The reference has no such bound: a dead server stalls Broker.Publish (broker/broker.go:58-84). */
int golhip_set_comm_timeout(golhip_t h, int64_t ms);
/* After GOLHIP_ERR_RCCL on a rank-mode handle: ncclCommAbort its communicator (RCCL aborts the
 * operations of it still running on the device, so a receive whose send never comes stops
 * spinning), after which golhip_destroy can drain the handle's streams and free its memory.
 * GOLHIP_ERR_STATE if the communicator has not failed. */
int golhip_comm_abort(golhip_t h);
int golhip_sync(golhip_t h);                         /* wait for all queued device work */
/* The whole-board kernel: a single-strip board of 128, 256 or 512 torus cells per row (any width up
 * to 512 whose lcm with 128 is one of them: the reference's 16/64/128/256/512 sizes) and 4 W R rows
 * (4 ... 512) runs in ONE workgroup holding the whole torus in registers, every golhip_step call as
 * one launch per 4096 generations: no temporal-blocking trapezoid, no halo lanes, no launch
 * boundary inside a call.  Its launches are therefore NOT bounded by the handle's k (the depth of
 * the temporal-blocking stencil launches; golhip_launch_plan lists them as up to 4096 deep), and
 * golhip_set_fixed_k(h, 1) turns it off (a depth sweep measures the k-deep stencil launches).  enable = -1 (default): boards of at most 256 rows (one CU does the
 * board's whole VALU work per generation: faster than the multi-workgroup slabs up to 256 rows,
 * slower at 512), 1: every board it fits, 0: never (A/B).  golhip_launch_kind reports it as
 * kind 4 (*param = 100 * waves + rows per segment).  GOLHIP_ERR_ARG outside -1 .. 1. */
int golhip_set_board_kernel(golhip_t h, int enable);
/* golhip_step with per-turn counts (alive_per_turn non-null) as ONE launch per count window of a
 * persistent slab kernel (gol_slabq): each slab waits for its 3 x 3 neighbourhood of slabs
 * through device counters (golhip_set_persistent_handoff) instead of for a launch boundary every 16
 * generations; the same board and counts as golhip_step (a tail under 16 turns runs through it).
 * Opt-in, for single-strip boards whose counting launch is a gol_slab2 12x7 / 16x6 / 12x8 / 16x4 slab
 * with at most one slab per CU (configs[1], configs[4]; GOLHIP_ERR_STATE otherwise), a handle with
 * k >= 16 and flip tracking off (golhip_track_flips: GOLHIP_ERR_STATE, use golhip_step).  Its
 * progress needs every slab resident at once: the call refuses with GOLHIP_ERR_STATE, before any
 * device work, when the occupancy query does not put the whole grid on the device or the slabs
 * exceed golhip_set_persistent_limit.  If a slab still waits over 200 ms (another process took
 * CUs) the call restores the board and turn it started from and returns GOLHIP_ERR_STATE: a failed
 * call never leaves the board half advanced (the reference's Publish gate never leaves the world
 * half-written either, broker/broker.go:109-120). */
int golhip_step_persistent(golhip_t h, int64_t turns, uint64_t *alive_per_turn);
/* The persistent slab's neighbour hand-off.  GOLHIP_HANDOFF_FENCED (default): agent-scope release /
 * acquire fences around each slab's block counter -- the memory model's own guarantee, ~2.6 us per
 * 16-generation block.  GOLHIP_HANDOFF_SC1: write-through (`sc1`) board stores drained before the
 * counter store and `sc1` loads, no fences -- the hand-off measured valid on gfx950 / ROCm 7.2 but not
 * guaranteed by the architecture documents; faster (configs[4] 0.64 vs 0.81 us/turn).  Opt-in. */
#define GOLHIP_HANDOFF_FENCED 0
#define GOLHIP_HANDOFF_SC1 1
int golhip_set_persistent_handoff(golhip_t h, int mode);
/* The CUs the caller owns for golhip_step_persistent: at most max_groups slabs (one workgroup per
 * CU each) may be assumed resident at once -- for a process sharing the GPU with other work (a
 * second engine, a CU-masked stream, another process).  0 (default): the whole device. */
int golhip_set_persistent_limit(golhip_t h, int max_groups);
/* Stable-slab skipping: the register-slab launches of single-strip boards skip every slab whose
 * neighbourhood did not change in the previous launch's last generation -- Life's radius-1 rule
 * keeps such a slab fixed for the launch's K generations -- copying it once and counting its cached
 * alive cells for each generation.  Results are identical either way.  enable = -1 (default):
 * boards with more slabs than CUs (with one slab per CU a launch lasts as long as its slowest
 * computed slab, so skipping saves nothing there; sparse 16384^2 runs 1.7x faster, dense boards
 * pay ~8 % for the flags), 1: every eligible launch, 0: never (A/B).  GOLHIP_ERR_ARG outside
 * -1 .. 1. */
int golhip_set_activity(golhip_t h, int enable);
/* Slab launches computed / skipped on this handle since it was created (stable-slab skipping). */
int golhip_activity_stats(golhip_t h, int64_t *computed, int64_t *skipped);
/* HIP-event timing of golhip_step calls on the handle's first strip (one event pair per call
 * around its back-to-back stencil launches); kernel_time reports the summed span, the number of
 * stencil launch blocks and generations. */
int golhip_timing(golhip_t h, int enable);
int golhip_kernel_time(golhip_t h, double *total_ms, int64_t *launches, int64_t *generations);
/* With timing on, on a board held as halo'd row strips (rank mode): the summed time the first
 * strip's compute stream waited, after each block's interior launch, for that block's two boundary
 * bands -- which wait for the halo exchange -- and the number of such blocks.  The part of a
 * rank's time its neighbours and the transport cost it (the N > 1 bench line's per-rank data). */
int golhip_edge_wait(golhip_t h, double *total_ms, int64_t *blocks);

#ifdef __cplusplus
}
#endif
#endif /* GOLHIP_H */
