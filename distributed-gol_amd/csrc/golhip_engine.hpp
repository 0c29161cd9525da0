// golhip_engine.hpp -- the engine's internal state and the functions its translation units share.
// Not part of the public ABI (include/golhip.h is).  The engine is split by role:
//   golhip_engine.hip   handles, the step loop (golhip_step), graph replays, timing, setters
//   engine_plan.hip     the launch planner: depths, bands, the kernel choice per board
//   engine_comm.hip     row strips over ranks: halo exchange (RCCL / peer copies / host transport),
//                       count reductions, the RCCL fail-fast waits, golhip_create_rank*
//   engine_cells.hip    alive-cell lists and CellFlipped extraction, the per-turn flips ring
//   engine_io.hip       host transfers (PGM bytes, uint64 words, random init) and checkpoints
// The tuning library adds tuning/engine_tuning.hip, which registers engine_hooks(); the production
// library has no hooks (every hook pointer below stays null there).
//
// Reference roles (Oliver-Cairns/distributed-gol):
//   * broker/broker.go:37-56  publish(): split the rows into strips -> strip_bounds(), one strip
//     per GPU (the reference's 4 servers become the node's GPUs);
//   * broker/broker.go:58-84,157-180  subscriberLoop/Publish: fan the FULL world out every turn and
//     stitch the strips back -> the board stays resident in HBM, only k halo rows per strip edge
//     move per k generations, by RCCL send/recv over xGMI on a dedicated comm stream that overlaps
//     the interior update;
//   * broker/broker.go:124-155  CheckStates/Pause (worldSave, turn) -> the resident board and
//     golhip_turn()/golhip_set_turn();
//   * server/server.go:21-107  the worker's next-state loop -> the planner's kernel launches.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <deque>
#include <string>
#include <thread>
#include <vector>

#include "../../include/golhip.h"
#include "golhip_internal.hpp"

namespace golhip {

constexpr int kVersion = 103;  // 103: golhip_set_persistent_limit / _handoff (round 6)
// Generations of per-turn counts finalized per launch (golhip_set_count_window changes it; at
// least the graph length kGraphGens: tests shrink it to exercise flushes).
constexpr int kCountWindowDefault = 4096;
constexpr int kCountWindowMin = 128;
// The register slab runs boards on which the streaming kernel would have at most this many
// minimal-band (max(K, 8)-row) waves per CU.  Round 4 sweep (profiles/r04/r04mid_tune_mid.log,
// 512 / 256 turns, every count equal): the slab is 7-11 % faster than streaming up to 16384^2
// without counts (12288^2 2.82 vs 3.14 us/turn, 16384^2 4.09 vs 4.40), even at 20480^2, and
// slower there with counts (9.33 vs 8.39); 16384^2 has 36 such waves per CU, 20480^2 55.
constexpr int64_t kSlabMaxWaves1PerCu = 40;
constexpr int64_t kStampWaves = 1 << 20;  // tuning library: waves of the per-wave stamp buffer
constexpr int64_t kStageBytes = 64ll << 20;
constexpr int kGraphGens = 128;  // generations per graph replay (<= count_window)
// Long runs replay larger graphs: each replay of a counting graph ends in a count finalize and a
// copy of its counts (~17 us together on a 5120^2 board, profiles/r02/small_board_timeline_split_k16.txt),
// paid per 4096 generations instead of per 128 (bounded by the count window).
constexpr int kGraphGensBig = 4096;
constexpr double kLaunchOverheadUs = 4.0;
// diff_slot of step_block: no flips / the last generation's flips into diffbuf / ring slot t >= 0
constexpr int64_t kDiffNone = -1, kDiffLast = -2;

// Default deadline of a host wait on RCCL-dependent work and of the communicator's set-up
// (golhip_set_comm_timeout(NULL, ms) changes it for later creates): well under the 600 s a driver
// gives a whole bench run, far above any legitimate wait (an 8-rank init takes seconds, a K-row
// exchange microseconds; stencil work queued by the host is added to each wait by its model).
extern std::atomic<int64_t> g_comm_timeout_ms;
extern thread_local std::string g_create_error;  // golhip_last_error(NULL)

struct Shard {
    int device = 0;
    int rank = 0;
    int64_t y0 = 0, rows = 0;
    hipStream_t compute = nullptr, comm = nullptr;
    hipStream_t edge = nullptr;  // boundary bands of a split board, concurrent with the interior
    hipEvent_t ev_ready = nullptr, ev_halo = nullptr, ev_edge = nullptr;
    uint32_t *buf[2] = {nullptr, nullptr};  // allocation base (halo rows first)
    unsigned long long *slots = nullptr;    // count_window x kCountSlots
    unsigned long long *scratch_u64 = nullptr;
    // the call's per-turn counts: dev_counts, or on a one-shard engine without RCCL, for calls that
    // replay no graph, pin_counts (pinned host memory, hipHostMalloc coherent): the count finalize
    // writes it directly and the call returns without a device-to-host copy (configs[0], 100
    // turns: the copy and its dispatch gap were ~17 of ~85 us per call)
    unsigned long long *d_counts = nullptr;  // = dev_counts or pin_counts for this call
    bool counts_host = false;
    unsigned long long *dev_counts = nullptr, *pin_counts = nullptr;
    size_t dev_counts_cap = 0, pin_counts_cap = 0;
    ncclComm_t comm_nccl = nullptr;
    // flips (gol/distributor.go:53-59): the last generation's flips board (golhip_track_flips)
    // and a ring of one flips board per turn (golhip_step_flips), rows x pitch words each
    uint32_t *diffbuf = nullptr;
    uint32_t *ring = nullptr;
    // extraction scratch, allocated once (grown only for a larger ring / cell list): per-row
    // counts, their exclusive scan, per-slot totals and the emitted (x, y) pairs
    uint32_t *ex_rowcounts = nullptr;
    unsigned long long *ex_offsets = nullptr;
    unsigned long long *ex_slot_counts = nullptr;
    unsigned long long *ex_block_sums = nullptr;  // kScanBlocks: the multi-block scan's partials
    int64_t ex_rows_cap = 0, ex_slots_cap = 0;
    int32_t *ex_xy = nullptr;
    size_t ex_xy_cap = 0;
    // device staging of host transfers (PGM bytes, uint64 words, the checkpoint byte codec),
    // allocated once at create: no host-facing call allocates or frees device memory (a hipFree
    // synchronises the whole device, and every `s` snapshot / PGM store used to pay one)
    uint8_t *stage = nullptr;
    int64_t stage_bytes = 0;
    // stable-slab skipping (StencilParams::act): 4 x act_cap uint32 flags, 2 uint64 counters
    uint32_t *act = nullptr;
    int64_t act_cap = 0;
    unsigned long long *act_stats = nullptr;
    // golhip_step_persistent: one block counter per slab + the error word
    uint32_t *pflags = nullptr;
    int64_t pflags_cap = 0;
    uint32_t *psave = nullptr;  // the board as of the call's start (restored when a window fails)
};

struct TimingPair {
    hipEvent_t a, b;
};

// A captured run of M K-generation blocks (small boards are launch-bound: one graph replay
// replaces 2M launches).  Kernel arguments are baked in, so a graph is specific to the buffer
// parity it starts from; M is even, so it ends on the parity it started from.
struct GraphEntry {
    int K = 0, M = 0, cur = 0;
    bool counting = false;
    int64_t band = 0;
    int tail_bands = 0, tail_rows = 0;  // golhip_set_tail_bands at capture
    // stable-slab skipping: a graph's first launch always recomputes its flags (act_reset), so a
    // replay never trusts flags of another state; after it the flags are those of its geometry
    bool act_after = false;
    int64_t act_key_after[3] = {0, 0, 0};
    hipGraphExec_t exec = nullptr;
};

// Fault injection of the tuning library (GOLHIP_FAULT, tests/test_gpu_failfast.py); none in
// production.
enum class Fault { none, stall, skip_send, slab_stall };

}  // namespace golhip

struct golhip_engine {
    int64_t width = 0, height = 0, L = 0, pitch = 0;
    int32_t wd = 0;
    int world_size = 1;
    int k = 1, halo = 0, band_rows = 0;
    int tail_bands = 0, tail_rows = 0;  // golhip_set_tail_bands: graded bands (0 = uniform)
    int count_window = 4096;            // generations per count-window finalize
    int variant = golhip::kVariantProd; // fastest measured per depth (golhip_internal.hpp)
    int cus = 0;                        // compute units of the first device (grid sizing)
    int persistent_limit = 0;           // golhip_set_persistent_limit: slabs the caller owns CUs for (0 = all)
    int persistent_handoff = GOLHIP_HANDOFF_FENCED;  // golhip_set_persistent_handoff
    bool fixed_k = false;               // golhip_set_fixed_k: long runs launch exactly k deep
    bool track_flips = false;  // golhip_track_flips: every step ends with a flips-writing launch
    bool diff_valid = false;   // shards' diffbuf holds the flips of the last generation
    int64_t ring_cap = 0;      // turns per golhip_step_flips call (flips ring slots)
    int64_t ring_turns = 0;    // turns held in the ring by the last golhip_step_flips
    int waves_per_cu[golhip::kMaxK + 1][golhip::kNumVariants] = {};  // occupancy cache per (K, variant)
    bool rank_mode = false;
    // golhip_create_rank_host: the caller's host transport instead of RCCL, with pinned host
    // buffers for the 4 K-row transfers of an exchange (halo rows x pitch words each)
    bool host_comm_on = false;
    golhip_host_comm host_comm{};
    void *hc_buf[4] = {nullptr, nullptr, nullptr, nullptr};
    bool split = false;  // board held as halo'd row strips (world > 1, or GOLHIP_RING_SELF)
    // A/B selectors of the tuning library (GOLHIP_SPLIT / GOLHIP_TILE / GOLHIP_SLAB /
    // GOLHIP_EDGE_PRIO / GOLHIP_EDGE_FIRST / GOLHIP_EDGE_SETPRIO, set by engine_hooks()->configure);
    // production keeps these defaults: the automatic choice
    int force_split = 0;  // 0 = automatic
    int force_tile = -1;  // -1 automatic, 0 never, T > 0 always (tile height T)
    int force_slab = -1;  // -1 automatic, 0 never, [NC*10000 +] W*100 + S always (slab shape)
    bool edge_prio = false;   // comm/edge streams at high priority
    bool edge_first = false;  // boundary bands submitted before the interior
    // the boundary bands' waves raise their issue priority (StencilParams::prio)
    int edge_setprio = 1;
    int graph_mode = -1;  // golhip_set_graphs: -1 automatic, 0 never, 1 whenever the plan allows
    // stable-slab skipping (golhip_set_activity: -1 automatic -- boards with more slabs than CUs --,
    // 0 off, 1 on): the slab flags on the shard hold the state of the last launch when act_valid,
    // for slab geometry act_key (T * 64 + W, nbands, nchunks)
    int activity = -1;
    bool act_valid = false;
    // the whole-board kernel (golhip_set_board_kernel: -1 automatic -- boards of at most
    // kBoardAutoRows rows --, 0 off, 1 every board it fits)
    int board_kernel = -1;
    int64_t act_key[3] = {0, 0, 0};
    // RCCL fail-fast (rank mode): every host wait on work that can depend on an RCCL transfer polls
    // ncclCommGetAsyncError against a deadline and fails the handle when it passes
    // (golhip_set_comm_timeout); the communicator is non-blocking, so no RCCL call blocks the host
    int64_t comm_timeout_ms = 0;
    double queued_s = 0.0;  // modelled seconds of stencil work queued since the last full sync
    bool comm_failed = false;
    bool comm_setup_done = false;  // the communicator's set-up completed
    // depth of the boundary bands the last split block ran on the edge stream (0: none, e.g. a strip
    // shorter than 3K or a non-split launch): its rows [0, K) and [rows - K, rows) are exactly what
    // the next exchange sends, so with K' <= edge_k that exchange waits only for those bands
    int edge_k = 0;
    std::string comm_pending;  // the last RCCL operation enqueued (rank, peers, K, bytes)
    // every RCCL operation enqueued and not yet known complete, oldest first, with an event recorded
    // behind it on its stream: a failed wait names the FIRST incomplete one (the stuck transfer),
    // not merely the last one queued
    std::deque<std::pair<hipEvent_t, std::string>> rccl_ops;
    std::vector<hipEvent_t> rccl_ev_pool;
    golhip::Fault fault = golhip::Fault::none;  // tuning library only (GOLHIP_FAULT)
    int64_t exchanges = 0;                      // halo exchanges enqueued (fault targeting, tests)
    // tuning library, GOLHIP_VARIANT=stamp: per-wave timestamps of the last single-strip launch
    uint64_t *stamp_buf = nullptr;
    int64_t stamp_waves = 0;
    int stamp_words = 4;  // uint64 per wave of the last stamped launch (gol_slab2: 8)
    std::vector<golhip::Shard> shards;
    int cur = 0;
    bool prev_valid = false;
    int64_t turn = 0;
    std::string err;
    // graph replay of step blocks (single strip, small boards)
    std::vector<golhip::GraphEntry> graphs;
    unsigned long long *g_counts = nullptr;  // counts written by a counting graph
    // timing
    bool timing = false;
    std::vector<golhip::TimingPair> tpool;
    size_t tused = 0;
    double tms = 0.0;
    int64_t tlaunches = 0, tgens = 0;
    // split boards: per block, the compute stream's wait for the boundary bands after its interior
    // (an event pair around the join; golhip_edge_wait)
    std::vector<golhip::TimingPair> tedge;
    size_t tedge_used = 0;
    double tedge_ms = 0.0;
    int64_t tedge_blocks = 0;

    uint32_t *row0(const golhip::Shard &s, int which) const {
        return s.buf[which] + (int64_t)halo * pitch;
    }
    int64_t rep() const { return L / width; }
};

namespace golhip {

// ---- the tuning library's engine hooks (tuning/engine_tuning.hip; null in production) ---------
struct EngineHooks {
    // create (after the geometry is set): the A/B selectors read from the environment
    void (*configure)(golhip_t h) = nullptr;
    // create, before the shards are allocated: extra device state (the stamp buffer)
    int (*create)(golhip_t h) = nullptr;
    void (*destroy)(golhip_t h) = nullptr;
    // a single-strip launch of depth K is about to be issued with params p (p.diff: its flips
    // board, null for none): the stamp handles point p.diff / p.stamp at their stamp buffer
    void (*launch_params)(golhip_t h, const Shard &s, int K, bool counting, StencilParams &p) = nullptr;
    // the end of a golhip_step call's device work was enqueued (Fault::stall: a 20 s stall of the
    // compute stream)
    int (*after_steps)(golhip_t h) = nullptr;
    // transfer i of a halo exchange's RCCL group is about to be enqueued: true leaves it out
    // (Fault::skip_send: a send the peer's receive never matches -- a stuck RCCL transfer)
    bool (*skip_xfer)(golhip_t h, const golhip_xfer &x, int i) = nullptr;
};
const EngineHooks *engine_hooks();
void set_engine_hooks(const EngineHooks *hooks);

// ---- errors ----------------------------------------------------------------------------------
int fail(golhip_t h, int code, const char *fmt, ...);

#define HIPCHK(h, expr)                                                                     \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return ::golhip::fail((h), e_ == hipErrorOutOfMemory ? GOLHIP_ERR_OOM : GOLHIP_ERR_HIP, \
                                  "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

#define SYNCCHK(h, stream)                             \
    do {                                               \
        int rc_ = ::golhip::wait_stream((h), (stream)); \
        if (rc_) return rc_;                           \
    } while (0)

// ---- engine_comm.hip: waits, the RCCL fail-fast, strips and the halo exchange ----------------
using Clock = std::chrono::steady_clock;
// True when device work of this handle can wait on an RCCL transfer (rank mode over RCCL).
bool rccl_waits(golhip_t h);
// hipStreamSynchronize, bounded by the RCCL deadline in rank mode.
int wait_stream(golhip_t h, hipStream_t st);
// Poll `done` (0 = finished, 1 = not yet, < 0 = error code already set) until it finishes, the
// communicator reports an asynchronous error, or the deadline passes.
int poll_until_fn(golhip_t h, const char *what, int (*done)(void *), void *ctx);
template <class F>
int poll_until(golhip_t h, const char *what, F &&done) {
    return poll_until_fn(h, what, [](void *c) -> int { return (*static_cast<F *>(c))(); }, &done);
}
void strip_bounds(int64_t height, int world, int rank, int64_t &y0, int64_t &rows);
// A device-to-host copy on stream st into memory the caller owns (pageable: the copy blocks the host
// until the stream's earlier work is done).  On a handle whose work can wait on RCCL the stream is
// first waited for with the deadline (a stuck transfer then fails the call instead of blocking the
// host inside the copy for ever).
int copy_to_host(golhip_t h, void *dst, const void *src, size_t bytes, hipStream_t st);
// ncclCommAbort(comm) bounded by ms: true when it returned in time.  The abort makes RCCL kernels
// spinning on a transfer exit, but it also waits for the device work its frees depend on -- a
// stream stuck on something else (a hung kernel, a host callback) would hold it for ever, so it
// runs on a helper thread that is left behind (detached) when the deadline passes.
bool comm_abort_within(ncclComm_t comm, int64_t ms);
int exchange_halos(golhip_t h, int K, bool record_ready = true);
int reduce_u64(golhip_t h, const std::vector<unsigned long long *> &bufs, size_t n, uint64_t *out);
void release_rccl_ops(golhip_t h);
int sync_all(golhip_t h);

// ---- golhip_engine.hip: shards, creation --------------------------------------------------------
int64_t lcm64(int64_t a, int64_t b);
int validate_geometry(int width, int height, int world, int k);
int setup_engine(golhip_t h, int width, int height, int world, int k);
int check_device_arch(golhip_t h, int device);
int create_common(golhip_t h);
// drain_ms > 0 (a handle whose work can wait on RCCL): wait at most that long, in all, for the
// shard's streams; a stream still busy after it is left to the process's teardown, and its memory
// is not freed under it.
void free_shard(Shard &s, int64_t drain_ms = 0, bool comm_failed = false);

// ---- engine_plan.hip: the launch planner --------------------------------------------------------
// Rows per strip the planner ranks depths by: the largest strip, ceil(height / strips) (every rank
// of a rank-mode board plans the same depths).
int64_t strip_plan_rows(int64_t height, int strips);
inline int64_t plan_rows(golhip_t h) { return strip_plan_rows(h->height, h->world_size); }
int pick_k(int n);
double launch_rate_tcups(int K, double cells = 0.0);
int best_rate_k(int kmax, double cells);
int plan_first_k(int64_t n, int kmax, double cells);
int slab_first_k(int64_t n, int kmax);
int64_t auto_band(golhip_t h, int64_t rows_total, int K, int64_t reserve_waves = 0, bool counting = false);
int pick_split(golhip_t h, int64_t rows_total, int K);
struct RegKernel {
    int kind = 0;  // 0 none (streaming), 2 gol_tile, 3 gol_slab
    int T = 0, W = 0, S = 0, NC = 4;
    int out_rows() const { return T; }  // output rows per tile / slab
};
RegKernel pick_reg_kernel(golhip_t h, int64_t rows_total, int K, bool counting);
// sh (nullable): the shard launched on, for stable-slab skipping of its slab launches; par: the
// input buffer's parity (the slab flags' parity); act_reset_first: recompute the flags even if they
// look valid (a captured graph's first launch)
hipError_t launch_auto(golhip_t h, int K, const uint32_t *in, uint32_t *out, const StencilParams &p,
                       unsigned long long *slots, hipStream_t s, Shard *sh = nullptr, int par = 0,
                       bool act_reset_first = false);
// The flag arrays a K-deep launch of this single-strip board needs for stable-slab skipping
// (allocated outside any graph capture); GOLHIP_OK when none are needed.
int ensure_activity(golhip_t h, Shard &s, int K, bool counting);
StencilParams make_params(golhip_t h, const Shard &s, int K, int64_t r0b, int64_t r0e, int64_t r1b,
                          int64_t r1e, int64_t reserve_waves = 0, bool counting = false);
bool small_board(double cells, int K);
// The launch sequence of one golhip_step call (also exported as golhip_launch_plan): small boards
// replay graphs of M launches of the deepest depth, then plan the tail; large boards run the
// best-rate depth in bulk and plan the last < 2 bulk depths with plan_first_k.
// next() returns 0 for one graph replay (M x Kfull generations), else one launch's depth.
struct LaunchPlanner {
    double cells;
    int Kfull, Kbulk, M, Mbig, last_M = 0;
    bool graphs;
    int64_t left;
    bool keep_last;  // the last generation is always a plain launch (it writes the flips)
    bool reg = false;  // register-slab board: tails by fewest launches (slab_first_k)
    LaunchPlanner(double cells_, int k, int64_t turns, bool small, bool fixed = false,
                  bool keep_last_ = false, int window = 4096, bool stream = false, bool reg_ = false);
    int next();
    // true when this plan replays at least one graph (the call's counts then come from per-replay
    // copies, which pinned host memory makes slower: run_steps)
    bool replays() const { return graphs; }
};

// ---- engine_cells.hip ---------------------------------------------------------------------------
// Kernel variants whose launches can write a generation's flips beside their output.
bool variant_writes_flips(int v);
int ensure_extract_scratch(golhip_t h, Shard &s, int64_t rows, int64_t slots);

// Whether golhip_step runs this single-strip board with the whole-board kernel (stencil_board.hip),
// and its shape.
bool board_applies(golhip_t h, int *W = nullptr, int *R = nullptr);

// ---- golhip_engine.hip: the step loop -----------------------------------------------------------
int run_steps(golhip_t h, int64_t turns, uint64_t *alive_per_turn, bool ring);

}  // namespace golhip
