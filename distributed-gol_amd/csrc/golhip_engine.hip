// golhip_engine.hip -- host side of libgolhip: handles, device memory, streams, RCCL halo
// exchange and the C ABI declared in include/golhip.h.
//
// Reference roles this file takes over (Oliver-Cairns/distributed-gol):
//   * broker/broker.go:37-56  publish(): split the rows into strips -> golhip_strip_bounds(),
//     one strip per GPU (the reference's 4 servers become the node's GPUs);
//   * broker/broker.go:58-84,157-180  subscriberLoop/Publish: fan the FULL world out every turn
//     and stitch the strips back -> the board stays resident in HBM, only k halo rows per strip
//     edge move per k generations, by RCCL send/recv over xGMI on a dedicated comm stream that
//     overlaps the interior update;
//   * broker/broker.go:124-155  CheckStates/Pause (worldSave, turn) -> the resident board and
//     golhip_turn()/golhip_set_turn().
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/golhip.h"
#include "golhip_internal.hpp"

using golhip::StencilParams;

namespace {

constexpr int kVersion = 101;
// Generations of per-turn counts finalized per launch (golhip_set_count_window changes it; at
// least the graph length kGraphGens: tests shrink it to exercise flushes).
constexpr int kCountWindowDefault = 4096;
constexpr int kCountWindowMin = 128;
constexpr bool kTuningBuildEngine = golhip::kTuningBuild;
// The register slab runs boards on which the streaming kernel would have at most this many
// minimal-band (max(K, 8)-row) waves per CU.  Round 4 sweep (profiles/r04/r04mid_tune_mid.log,
// 512 / 256 turns, every count equal): the slab is 7-11 % faster than streaming up to 16384^2
// without counts (12288^2 2.82 vs 3.14 us/turn, 16384^2 4.09 vs 4.40), even at 20480^2, and
// slower there with counts (9.33 vs 8.39); 16384^2 has 36 such waves per CU, 20480^2 55.
constexpr int64_t kSlabMaxWaves1PerCu = 40;
// calls up to this many turns return their counts pinned: shorter than the planner's smallest
// replayed graph (128 generations), whose per-replay count copy into pinned memory cost more than
// the one device-to-host copy it saves (1600 turns at 512^2: 0.570 -> 0.705 us/turn with 4096)
constexpr int64_t kPinnedCountTurns = 127;
constexpr int64_t kStampWaves = 1 << 20;  // tuning build: waves of the per-wave stamp buffer
// Default deadline of a host wait on RCCL-dependent work and of the communicator's set-up
// (golhip_set_comm_timeout(NULL, ms) changes it for later creates): well under the 600 s a driver
// gives a whole bench run, far above any legitimate wait (an 8-rank init takes seconds, a K-row
// exchange microseconds; stencil work queued by the host is added to each wait by its model).
std::atomic<int64_t> g_comm_timeout_ms{120000};

struct Shard {
    int device = 0;
    int rank = 0;
    int64_t y0 = 0, rows = 0;
    hipStream_t compute = nullptr, comm = nullptr;
    hipStream_t edge = nullptr;  // boundary bands of a split board, concurrent with the interior
    hipEvent_t ev_ready = nullptr, ev_halo = nullptr, ev_edge = nullptr;
    // tuning (GOLHIP_JOIN=1): the split step's join of the boundary bands as a stream write/wait
    // of a device word instead of an event wait
    uint32_t *join_flag = nullptr;
    uint32_t join_seq = 0;
    uint32_t *buf[2] = {nullptr, nullptr};  // allocation base (halo rows first)
    unsigned long long *slots = nullptr;    // count_window x kCountSlots
    unsigned long long *scratch_u64 = nullptr;
    // the call's per-turn counts: dev_counts, or on a one-shard engine without RCCL for calls of
    // at most kPinnedCountTurns (127) turns pin_counts (pinned host memory, hipHostMalloc coherent): the
    // count finalize writes it directly and the call returns without a device-to-host copy
    // (configs[0], 100 turns: the copy and its dispatch gap were ~17 of ~85 us per call)
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
    hipGraphExec_t exec = nullptr;
};

}  // namespace

struct golhip_engine {
    int64_t width = 0, height = 0, L = 0, pitch = 0;
    int32_t wd = 0;
    int world_size = 1;
    int k = 1, halo = 0, band_rows = 0;
    int tail_bands = 0, tail_rows = 0;  // golhip_set_tail_bands: graded bands (0 = uniform)
    int count_window = 4096;  // generations per count-window finalize
    int variant = golhip::kVariantProd;  // fastest measured per depth (golhip_internal.hpp)
    int cus = 0;                 // compute units of the first device (grid sizing)
    bool fixed_k = false;        // golhip_set_fixed_k: long runs launch exactly k deep
    bool track_flips = false;    // golhip_track_flips: every step ends with a flips-writing launch
    bool diff_valid = false;     // shards' diffbuf holds the flips of the last generation
    int64_t ring_cap = 0;        // turns per golhip_step_flips call (flips ring slots)
    int64_t ring_turns = 0;      // turns held in the ring by the last golhip_step_flips
    int waves_per_cu[golhip::kMaxK + 1][golhip::kNumVariants] = {};  // occupancy cache per (K, variant)
    bool rank_mode = false;
    // golhip_create_rank_host: the caller's host transport instead of RCCL, with pinned host
    // buffers for the 4 K-row transfers of an exchange (halo rows x pitch words each)
    bool host_comm_on = false;
    golhip_host_comm host_comm{};
    void *hc_buf[4] = {nullptr, nullptr, nullptr, nullptr};
    bool split = false;  // board held as halo'd row strips (world > 1, or GOLHIP_RING_SELF)
    // tuning build only (GOLHIP_SPLIT / GOLHIP_TILE / GOLHIP_SLAB); the production build keeps the
    // automatic choice
    int force_split = 0;  // 0 = automatic
    int force_tile = -1;  // -1 automatic, 0 never, T > 0 always (tile height T)
    int force_slab = -1;  // -1 automatic, 0 never, [NC*10000 +] W*100 + S always (slab shape)
    bool edge_prio = false;   // tuning: comm/edge streams at high priority (GOLHIP_EDGE_PRIO)
    bool edge_first = false;  // tuning: boundary bands submitted before the interior
    // the boundary bands' waves raise their issue priority (StencilParams::prio); tuning knob
    // GOLHIP_EDGE_SETPRIO=0 turns it off for A/B
    int edge_setprio = 1;
    int join_mode = 0;  // tuning (GOLHIP_JOIN): 0 event wait, 1 stream write/wait of a device word
    int graph_mode = -1;  // golhip_set_graphs: -1 automatic, 0 never, 1 whenever the plan allows
    // RCCL fail-fast (rank mode): every host wait on work that can depend on an RCCL transfer polls
    // ncclCommGetAsyncError against a deadline and fails the handle when it passes
    // (golhip_set_comm_timeout); the communicator is non-blocking, so no RCCL call blocks the host
    int64_t comm_timeout_ms = 0;
    double queued_s = 0.0;  // modelled seconds of stencil work queued since the last full sync
    bool comm_failed = false;
    bool comm_setup_done = false;  // the communicator's set-up completed (no abort after it)
    // depth of the boundary bands the last split block ran on the edge stream (0: none, e.g. a strip
    // shorter than 3K or a non-split launch): its rows [0, K) and [rows - K, rows) are exactly what
    // the next exchange sends, so with K' <= edge_k that exchange waits only for those bands
    int edge_k = 0;
    std::string comm_pending;  // the last RCCL operation enqueued (rank, peers, K, bytes)
    // GOLHIP_RING_SELF=2 (test hook): every step's work ends in a 20 s stall of the compute stream
    // (a rank whose device work does not finish in time); nothing RCCL is queued behind it
    int test_ring_mode = 1;
    // tuning build, GOLHIP_VARIANT=stamp: per-wave timestamps of the last single-strip launch
    uint64_t *stamp_buf = nullptr;
    int64_t stamp_waves = 0;
    int stamp_words = 4;  // uint64 per wave of the last stamped launch (gol_slab2: 8)
    std::vector<Shard> shards;
    int cur = 0;
    bool prev_valid = false;
    int64_t turn = 0;
    std::string err;
    // graph replay of step blocks (single strip, small boards)
    std::vector<GraphEntry> graphs;
    unsigned long long *g_counts = nullptr;  // counts written by a counting graph
    // timing
    bool timing = false;
    std::vector<TimingPair> tpool;
    size_t tused = 0;
    double tms = 0.0;
    int64_t tlaunches = 0, tgens = 0;

    uint32_t *row0(const Shard &s, int which) const {
        return s.buf[which] + (int64_t)halo * pitch;
    }
    int64_t rep() const { return L / width; }
};

namespace {

thread_local std::string g_create_error;  // golhip_last_error(NULL): why the last create failed

int fail(golhip_t h, int code, const char *fmt, ...) {
    if (h) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        h->err = buf;
    }
    return code;
}

#define HIPCHK(h, expr)                                                                     \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail((h), e_ == hipErrorOutOfMemory ? GOLHIP_ERR_OOM : GOLHIP_ERR_HIP,   \
                        "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

// ---- RCCL fail-fast --------------------------------------------------------------------------
// True when device work of this handle can wait on an RCCL transfer (rank mode over RCCL: the
// boundary bands wait for the halo event, the compute stream for the boundary bands, counts for
// the all-reduce).  Only then do host waits poll; everything else synchronises directly.
bool rccl_waits(golhip_t h) { return h->rank_mode && h->split && !h->host_comm_on; }

// Fail the call with the pending operation named; the handle refuses device work afterwards
// (comm_failed).  Before the communicator's set-up has completed nothing of it runs on the device,
// and ncclCommAbort stops its bootstrap.  After it, the communicator is NOT aborted: ncclCommAbort
// frees its device state while RCCL kernels queued on this rank's streams behind the stuck one may
// still run -- measured on the one-GPU box, an abort with exchanges queued behind a stalled comm
// stream left the GPU with a memory-access fault (profiles/r04/failfast.txt).  The communicator
// and the strips are left in place (golhip_destroy leaks what a stuck stream may still touch) and
// the caller is expected to end the process (bench.py exits at once); the process teardown
// removes its queues.
int comm_abort(golhip_t h, const char *why, ncclResult_t state) {
    const bool before_setup = !h->comm_setup_done;
    if (before_setup)
        for (auto &s : h->shards)
            if (s.comm_nccl) {
                (void)ncclCommAbort(s.comm_nccl);
                s.comm_nccl = nullptr;
            }
    h->comm_failed = true;
    return fail(h, GOLHIP_ERR_RCCL, "rank %d of %d: %s: %s (communicator state: %s); %s",
                h->shards.empty() ? -1 : h->shards[0].rank, h->world_size, why,
                h->comm_pending.empty() ? "no RCCL operation pending" : h->comm_pending.c_str(),
                ncclGetErrorString(state),
                before_setup ? "communicator aborted"
                             : "communicator left in place, end the process (RCCL work may still be queued)");
}

using Clock = std::chrono::steady_clock;
// Deadline of a wait: the handle's timeout plus 10x the modelled time of the stencil work the host
// queued since the last full sync (a long golhip_step of a big board is not a hang).
int64_t wait_budget_ms(golhip_t h) {
    return (int64_t)std::min((double)h->comm_timeout_ms + 10.0 * h->queued_s * 1e3, 3.6e6);
}

// Poll `done` (0 = finished, 1 = not yet, < 0 = error code already set) until it finishes, the
// communicator reports an asynchronous error, or the deadline passes.
template <class F>
int poll_until(golhip_t h, const char *what, F &&done) {
    const int64_t budget_ms = wait_budget_ms(h);
    const Clock::time_point deadline = Clock::now() + std::chrono::milliseconds(budget_ms);
    int spins = 0;
    for (;;) {
        const int r = done();
        if (r <= 0) return r;
        for (auto &s : h->shards) {
            ncclResult_t st = ncclSuccess;
            if (s.comm_nccl && ncclCommGetAsyncError(s.comm_nccl, &st) == ncclSuccess &&
                st != ncclSuccess && st != ncclInProgress)
                return comm_abort(h, what, st);
        }
        if (Clock::now() > deadline) {
            ncclResult_t st = ncclInProgress;
            if (!h->shards.empty() && h->shards[0].comm_nccl)
                (void)ncclCommGetAsyncError(h->shards[0].comm_nccl, &st);
            char buf[160];
            std::snprintf(buf, sizeof buf, "%s did not complete within %lld ms", what,
                          (long long)budget_ms);
            return comm_abort(h, buf, st);
        }
        if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(spins > 4096 ? 200 : 20));
    }
}

// hipStreamSynchronize, bounded by the RCCL deadline in rank mode.
int wait_stream(golhip_t h, hipStream_t st) {
    if (h->comm_failed)
        return fail(h, GOLHIP_ERR_RCCL, "the communicator failed earlier: %s", h->comm_pending.c_str());
    if (!rccl_waits(h)) {
        const hipError_t e = hipStreamSynchronize(st);
        if (e != hipSuccess)
            return fail(h, GOLHIP_ERR_HIP, "hipStreamSynchronize: %s", hipGetErrorString(e));
        return GOLHIP_OK;
    }
    return poll_until(h, "device work behind the RCCL transfers", [&]() -> int {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) return 0;
        if (e == hipErrorNotReady) return 1;
        return fail(h, GOLHIP_ERR_HIP, "hipStreamQuery: %s", hipGetErrorString(e));
    });
}

// After a non-blocking RCCL call: wait until the communicator has finished setting it up
// (ncclInProgress -> ncclSuccess) before the next RCCL call, bounded by the deadline.
int comm_ready(golhip_t h, ncclComm_t c, const char *what) {
    return poll_until(h, what, [&]() -> int {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t q = ncclCommGetAsyncError(c, &st);
        if (q != ncclSuccess) return comm_abort(h, what, q);
        if (st == ncclInProgress) return 1;
        return st == ncclSuccess ? 0 : comm_abort(h, what, st);
    });
}

#define SYNCCHK(h, stream)                      \
    do {                                        \
        int rc_ = wait_stream((h), (stream));   \
        if (rc_) return rc_;                    \
    } while (0)

// An RCCL call on a non-blocking communicator: ncclInProgress is not an error (comm_ready waits).
#define NCCLCALL(h, what, expr)                                                                   \
    do {                                                                                          \
        ncclResult_t r_ = (expr);                                                                 \
        if (r_ != ncclSuccess && r_ != ncclInProgress) return comm_abort((h), (what), r_);        \
    } while (0)

int64_t lcm64(int64_t a, int64_t b) { return a / std::gcd(a, b) * b; }

void strip_bounds(int64_t height, int world, int rank, int64_t &y0, int64_t &rows) {
    // balanced contiguous split (the reference's publish() splits ImageSize/numServers and hands
    // the remainder to the first strips, broker/broker.go:38-46; same coverage here, any height)
    y0 = height * rank / world;
    rows = height * (rank + 1) / world - y0;
}

int check_device_arch(golhip_t h, int device) {
    hipDeviceProp_t prop;
    HIPCHK(h, hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(h, GOLHIP_ERR_NODEV, "device %d is %s, libgolhip is built for gfx950", device,
                    prop.gcnArchName);
    return GOLHIP_OK;
}

// Extraction scratch for `rows` rows (a tall board of `slots` slots for the flips ring): grown,
// never shrunk -- a growth frees and reallocates, so it only happens for a larger ring.
int ensure_extract_scratch(golhip_t h, Shard &s, int64_t rows, int64_t slots) {
    if (rows <= s.ex_rows_cap && slots <= s.ex_slots_cap) return GOLHIP_OK;
    HIPCHK(h, hipSetDevice(s.device));
    SYNCCHK(h, s.compute);
    if (!s.ex_block_sums)
        HIPCHK(h, hipMalloc(&s.ex_block_sums, sizeof(unsigned long long) * golhip::kScanBlocks));
    if (rows > s.ex_rows_cap) {
        if (s.ex_rowcounts) HIPCHK(h, hipFree(s.ex_rowcounts));
        if (s.ex_offsets) HIPCHK(h, hipFree(s.ex_offsets));
        s.ex_rowcounts = nullptr;
        s.ex_offsets = nullptr;
        HIPCHK(h, hipMalloc(&s.ex_rowcounts, sizeof(uint32_t) * (size_t)rows));
        HIPCHK(h, hipMalloc(&s.ex_offsets, sizeof(unsigned long long) * (size_t)(rows + 1)));
        s.ex_rows_cap = rows;
    }
    if (slots > s.ex_slots_cap) {
        if (s.ex_slot_counts) HIPCHK(h, hipFree(s.ex_slot_counts));
        s.ex_slot_counts = nullptr;
        HIPCHK(h, hipMalloc(&s.ex_slot_counts, sizeof(unsigned long long) * (size_t)slots));
        s.ex_slots_cap = slots;
    }
    return GOLHIP_OK;
}

constexpr int64_t kStageBytes = 64ll << 20;

int alloc_shard(golhip_t h, Shard &s) {
    HIPCHK(h, hipSetDevice(s.device));
    HIPCHK(h, hipStreamCreateWithFlags(&s.compute, hipStreamNonBlocking));
    // comm and edge streams at the default priority: high-priority queues for them (so the bands'
    // few workgroups dispatch ahead of the interior's) ran the 65536^2 ring of one 16 % SLOWER over
    // 1000 turns (r04g vs r04f, profiles/r04/r04h_edge_ab_p*.log); kept as a tuning knob
    int lo_prio = 0, hi_prio = 0;
    HIPCHK(h, hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
    const int edge_prio = h->edge_prio ? hi_prio : lo_prio;
    HIPCHK(h, hipStreamCreateWithPriority(&s.comm, hipStreamNonBlocking, edge_prio));
    HIPCHK(h, hipStreamCreateWithPriority(&s.edge, hipStreamNonBlocking, edge_prio));
    HIPCHK(h, hipEventCreateWithFlags(&s.ev_ready, hipEventDisableTiming));
    HIPCHK(h, hipEventCreateWithFlags(&s.ev_halo, hipEventDisableTiming));
    HIPCHK(h, hipEventCreateWithFlags(&s.ev_edge, hipEventDisableTiming));
    if (kTuningBuildEngine) {
        HIPCHK(h, hipMalloc(&s.join_flag, sizeof(uint32_t)));
        HIPCHK(h, hipMemsetAsync(s.join_flag, 0, sizeof(uint32_t), s.compute));
    }
    const size_t words = (size_t)(s.rows + 2 * (int64_t)h->halo) * (size_t)h->pitch;
    for (int i = 0; i < 2; ++i) {
        HIPCHK(h, hipMalloc(&s.buf[i], words * sizeof(uint32_t)));
        HIPCHK(h, hipMemsetAsync(s.buf[i], 0, words * sizeof(uint32_t), s.compute));
    }
    HIPCHK(h, hipMalloc(&s.slots, sizeof(unsigned long long) * h->count_window * golhip::kCountSlots));
    HIPCHK(h, hipMemsetAsync(s.slots, 0,
                             sizeof(unsigned long long) * h->count_window * golhip::kCountSlots,
                             s.compute));
    HIPCHK(h, hipMalloc(&s.scratch_u64, sizeof(unsigned long long) * 4));
    // the transfer stage: the shard's whole byte board if it fits in kStageBytes, else row chunks
    // of it (a byte row is the widest unit any transfer stages)
    // (GOLHIP_STAGE_BYTES, read at create, shrinks it: tests force multi-chunk transfers)
    int64_t cap = kStageBytes;
    if (const char *e = std::getenv("GOLHIP_STAGE_BYTES")) cap = std::max<int64_t>(1, std::atoll(e));
    // at least one row of every transfer unit: a byte row (width bytes) and a uint64 word row
    // (8 * ceil(width / 64) bytes, larger than a byte row for widths below 8)
    const int64_t row_unit = std::max<int64_t>(h->width, 8 * ((h->width + 63) / 64));
    s.stage_bytes = std::max<int64_t>(row_unit, std::min<int64_t>(cap, s.rows * h->width));
    HIPCHK(h, hipMalloc(&s.stage, (size_t)s.stage_bytes));
    SYNCCHK(h, s.compute);
    return ensure_extract_scratch(h, s, s.rows, 1);
}

// drain_ms > 0 (a handle whose work can wait on RCCL): wait at most that long for the streams; a
// stream still busy after it (an RCCL transfer nothing will ever match) is left to the process's
// teardown, and its memory is not freed under it.
void free_shard(Shard &s, int64_t drain_ms = 0, bool comm_failed = false) {
    (void)hipSetDevice(s.device);
    bool drained = true;
    for (hipStream_t st : {s.compute, s.comm, s.edge}) {
        if (!st) continue;
        if (drain_ms <= 0) {
            (void)hipStreamSynchronize(st);
            continue;
        }
        const Clock::time_point end = Clock::now() + std::chrono::milliseconds(drain_ms);
        hipError_t e;
        while ((e = hipStreamQuery(st)) == hipErrorNotReady && Clock::now() < end)
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        drained = drained && e != hipErrorNotReady;
    }
    // a failed communicator is left alone (comm_abort); a stuck stream keeps what it may touch
    if (s.comm_nccl && drained && !comm_failed) (void)ncclCommDestroy(s.comm_nccl);
    if (!drained) {
        s = Shard{};
        return;
    }
    for (auto &b : s.buf)
        if (b) (void)hipFree(b);
    if (s.slots) (void)hipFree(s.slots);
    if (s.scratch_u64) (void)hipFree(s.scratch_u64);
    if (s.dev_counts) (void)hipFree(s.dev_counts);
    if (s.pin_counts) (void)hipHostFree(s.pin_counts);
    for (void *q : {(void *)s.diffbuf, (void *)s.ring, (void *)s.ex_rowcounts, (void *)s.ex_offsets,
                    (void *)s.ex_slot_counts, (void *)s.ex_xy, (void *)s.stage,
                    (void *)s.ex_block_sums})
        if (q) (void)hipFree(q);
    if (s.ev_ready) (void)hipEventDestroy(s.ev_ready);
    if (s.ev_halo) (void)hipEventDestroy(s.ev_halo);
    if (s.ev_edge) (void)hipEventDestroy(s.ev_edge);
    if (s.join_flag) (void)hipFree(s.join_flag);
    if (s.compute) (void)hipStreamDestroy(s.compute);
    if (s.comm) (void)hipStreamDestroy(s.comm);
    if (s.edge) (void)hipStreamDestroy(s.edge);
    s = Shard{};
}

// Rows per strip the launch planner ranks depths by: the largest strip of the board,
// ceil(height / strips).  Each launch of a split board exchanges K-row halos, so in rank mode every
// rank MUST run the same depth sequence (a different K on one rank would mismatch the
// ncclSend/ncclRecv sizes): planning from a quantity every rank shares -- not the rank's own,
// possibly one row shorter, strip -- guarantees that (golhip_launch_plan uses the same rows).
int64_t strip_plan_rows(int64_t height, int strips) { return (height + strips - 1) / strips; }
int64_t plan_rows(golhip_t h) { return strip_plan_rows(h->height, h->world_size); }

// Kernel variants whose launches can write a generation's flips beside their output (the
// production drift family; gol_step1 at K = 1).  The A/B-experiment variants cannot.
bool variant_writes_flips(int v) {
    return v == golhip::kVariantProd || v == golhip::kVariantDriftLds || v == golhip::kVariantDrift62 ||
           v == golhip::kVariantPre63 || v == golhip::kVariantProdMask;
}

int validate_geometry(int width, int height, int world, int k) {
    if (width <= 0 || height <= 0 || world <= 0) return GOLHIP_ERR_ARG;
    if (k < 1 || k > golhip::kMaxK) return GOLHIP_ERR_ARG;
    // row strips must be able to send k halo rows to each neighbour (a single strip wraps
    // rows modulo the height and needs nothing)
    if (world > 1 && (int64_t)height / world < k) return GOLHIP_ERR_ARG;
    return GOLHIP_OK;
}

int setup_engine(golhip_t h, int width, int height, int world, int k) {
    h->width = width;
    h->height = height;
    h->L = lcm64(width, 128);
    h->wd = (int32_t)(h->L / 32);
    h->pitch = h->wd;
    h->world_size = world;
    h->k = k;
    h->split = world > 1;
    h->halo = h->split ? k : 0;
    h->count_window = kCountWindowDefault;
    h->comm_timeout_ms = g_comm_timeout_ms.load();
#ifdef GOLHIP_TUNING
    // The tuning build's selectors (read at create).  The production library reads none of them:
    // a stray variable cannot change its kernels (the setters below are the explicit interface).
    if (const char *e = std::getenv("GOLHIP_BAND_ROWS")) h->band_rows = std::atoi(e);
    // measurement knob (scripts/pmc_passes.sh): every bulk launch exactly k deep, as
    // golhip_set_fixed_k(h, 1) -- the planner would otherwise run its fastest depth <= k
    if (const char *e = std::getenv("GOLHIP_FIXED_K")) h->fixed_k = std::atoi(e) != 0;
    if (const char *e = std::getenv("GOLHIP_COUNT_WINDOW"))
        h->count_window = std::max(kCountWindowMin, std::atoi(e));
    if (const char *e = std::getenv("GOLHIP_GRAPHS")) h->graph_mode = std::atoi(e) != 0;
    if (const char *e = std::getenv("GOLHIP_SPLIT")) h->force_split = std::atoi(e);
    if (const char *e = std::getenv("GOLHIP_TILE")) h->force_tile = std::atoi(e);
    if (const char *e = std::getenv("GOLHIP_SLAB")) h->force_slab = std::atoi(e);
    if (const char *e = std::getenv("GOLHIP_EDGE_PRIO")) h->edge_prio = std::atoi(e) != 0;
    if (const char *e = std::getenv("GOLHIP_EDGE_FIRST")) h->edge_first = std::atoi(e) != 0;
    if (const char *e = std::getenv("GOLHIP_EDGE_SETPRIO")) h->edge_setprio = std::atoi(e) != 0;
    if (const char *e = std::getenv("GOLHIP_JOIN")) h->join_mode = std::atoi(e);
    if (const char *e = std::getenv("GOLHIP_VARIANT"))
        h->variant = std::strcmp(e, "chain") == 0     ? golhip::kVariantChain
                     : std::strcmp(e, "skew") == 0   ? golhip::kVariantSkew
                     : std::strcmp(e, "skew2") == 0  ? golhip::kVariantSkewD2
                     : std::strcmp(e, "chain2") == 0 ? golhip::kVariantChainD2
                     : std::strcmp(e, "skewlds") == 0 ? golhip::kVariantSkewLdsPf
                     : std::strcmp(e, "skewlds2") == 0 ? golhip::kVariantSkewLdsD2
                     : std::strcmp(e, "chainlds2") == 0 ? golhip::kVariantChainLdsD2
                     : std::strcmp(e, "chainlds") == 0 ? golhip::kVariantChainLdsPf
                     : std::strcmp(e, "driftzip") == 0 ? golhip::kVariantDriftZip
                     : std::strcmp(e, "drift62") == 0 ? golhip::kVariantDrift62
                     : std::strcmp(e, "driftnf") == 0 ? golhip::kVariantDriftNoFill
                     : std::strcmp(e, "driftlds") == 0 ? golhip::kVariantDriftLds
                     : std::strcmp(e, "pre63") == 0 ? golhip::kVariantPre63
                     : std::strcmp(e, "prodmask") == 0 ? golhip::kVariantProdMask
                     : std::strcmp(e, "stamp") == 0 ? golhip::kVariantStamp
                                                       : golhip::kVariantProd;  // prod
#endif
    return GOLHIP_OK;
}

// Largest supported launch depth <= n.
int pick_k(int n) {
    int kk = 1;
    for (int c : {32, 24, 20, 16, 14, 12, 10, 8, 6, 4, 2, 1})  // 24 / 20: tuning build only
        if (c <= n && golhip::stencil_k_supported(c)) {
            kk = c;
            break;
        }
    return kk;
}

// Measured throughput of a K-generation launch of the production variant, T cell-updates/s, on a
// pre-heated chip (profiles/r02/r02ad_bulk_depth.txt and the k sweeps of the round-2 bench lines:
// 65536^2, 256+ generations per depth; 6 interpolated), and the fixed cost of one launch (kernel
// boundary + the last round's drain, us).  Boards of >= 2^35 cells per strip have their own
// ranking: at 262144^2 (2096-row bands) K = 16 runs 129 vs 122 at K = 12, while every smaller
// streaming board measured runs K = 12 faster (16384^2 +17 %, 32768^2 +9.5 %, 65536^2 +2.3 %,
// 131072^2 +3 %: r02ae/r02af).  Only the ranking and the ratios matter to the planner.
// Round 3: with the pre-shifted geometry on every non-counting launch, strips of 2^31 .. 2^35
// cells (65536^2 and up) rank K = 14 first: 125.5-125.8 vs 123.8-124.3 (K = 12) and 124.0-124.8
// (K = 16) TCUPS in a lockstep A/B and two default-bench k sweeps (profiles/r03/r03ae_*,
// r03ab_bench.json, r03ah_bench.json); smaller streaming boards (graph replays) keep K = 12.
constexpr double kLargeStripCells = 34359738368.0;  // 2^35
constexpr double kMidStripCells = 2147483648.0;     // 2^31
double launch_rate_tcups(int K, double cells = 0.0) {
    const bool large = cells >= kLargeStripCells;
    if (!large && cells >= kMidStripCells) {
        switch (K) {
            case 12: return 124.1;
            case 14: return 125.6;
            case 16: return 124.4;
            default: break;
        }
    }
    switch (K) {
        case 1: return 22.8;
        case 2: return 35.4;
        case 4: return 68.4;
        case 6: return 92.0;
        case 8: return 115.4;
        case 10: return 116.7;  // 120.9 on sparse boards; 20 turns as 10 + 10 ran 97.7 TCUPS vs 111.8 as 12 + 8
        case 12: return large ? 122.0 : 123.6;
        case 14: return large ? 125.0 : 122.1;
        case 16: return large ? 129.0 : 120.2;
        case 32: return 100.9;
        default: return 50.0;
    }
}

// The depth <= kmax with the highest measured rate: the bulk depth of long runs (k is the maximum
// depth; deeper is not always faster -- 12 and 14 keep 5 waves per SIMD, 16 keeps 4, and the
// band trapezoid of a K-deep launch grows with K).
int best_rate_k(int kmax, double cells) {
    int best = 1;
    for (int K = 1; K <= kmax; ++K)
        if (golhip::stencil_k_supported(K) && launch_rate_tcups(K, cells) > launch_rate_tcups(best, cells))
            best = K;
    return best;
}
constexpr double kLaunchOverheadUs = 4.0;

// Launch depths for `n` remaining generations (n < 2 * kmax): the sequence of supported depths
// <= kmax summing to n with the least modelled time sum(cells * K / rate(K) + overhead).  The
// greedy largest-first split ran 20 turns as 16 + 4 (the 4-level launch at half the rate);
// this gives 12 + 8.  The first depth of the plan is returned; callers re-plan each launch.
int plan_first_k(int64_t n, int kmax, double cells) {
    if (n <= 0) return 1;
    const int N = (int)n;
    std::vector<double> best(N + 1, 1e300);
    std::vector<int> first(N + 1, 1);
    best[0] = 0.0;
    for (int m = 1; m <= N; ++m)
        for (int K : {32, 16, 14, 12, 10, 8, 6, 4, 2, 1}) {
            if (K > m || K > kmax || !golhip::stencil_k_supported(K)) continue;
            const double c = best[m - K] + cells * K / (launch_rate_tcups(K, cells) * 1e6) + kLaunchOverheadUs;
            if (c < best[m]) {
                best[m] = c;
                first[m] = K;
            }
        }
    return first[N];
}

// Rows per wave band of a stencil launch over rows_total rows.  reserve_waves: resident wave
// slots to leave free for a concurrent launch (the boundary bands of a split board).
int64_t auto_band(golhip_t h, int64_t rows_total, int K, int64_t reserve_waves = 0,
                  bool counting = false) {
    if (h->band_rows > 0) return h->band_rows;
    const int64_t per = golhip::chunk_words(K, h->variant, counting);
    const int64_t nchunks = (h->wd + per - 1) / per;
    // Fill the chip in whole rounds of resident waves (CUs x resident waves per CU), so every
    // SIMD gets the same number of equal bands.
    if (h->cus == 0) {
        hipDeviceProp_t prop;
        h->cus = hipGetDeviceProperties(&prop, h->shards[0].device) == hipSuccess
                     ? prop.multiProcessorCount
                     : 256;
    }
    int &wpc = h->waves_per_cu[K][h->variant];
    if (wpc == 0) wpc = golhip::stencil_waves_per_cu(K, h->variant);
    // The one-generation kernel (K = 1, production variant) is HBM-bound: it runs best with 2
    // long-streaming waves per SIMD in one round (measured: 2/SIMD 21.9, 4/SIMD 21.1, 1/SIMD
    // 19.6 TCUPS at 65536^2; uneven rounds lose 10-20 %, profiles/r01_tune_step1.txt).
    const bool step1 = K == 1 && golhip::variant_is_production_family(h->variant);
    const int64_t capacity = (int64_t)h->cus * (step1 ? golhip::kStep1WavesPerCu : wpc);
    constexpr int64_t kMaxBand = 4096;
    const bool skew = h->variant == golhip::kVariantSkew || h->variant == golhip::kVariantSkewD2 ||
                      h->variant == golhip::kVariantSkewLdsPf ||
                      h->variant == golhip::kVariantSkewLdsD2;
    const int64_t lag = skew ? 3 * K - 1 : 2 * K;
    // A wave runs band + lag steps in blocks of 8 (the kernel's prefetch ring); bands are rounded
    // so that full bands end on a block boundary instead of computing up to 7 discarded rows.
    auto aligned = [&](int64_t b) {
        return step1 ? b : std::max<int64_t>(8, (b + lag + 7) / 8 * 8 - lag);
    };
    int64_t band;
    if (step1) {
        // Waves = bands x chunks.  At most `slots` bands are resident at once; use the fewest
        // whole rounds of `slots` bands that keep a band <= kMaxBand rows and split the rows
        // evenly over them.
        const int64_t slots = std::max<int64_t>(1, (capacity - reserve_waves) / nchunks);
        const int64_t rounds = (rows_total + slots * kMaxBand - 1) / (slots * kMaxBand);
        band = (rows_total + rounds * slots - 1) / (rounds * slots);
    } else {
        // K >= 2 (VALU-bound): bands x chunks come to just under an integer m waves per SIMD
        // (a remainder band counting by its length), m from two to four rounds of residency,
        // choosing the m with the least modelled time m x (band + K) (K ~ a wave's pipeline-fill
        // cost in rows).  Measured (profiles/r01_tune_band16.txt): GCUPS follows a sawtooth of
        // period one wave per SIMD -- at 65536^2, k = 16: 111.7 at band 264 (8.0 waves/SIMD),
        // 103.2 at band 256 (8.2), 106.5 at one round (band 528); at 262144^2 the waves just over
        // a multiple lose 5-10 % the same way.
        const int64_t simds = 4 * (int64_t)h->cus;  // gfx9: 4 SIMDs per CU
        const int64_t m0 = std::max<int64_t>(2, 2 * (int64_t)wpc / 4);
        // The concurrent boundary bands (reserve_waves waves of K rows each) are short: they count
        // by their rows of work, not as whole wave slots (a full slot each pushed the 65536-row
        // interior from 264- to 272-row bands: -2.5 % on the RCCL ring of one).
        const double work = (double)rows_total * (double)nchunks + (double)reserve_waves * K;
        // Among m within 1 % of the least cost take the largest (more, shorter bands measured
        // 3 % faster at 262144^2: band 2232 vs 3728).
        std::vector<std::pair<int64_t, double>> cand;  // (band, cost) per m
        for (int64_t m = m0; m <= 2 * m0 || cand.empty(); ++m) {
            const double slots = (double)(m * simds);
            if (slots <= 0) continue;
            const int64_t b = aligned(std::max<int64_t>(1, (int64_t)std::ceil(work / slots)));
            if (b > kMaxBand && m < 64) continue;
            cand.push_back({b, (double)m * (double)(b + K)});
        }
        double best = cand[0].second;
        for (auto &c : cand) best = std::min(best, c.second);
        band = cand[0].first;
        for (auto &c : cand)
            if (c.second <= 1.01 * best) band = c.first;
    }
    // Small boards (fewer rows than a round of minimal bands) are latency-bound: a wave's work is
    // band*K level updates plus the K(K-1) of its pipeline fill, so bands shorter than K mostly
    // add fill; K-row bands measured best (profiles/r01_tune_small_*).
    band = std::max<int64_t>(band, std::min<int64_t>(std::max(K, 8), rows_total));
    band = std::max<int64_t>(band, 1);
    if (band < rows_total) band = aligned(band);
    return std::min(band, std::max<int64_t>(rows_total, 1));
}

// Waves per (band, chunk) of a launch over rows_total rows: the level-split kernel (S = 2, 4 or 8)
// when even minimal bands leave the chip short of waves (small boards, latency-bound), else 1.
// GOLHIP_SPLIT=1/2/4/8 forces it (tests, tuning).
int pick_split(golhip_t h, int64_t rows_total, int K) {
    if (!golhip::variant_is_production_family(h->variant)) return 1;
    if (h->force_split > 0)
        return h->force_split > 1 && golhip::stencil_split_supported(K, h->force_split)
                   ? h->force_split
                   : 1;
    // measured (profiles/r01_tune_small.txt): a gain at K = 16 (-10 % per turn at 5120^2), none
    // at K = 12 and a loss at K = 8, where the lockstep barriers cost more than the shorter chain
    if (K < 16) return 1;
    const int64_t per = golhip::chunk_words(K, h->variant);
    const int64_t nchunks = (h->wd + per - 1) / per;
    const int64_t minband = std::max(K, 8);
    const int64_t waves1 = (rows_total + minband - 1) / minband * nchunks;
    int &wpc = h->waves_per_cu[K][h->variant];
    if (wpc == 0) wpc = golhip::stencil_waves_per_cu(K, h->variant);
    const int64_t capacity = (int64_t)h->cus * wpc;
    // S = 8 (two levels per wave at K = 16) on the boards that fit S = 4 in one round: its waves
    // are light (few VGPRs), so up to two rounds' worth: 5120^2 with counts 1.70 -> 1.58 us per
    // turn, 4096^2 1.49 -> 1.35 (profiles/r01_tune_small_split8.txt)
    if (golhip::stencil_split_supported(K, 8) && waves1 * 8 <= 2 * capacity) return 8;
    for (int S : {4, 2})
        if (golhip::stencil_split_supported(K, S) && waves1 * S <= capacity) return S;
    return 1;
}

// The register kernels for boards too small for the streaming kernel (stencil_tile.hip): gol_tile
// (one wave per T + 2K row tile) and gol_slab (a workgroup of W waves x S rows, edge rows through
// LDS).  They replace the streaming band's pipeline fill (2K rows per band, one dependency chain
// per wave) by a K-row trapezoid per tile/slab with every row of a generation independent; they
// win where the streaming kernel cannot get both tall bands and enough waves (small boards;
// profiles/r02/tune_tile.txt).
struct RegKernel {
    int kind = 0;  // 0 none (streaming), 2 gol_tile, 3 gol_slab
    int T = 0, W = 0, S = 0, NC = 4;
    int out_rows() const { return T; }  // output rows per tile / slab
};
RegKernel pick_reg_kernel(golhip_t h, int64_t rows_total, int K, bool counting) {
    RegKernel rk;
    if (!golhip::variant_is_production_family(h->variant) || h->split) return rk;
    // an explicit level split or band height (tests, tuning) asks for the streaming kernels
    const bool forced = h->force_tile > 0 || h->force_slab > 0;
    if (!forced && (h->force_split > 0 || h->band_rows > 0)) return rk;
    // the input descriptor spans the board's rows; offsets are 32-bit signed
    if ((int64_t)h->height * h->pitch * 4 >= ((int64_t)1 << 31)) return rk;
    if (h->force_tile > 0) {
        if (golhip::stencil_tile_supported(K, h->force_tile)) rk.kind = 2, rk.T = h->force_tile;
        return rk;
    }
    if (h->force_slab > 0) {  // [NC x 10000 +] W x 100 + S
        const int NC = h->force_slab >= 10000 ? h->force_slab / 10000 : 4;
        const int W = h->force_slab / 100 % 100, S = h->force_slab % 100;
        // NC = 14 (gol_slabp): P = 64 / (wd + 2) segments of S rows per wave, boards of <= 62 words
        const int P = NC == 14 ? (h->wd <= 62 ? (int)(64 / (h->wd + 2)) : 0) : 1;
        if (P > 0 && W * P * S - 2 * K >= 1 && golhip::stencil_slab_supported(K, W, S, NC))
            rk.kind = 3, rk.W = W, rk.S = S, rk.NC = NC, rk.T = W * P * S - 2 * K;
        return rk;
    }
    if (h->force_tile == 0 || h->force_slab == 0) return rk;
    // automatic: the slab shape measured best for this depth (profiles/r02/small_boards.txt: at
    // K = 16, 8 waves x 12 rows -- 64 output rows per slab, 240 slabs at 5120^2, about one per CU
    // -- 1.33 us per turn with counts vs 1.62 for the level split, 1.21 vs 1.35 at 4096^2, 2.45
    // vs 2.87 at 8192^2), on boards where the streaming kernel has at most kSlabMaxWaves1PerCu
    // minimal-band waves per CU (round 4: 40, up from 16)
    // (2 row chains per wave at 8 x 12: 1 % over 4, fewer segment-start sums).  Counting
    // launches at K = 16 take 12 waves x 8 rows: its four pure-halo waves (2S <= K) skip the
    // counts and flush the other waves' per-generation sums during the launch (5120^2 with every
    // count 1.005 -> 0.998 us/turn, 4096^2 0.951 -> 0.939; without counts 8 x 12 stays faster,
    // 0.814 vs 0.848: profiles/r02/r02ab_slab_shapes.txt)
    if (h->cus == 0) {
        hipDeviceProp_t prop;
        h->cus = hipGetDeviceProperties(&prop, h->shards[0].device) == hipSuccess
                     ? prop.multiProcessorCount
                     : 256;
    }
    const int64_t per = golhip::chunk_words(K, h->variant, counting);
    const int64_t nchunks = (h->wd + per - 1) / per;
    const int64_t minband = std::max(K, 8);
    const int64_t waves1 = (rows_total + minband - 1) / minband * nchunks;
    if (waves1 > kSlabMaxWaves1PerCu * (int64_t)h->cus) return rk;
    // K = 16: among the candidate shapes, the least modelled time: a slab is one workgroup per
    // CU, and its time is set by the SIMD with the most rows to update each generation, ceil(W/4)
    // waves x S rows, times the rounds of workgroups over the CUs.  The board decides: 5120^2
    // keeps 12 x 8 (240 slabs; 12 x 7 would need 297 > 256 CUs), 4096^2 takes 12 x 7 (237 slabs,
    // 21 rows per SIMD instead of 24): 0.926 -> 0.869 us/turn with every count, 0.791 -> 0.770
    // without (profiles/r03/r03e_tune_slab.log).  Ties keep the earlier shape: 8 x 12 measured
    // best at 5120^2 with and without counts once the counting loop lost its add3 tree and the
    // exchange its branches (0.916 vs 0.931 us/turn for 12 x 8 with every count, 0.806 vs 0.828
    // without: profiles/r03/r03k_tune_slab.log).
    // Narrow boards (wd <= 30 packed words, P = 64 / (wd + 2) >= 2 row segments per wave: the
    // reference's test sizes up to 512 and configs[0]) take the packed slab gol_slabp (NC = 14):
    // the launch is a chain of barrier-bound generations, fastest with few waves per workgroup --
    // the first of 4 / 6 / 8 waves x 3 rows whose workgroups fit one round over the CUs, else 8 x 3
    // (1600 turns, every count: 512^2 4 x 3 0.570 us/turn vs 0.811 for gol_slab2 12 x 7; 4096 x 512
    // 6 x 3 0.598 (4 x 3 with 1024 workgroups 0.806); 640^2 (P = 2) 6 x 3 0.604 / 8 x 3 0.590 vs
    // 0.809; without counts 0.37 - 0.42 vs 0.70: profiles/r04/r04p4_narrow_sweep.log, r04p5)
    if (K == 16 && h->wd <= 30) {
        const int P = (int)(64 / (h->wd + 2));
        for (const int W : {4, 6, 8}) {
            const int T = W * P * 3 - 2 * K;
            if (T < 1 || !golhip::stencil_slab_supported(K, W, 3, 14)) continue;
            rk.kind = 3, rk.W = W, rk.S = 3, rk.NC = 14, rk.T = T;
            if ((rows_total + T - 1) / T <= h->cus) break;
        }
        if (rk.kind) return rk;
    }
    struct Cand {
        int W, S, NC;
    };
    // Round 4: gol_slab2 (NC = 9, the edge hand-off off the critical path) at K = 16, in the
    // measured order of the model's ties (profiles/r04/r04c_tune_slab.log, 4096 turns, every count
    // checked): with counts 8 x 12 0.843 / 16 x 6 0.844 / 12 x 8 0.856 us/turn at 5120^2, without
    // counts 16 x 6 0.735 / 12 x 8 0.744 / 8 x 12 0.790; 4096^2 takes 12 x 7 either way (0.781 /
    // 0.662: 237 slabs, 21 rows per SIMD).
    // With counts the shapes whose pure-halo waves used to flush a generation after every barrier
    // (2S <= K: 16 x 6, 12 x 7, 12 x 8) flush every generation at the end of the launch instead
    // (NC = 12): the per-barrier flush sat on each generation's critical path -- 5120^2 16 x 6
    // 0.852 -> 0.772 us/turn, 4096^2 12 x 7 0.782 -> 0.730 (profiles/r04/r04u_tune.log; moving
    // the 8 x 12 flush INTO the loop instead cost 0.844 -> 0.945, r04t).
    static constexpr Cand kCount16[] = {{16, 6, 12}, {8, 12, 9}, {12, 8, 12}, {12, 7, 12}};
    static constexpr Cand kPlain16[] = {{16, 6, 9}, {12, 8, 9}, {8, 12, 9}, {12, 7, 9}};
    static constexpr Cand kOther[] = {{8, 8, 4}};
    const Cand *cands = K == 16 ? (counting ? kCount16 : kPlain16) : kOther;
    const int ncand = K == 16 ? 4 : 1;
    double best = 1e300;
    for (int i = 0; i < ncand; ++i) {
        const Cand c = cands[i];
        if (!golhip::stencil_slab_supported(K, c.W, c.S, c.NC)) continue;
        const int64_t T = (int64_t)c.W * c.S - 2 * K;
        if (T < 1) continue;
        const int64_t slabs = (rows_total + T - 1) / T * ((h->wd + golhip::kTileChunkWords - 1) /
                                                         golhip::kTileChunkWords);
        const int64_t rounds = (slabs + h->cus - 1) / h->cus;
        const double cost = (double)rounds * (double)((c.W + 3) / 4) * c.S;
        if (cost < best) {  // ties keep the earlier (measured-preferred) shape
            best = cost;
            rk.kind = 3, rk.W = c.W, rk.S = c.S, rk.NC = c.NC, rk.T = (int)T;
        }
    }
    return rk;
}

// Largest band the kernels' 32-bit store offsets can address: a band's output descriptor spans
// band * rowbytes bytes, and dropped stores use offset kOutOfRange (2^30) + row * rowbytes, so
// band * rowbytes must stay below 2^30 (golhip_kernels.hip, buffer_store_words).  At 262144 wide
// that is 32767 rows; only --band-rows / very wide boards can reach it.
int64_t max_band_rows(golhip_t h) {
    const int64_t rowbytes = h->pitch * 4;
    return std::max<int64_t>(1, ((int64_t)1 << 30) / rowbytes - 1);
}

// Launch the K-generation stencil described by p (level-split kernel when pick_split says so).
hipError_t launch_auto(golhip_t h, int K, const uint32_t *in, uint32_t *out,
                       const StencilParams &p, unsigned long long *slots, hipStream_t s) {
    const int64_t rows_total = (p.r0e - p.r0b) + (p.r1e - p.r1b);
    if (const RegKernel rk = pick_reg_kernel(h, rows_total, K, slots != nullptr); rk.kind) {
        StencilParams q = p;
        const int T = rk.out_rows();
        q.band = T;
        q.band2 = q.nbig0 = 0;
        q.nbands0 = (p.r0e - p.r0b + T - 1) / T;
        q.nbands = q.nbands0 + (p.r1e - p.r1b + T - 1) / T;
        q.nchunks = (int32_t)((h->wd + golhip::kTileChunkWords - 1) / golhip::kTileChunkWords);
        return rk.kind == 2 ? golhip::launch_stencil_tile(K, T, in, out, q, slots, s)
                            : golhip::launch_stencil_slab(K, rk.W, rk.S, rk.NC, in, out, q, slots, s);
    }
    const int S = pick_split(h, rows_total, K);
    if (S > 1) {
        // the level-split kernel has its own column geometry (half-word halo for K <= 16)
        StencilParams q = p;
        if (q.band2 > 0) {  // uniform bands for the level-split kernel
            q.band2 = q.nbig0 = 0;
            q.nbands0 = (p.r0e - p.r0b + p.band - 1) / p.band;
            q.nbands = q.nbands0 + (p.r1e - p.r1b + p.band - 1) / p.band;
        }
        const int per = golhip::split_chunk_words(K);
        q.nchunks = (int32_t)((h->wd + per - 1) / per);
        return golhip::launch_stencil_split(K, S, in, out, q, slots, s);
    }
    return golhip::launch_stencil(K, h->variant, in, out, p, slots, s);
}

// counting: the launch writes per-generation counts (its kernel, hence its column geometry,
// can differ: chunk_words / prod_pre)
StencilParams make_params(golhip_t h, const Shard &s, int K, int64_t r0b, int64_t r0e,
                          int64_t r1b, int64_t r1e, int64_t reserve_waves = 0, bool counting = false) {
    StencilParams p{};
    p.pitch = h->pitch;
    p.r0b = r0b;
    p.r0e = r0e;
    p.r1b = r1b;
    p.r1e = r1e;
    const int64_t total = (r0e - r0b) + (r1e - r1b);
    p.band = std::min(auto_band(h, std::max<int64_t>(total, 1), K, reserve_waves, counting), max_band_rows(h));
    p.nbands0 = (r0e - r0b + p.band - 1) / p.band;
    // graded bands (golhip_set_tail_bands): range 0 ends in tail_bands bands of tail_rows rows
    const int64_t n2 = h->tail_bands, b2 = h->tail_rows, R0 = r0e - r0b;
    if (n2 > 0 && b2 > 0 && b2 < p.band && R0 > n2 * b2) {
        p.nbig0 = (R0 - n2 * b2) / p.band;
        p.band2 = b2;
        p.nbands0 = p.nbig0 + (R0 - p.nbig0 * p.band + b2 - 1) / b2;
    }
    p.nbands = p.nbands0 + (r1e - r1b + p.band - 1) / p.band;
    p.wrap_rows = h->split ? 0 : h->height;
    p.lo = -(int64_t)h->halo;
    p.hi = s.rows + h->halo;
    p.wd = h->wd;
    const int per = golhip::chunk_words(K, h->variant, counting);
    p.nchunks = (h->wd + per - 1) / per;
    return p;
}

int timing_begin(golhip_t h, Shard &s, hipEvent_t *stop) {
    *stop = nullptr;
    if (!h->timing || &s != &h->shards[0]) return GOLHIP_OK;
    if (h->tused == h->tpool.size()) {
        TimingPair tp;
        HIPCHK(h, hipEventCreate(&tp.a));
        HIPCHK(h, hipEventCreate(&tp.b));
        h->tpool.push_back(tp);
    }
    TimingPair &tp = h->tpool[h->tused++];
    HIPCHK(h, hipEventRecord(tp.a, s.compute));
    *stop = tp.b;
    return GOLHIP_OK;
}

int timing_collect(golhip_t h) {
    if (h->tused == 0) return GOLHIP_OK;
    HIPCHK(h, hipSetDevice(h->shards[0].device));
    for (size_t i = 0; i < h->tused; ++i) {
        if (rccl_waits(h)) {
            const hipEvent_t ev = h->tpool[i].b;
            int rc = poll_until(h, "a timed launch behind the RCCL transfers", [&]() -> int {
                const hipError_t e = hipEventQuery(ev);
                return e == hipSuccess ? 0 : e == hipErrorNotReady ? 1 : fail(h, GOLHIP_ERR_HIP,
                    "hipEventQuery: %s", hipGetErrorString(e));
            });
            if (rc) return rc;
        }
        HIPCHK(h, hipEventSynchronize(h->tpool[i].b));
        float ms = 0.f;
        HIPCHK(h, hipEventElapsedTime(&ms, h->tpool[i].a, h->tpool[i].b));
        h->tms += ms;
    }
    h->tused = 0;
    return GOLHIP_OK;
}

// The 4 transfers of a K-row exchange for one strip (toroidal ring of strips).  Order matters
// when up == down (world 2): sends to `down` first and receives from `up` first, so the i-th send
// of one rank to a peer matches the i-th receive of that peer (RCCL per-peer ordering).
void halo_plan(int world, int rank, int64_t rows, int K, golhip_xfer out[4]) {
    const int up = (rank - 1 + world) % world, down = (rank + 1) % world;
    out[0] = {0, down, rows - K, K};  // my last K rows -> the top halo of the strip below
    out[1] = {0, up, 0, K};           // my first K rows -> the bottom halo of the strip above
    out[2] = {1, up, -(int64_t)K, K}; // top halo <- last K rows of the strip above
    out[3] = {1, down, rows, K};      // bottom halo <- first K rows of the strip below
}

// Exchange K halo rows between neighbouring strips on the comm streams.
//  * rank mode (one process per GPU): RCCL send/recv over xGMI, the plan above in one group;
//  * single process (golhip_create / golhip_create_strips): every strip pulls its two halos from
//    its neighbours' rows with peer copies (xGMI between devices, a D2D copy on one device).
// record_ready = false: the caller recorded ev_ready (the end of the previous block) itself, before
// enqueueing this block's interior (step_block's interior-first order).
int exchange_halos(golhip_t h, int K, bool record_ready = true) {
    const size_t bytes = (size_t)K * (size_t)h->pitch * sizeof(uint32_t);
    if (record_ready)
        for (auto &s : h->shards) {
            HIPCHK(h, hipSetDevice(s.device));
            HIPCHK(h, hipEventRecord(s.ev_ready, s.compute));
        }
    if (h->host_comm_on) {
        // host transport: stage the two sends through pinned host memory (after the block that
        // wrote them), hand the ordered plan to the caller, copy the two halos back on the comm
        // stream; synchronous on the host (a test / fallback transport, not the RCCL fast path)
        Shard &s = h->shards[0];
        golhip_xfer plan[4];
        halo_plan(h->world_size, s.rank, s.rows, K, plan);
        uint32_t *r0 = h->row0(s, h->cur);
        for (int i = 0; i < 4; ++i)
            if (plan[i].kind == 0)
                HIPCHK(h, hipMemcpyAsync(h->hc_buf[i], r0 + plan[i].row * h->pitch, bytes,
                                         hipMemcpyDeviceToHost, s.compute));
        SYNCCHK(h, s.compute);
        if (h->host_comm.exchange(h->host_comm.ctx, plan, 4, h->hc_buf, bytes) != 0)
            return fail(h, GOLHIP_ERR_RCCL, "host transport: exchange of %d-row halos failed", K);
        for (int i = 0; i < 4; ++i)
            if (plan[i].kind == 1)
                HIPCHK(h, hipMemcpyAsync(r0 + plan[i].row * h->pitch, h->hc_buf[i], bytes,
                                         hipMemcpyHostToDevice, s.comm));
    } else if (h->rank_mode) {
        if (h->comm_failed)
            return fail(h, GOLHIP_ERR_RCCL, "the communicator failed earlier: %s", h->comm_pending.c_str());
        // Early exchange: the rows this exchange sends are the last block's boundary bands (edge
        // stream), done long before its interior -- so the transfer overlaps the previous block's
        // interior and the boundary bands of this block find their halos already in place.  The
        // halo rows it receives into were last read by the boundary bands two blocks back, which
        // precede the last block's bands on the edge stream.  Otherwise (deeper K than those
        // bands, no bands last block) it waits for the whole last block (ev_ready).
        for (auto &s : h->shards)
            HIPCHK(h, hipStreamWaitEvent(s.comm, K <= h->edge_k ? s.ev_edge : s.ev_ready, 0));
        Shard &s = h->shards[0];  // rank mode: one strip per process
        golhip_xfer plan[4];
        halo_plan(h->world_size, s.rank, s.rows, K, plan);
        // what a stuck exchange reports (golhip_last_error after ERR_RCCL)
        char desc[256];
        std::snprintf(desc, sizeof desc,
                      "halo exchange of K = %d rows (%zu bytes per transfer): send rows [%lld, +%d) "
                      "-> rank %d, rows [0, +%d) -> rank %d; receive rows [-%d, ...) <- rank %d, "
                      "[%lld, ...) <- rank %d",
                      K, bytes, (long long)(s.rows - K), K, plan[0].peer, K, plan[1].peer, K,
                      plan[2].peer, (long long)s.rows, plan[3].peer);
        h->comm_pending = desc;
        uint32_t *r0 = h->row0(s, h->cur);
        NCCLCALL(h, "ncclGroupStart", ncclGroupStart());
        for (int i = 0; i < 4; ++i) {
            const golhip_xfer &x = plan[i];
            uint32_t *p = r0 + x.row * h->pitch;
            if (x.kind == 0) {
                NCCLCALL(h, "ncclSend", ncclSend(p, bytes, ncclUint8, x.peer, s.comm_nccl, s.comm));
            } else {
                NCCLCALL(h, "ncclRecv", ncclRecv(p, bytes, ncclUint8, x.peer, s.comm_nccl, s.comm));
            }
        }
        NCCLCALL(h, "ncclGroupEnd", ncclGroupEnd());
        int rc = comm_ready(h, s.comm_nccl, "the halo exchange's RCCL group");
        if (rc) return rc;
    } else {
        const int n = (int)h->shards.size();
        for (int i = 0; i < n; ++i) {
            Shard &s = h->shards[i];
            Shard &up = h->shards[(i - 1 + n) % n], &down = h->shards[(i + 1) % n];
            HIPCHK(h, hipSetDevice(s.device));
            // the neighbours read this strip's rows in THEIR comm streams: this strip's next block
            // (which overwrites the buffer they read, the interior rows included when K shrinks)
            // waits for their previous copies (ev_halo still marks them), then for its own ones
            HIPCHK(h, hipStreamWaitEvent(s.compute, up.ev_halo, 0));
            HIPCHK(h, hipStreamWaitEvent(s.compute, down.ev_halo, 0));
            HIPCHK(h, hipStreamWaitEvent(s.comm, up.ev_ready, 0));
            HIPCHK(h, hipStreamWaitEvent(s.comm, down.ev_ready, 0));
            uint32_t *r0 = h->row0(s, h->cur);
            HIPCHK(h, hipMemcpyPeerAsync(r0 - (int64_t)K * h->pitch, s.device,
                                         h->row0(up, h->cur) + (up.rows - K) * h->pitch, up.device,
                                         bytes, s.comm));
            HIPCHK(h, hipMemcpyPeerAsync(r0 + s.rows * h->pitch, s.device, h->row0(down, h->cur),
                                         down.device, bytes, s.comm));
        }
    }
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        HIPCHK(h, hipEventRecord(s.ev_halo, s.comm));
    }
    return GOLHIP_OK;
}

// One K-generation block on every shard.  slot_gen >= 0: count the K generations into the count
// window at generation slot_gen (finalized later by flush_counts_window), -1: no counts.
// diff_slot: -1 no flips, kDiffLast the last generation's flips into diffbuf, t >= 0 into flips
// ring slot t (the launch's last generation's flips are written beside its output).
constexpr int64_t kDiffNone = -1, kDiffLast = -2;
int step_block(golhip_t h, int K, int64_t slot_gen, int64_t diff_slot = kDiffNone) {
    // Rank mode over RCCL: the interior needs no halo and touches nothing the exchange does (it
    // reads rows [0, rows), the receives write the halo rows, it writes the other buffer), so it
    // is enqueued FIRST: the host's RCCL group set-up (~15 us, ncclGroupEnd) then runs while the
    // interior does, instead of in front of it (profiles/r04/r04q_tail20_ring.txt).
    const bool interior_first = h->split && h->rank_mode && !h->host_comm_on && !h->edge_first &&
                                h->shards.size() == 1 && h->shards[0].rows >= 3 * K;
    if (h->split && !interior_first) {
        int rc = exchange_halos(h, K);
        if (rc) return rc;
    }
    const int nxt = h->cur ^ 1;
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        unsigned long long *slots =
            slot_gen >= 0 ? s.slots + slot_gen * golhip::kCountSlots : nullptr;
        const uint32_t *in = h->row0(s, h->cur);
        uint32_t *out = h->row0(s, nxt);
        uint32_t *diff = diff_slot == kDiffLast ? s.diffbuf
                         : diff_slot >= 0      ? s.ring + diff_slot * s.rows * h->pitch
                                               : nullptr;
        if (!h->split) {
            StencilParams p = make_params(h, s, K, 0, s.rows, 0, 0, 0, slots != nullptr);
            p.diff = diff;
            // tuning: the stamp variant's streaming gol_stencil writes p.diff as its stamps.  ONLY
            // that kernel: gol_step1 (K = 1) and the register kernels read a non-null p.diff as a
            // flips board of the strip's size (round 4: a K = 1 warmup launch wrote its flips over
            // the 32 MiB stamp buffer -- an illegal memory access)
            if (h->stamp_buf && !diff && K > 1 && pick_reg_kernel(h, s.rows, K, slots != nullptr).kind == 0 &&
                pick_split(h, s.rows, K) <= 1 && p.nbands * (int64_t)p.nchunks <= kStampWaves) {
                p.diff = reinterpret_cast<uint32_t *>(h->stamp_buf);
                h->stamp_waves = p.nbands * (int64_t)p.nchunks;
                h->stamp_words = 4;
            } else if (h->stamp_buf && !diff && K > 1) {
                // gol_slab2 writes its phase stamps through p.stamp (never p.diff)
                const RegKernel rk = pick_reg_kernel(h, s.rows, K, slots != nullptr);
                if (rk.kind == 3 && (rk.NC >= 9 && rk.NC <= 13) /* gol_slab2 / gol_slab3 */ &&
                    8 * p.nbands * (int64_t)p.nchunks * rk.W <= 4 * kStampWaves) {
                    p.stamp = h->stamp_buf;
                    h->stamp_waves = p.nbands * (int64_t)p.nchunks * rk.W;
                    h->stamp_words = 8;
                }
            }
            // a K-deep ring launch (ring_depth: a production register slab) writes the flips of
            // each of its K generations into K consecutive ring slots
            p.diff_stride = diff_slot >= 0 && K > 1 ? s.rows * h->pitch : 0;
            HIPCHK(h, launch_auto(h, K, in, out, p, slots, s.compute));
        } else if (s.rows >= 3 * K) {
            // The interior rows need no halo: they run while the halos are exchanged.  The two
            // boundary bands wait for the halos on their own stream and run concurrently with the
            // interior, in wave slots the interior launch leaves free for them; the compute stream
            // then joins them (counts and the next block need both).
            StencilParams pb = make_params(h, s, K, 0, K, s.rows - K, s.rows, 0, slots != nullptr);
            const int64_t edge_waves = pb.nbands * (int64_t)pb.nchunks;
            StencilParams pi = make_params(h, s, K, K, s.rows - K, 0, 0, edge_waves, slots != nullptr);
            pb.diff = pi.diff = diff;
            pb.prio = h->edge_setprio;
            // the bands read rows [K, 2K) and [rows - 2K, rows - K) the previous block's INTERIOR
            // wrote: with the early exchange the halo event no longer implies it (ev_ready marks
            // the compute stream at the end of the previous block).  Submission order (interior
            // first by default; edge_first: tuning A/B) only matters when both are ready at once
            if (interior_first) {
                HIPCHK(h, hipEventRecord(s.ev_ready, s.compute));  // the end of the previous block
                HIPCHK(h, golhip::launch_stencil(K, h->variant, in, out, pi, slots, s.compute));
                int rc = exchange_halos(h, K, false);
                if (rc) return rc;
            } else if (!h->edge_first) {
                HIPCHK(h, golhip::launch_stencil(K, h->variant, in, out, pi, slots, s.compute));
            }
            HIPCHK(h, hipStreamWaitEvent(s.edge, s.ev_ready, 0));
            HIPCHK(h, hipStreamWaitEvent(s.edge, s.ev_halo, 0));
            HIPCHK(h, golhip::launch_stencil(K, h->variant, in, out, pb, slots, s.edge));
            HIPCHK(h, hipEventRecord(s.ev_edge, s.edge));
            if (h->join_mode == 1 && s.join_flag)
                HIPCHK(h, hipStreamWriteValue32(s.edge, s.join_flag, ++s.join_seq, 0));
            if (h->edge_first)
                HIPCHK(h, golhip::launch_stencil(K, h->variant, in, out, pi, slots, s.compute));
            if (h->join_mode == 1 && s.join_flag)
                HIPCHK(h, hipStreamWaitValue32(s.compute, s.join_flag, s.join_seq, hipStreamWaitValueGte,
                                               0xFFFFFFFFu));
            else
                HIPCHK(h, hipStreamWaitEvent(s.compute, s.ev_edge, 0));
            h->edge_k = K;
        } else {
            h->edge_k = 0;
            HIPCHK(h, hipStreamWaitEvent(s.compute, s.ev_halo, 0));
            StencilParams p = make_params(h, s, K, 0, s.rows, 0, 0, 0, slots != nullptr);
            p.diff = diff;
            HIPCHK(h, golhip::launch_stencil(K, h->variant, in, out, p, slots, s.compute));
        }
    }
    if (h->timing) {
        h->tlaunches += 1;
        h->tgens += K;
    }
    {  // the wait deadline's allowance for queued work (rank mode, poll_until)
        const double cells = (double)h->L * (double)plan_rows(h);
        h->queued_s += cells * K / (launch_rate_tcups(K, cells) * 1e12) + kLaunchOverheadUs * 1e-6;
    }
    h->cur = nxt;
    h->turn += K;
    h->prev_valid = (K == 1);
    h->diff_valid = diff_slot == kDiffLast;
    return GOLHIP_OK;
}

// Depth of the next launch of golhip_step_flips (`left` turns to go): a register-slab launch of K
// generations writes K consecutive ring slots (every generation's flips, gol_slab LD = 2), so the
// ring runs the deepest depth <= left for which the board's automatic kernel choice is a
// production slab shape; anything else (strips, the streaming kernel of large boards, the tail)
// runs one-generation launches, each writing its slot.
int ring_depth(golhip_t h, int64_t left, bool counting) {
    if (h->split || h->shards.size() != 1) return 1;
    for (int K : {16, 12, 8}) {
        if (K > left || K > h->k) continue;
        const RegKernel rk = pick_reg_kernel(h, h->shards[0].rows, K, counting);
        if (rk.kind == 3 && golhip::stencil_slab_flips_every_gen(K, rk.W, rk.S, rk.NC)) return K;
    }
    return 1;
}

// Per-generation counts of the first n window generations -> s.d_counts[off, off + n), one
// finalize launch per window (it re-zeroes the slots) instead of one per K-generation block.
int flush_counts_window(golhip_t h, int n, int64_t off) {
    if (n <= 0) return GOLHIP_OK;
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        HIPCHK(h, golhip::launch_count_finalize(n, s.slots, s.d_counts + off, s.compute));
    }
    return GOLHIP_OK;
}

int sync_all(golhip_t h) {
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        SYNCCHK(h, s.comm);
        SYNCCHK(h, s.edge);
        SYNCCHK(h, s.compute);
    }
    h->queued_s = 0.0;
    return GOLHIP_OK;
}

// Sum n uint64 device values over every strip of the board into host memory `out`:
// strips of this process are summed on the host, ranks with one ncclAllReduce.
int reduce_u64(golhip_t h, const std::vector<unsigned long long *> &bufs, size_t n, uint64_t *out) {
    if (rccl_waits(h)) {
        Shard &s = h->shards[0];
        if (h->comm_failed)
            return fail(h, GOLHIP_ERR_RCCL, "the communicator failed earlier: %s", h->comm_pending.c_str());
        HIPCHK(h, hipSetDevice(s.device));
        char desc[128];
        std::snprintf(desc, sizeof desc, "ncclAllReduce of %zu uint64 counts (%zu bytes) over %d ranks",
                      n, n * sizeof(uint64_t), h->world_size);
        h->comm_pending = desc;
        NCCLCALL(h, "ncclAllReduce", ncclAllReduce(bufs[0], bufs[0], n, ncclUint64, ncclSum,
                                                   s.comm_nccl, s.compute));
        int rc = comm_ready(h, s.comm_nccl, "the count all-reduce");
        if (rc) return rc;
    }
    if (h->shards.size() == 1 && h->shards[0].counts_host && bufs[0] == h->shards[0].d_counts) {
        Shard &s = h->shards[0];  // pinned: written by the finalize kernels in stream order
        HIPCHK(h, hipSetDevice(s.device));
        SYNCCHK(h, s.compute);
        std::memcpy(out, bufs[0], n * sizeof(uint64_t));
        if (h->host_comm_on && h->split && h->host_comm.allreduce_u64(h->host_comm.ctx, out, n) != 0)
            return fail(h, GOLHIP_ERR_RCCL, "host transport: all-reduce of %zu counts failed", n);
        return GOLHIP_OK;
    }
    std::vector<uint64_t> tmp(n);
    for (size_t i = 0; i < h->shards.size(); ++i) {
        Shard &s = h->shards[i];
        HIPCHK(h, hipSetDevice(s.device));
        HIPCHK(h, hipMemcpyAsync(i == 0 ? out : tmp.data(), bufs[i], n * sizeof(uint64_t),
                                 hipMemcpyDeviceToHost, s.compute));
        SYNCCHK(h, s.compute);
        if (i > 0)
            for (size_t j = 0; j < n; ++j) out[j] += tmp[j];
    }
    if (h->host_comm_on && h->split && h->host_comm.allreduce_u64(h->host_comm.ctx, out, n) != 0)
        return fail(h, GOLHIP_ERR_RCCL, "host transport: all-reduce of %zu counts failed", n);
    return GOLHIP_OK;
}

// Cell lists, row-major (gol/distributor.go:153-166 alive cells, :53-59 flips): the set bits of
// a[i] (XOR b[i] when b is given) in the first `width` columns of each shard's rows.  slots > 1:
// a[i] is a tall board of `slots` consecutive boards of the shard's rows (the flips ring); the
// list is then slot-major (turn by turn), per_slot[t] = cells of slot t (nullable).  The scratch
// is preallocated; only a list longer than any before grows its output buffer.
int extract_cells(golhip_t h, const std::vector<const uint32_t *> &a,
                  const std::vector<const uint32_t *> &b, int64_t slots, int32_t *xy, size_t cap,
                  size_t *n, uint64_t *per_slot) {
    if (!n) return fail(h, GOLHIP_ERR_ARG, "n is null");
    const size_t ns = h->shards.size();
    std::vector<std::vector<unsigned long long>> cnt(ns, std::vector<unsigned long long>(slots));
    for (size_t i = 0; i < ns; ++i) {
        Shard &s = h->shards[i];
        const int64_t rows = s.rows * slots;
        int rc = ensure_extract_scratch(h, s, rows, slots);
        if (rc) return rc;
        HIPCHK(h, hipSetDevice(s.device));
        HIPCHK(h, golhip::launch_extract_count(a[i], b[i], h->pitch, rows, h->width,
                                               s.ex_rowcounts, s.ex_offsets, s.ex_block_sums,
                                               s.compute));
        HIPCHK(h, golhip::launch_extract_slot_counts(s.ex_offsets, s.rows, slots, s.ex_slot_counts,
                                                     s.compute));
        HIPCHK(h, hipMemcpyAsync(cnt[i].data(), s.ex_slot_counts,
                                 sizeof(unsigned long long) * (size_t)slots,
                                 hipMemcpyDeviceToHost, s.compute));
    }
    size_t total = 0;
    std::vector<size_t> shard_total(ns, 0);
    for (size_t i = 0; i < ns; ++i) {
        HIPCHK(h, hipSetDevice(h->shards[i].device));
        SYNCCHK(h, h->shards[i].compute);
        for (int64_t t = 0; t < slots; ++t) shard_total[i] += cnt[i][t];
        total += shard_total[i];
    }
    if (per_slot)
        for (int64_t t = 0; t < slots; ++t) {
            per_slot[t] = 0;
            for (size_t i = 0; i < ns; ++i) per_slot[t] += cnt[i][t];
        }
    *n = total;
    if (total > cap) return fail(h, GOLHIP_ERR_CAP, "%zu cells do not fit in cap %zu", total, cap);
    if (total == 0) return GOLHIP_OK;
    if (!xy) return fail(h, GOLHIP_ERR_ARG, "xy is null");
    // slot t of the output: the shards' cells of slot t in shard (row strip) order
    std::vector<size_t> slot_base(slots + 1, 0);
    for (int64_t t = 0; t < slots; ++t) {
        slot_base[t + 1] = slot_base[t];
        for (size_t i = 0; i < ns; ++i) slot_base[t + 1] += cnt[i][t];
    }
    for (size_t i = 0; i < ns; ++i) {
        Shard &s = h->shards[i];
        if (shard_total[i] == 0) continue;
        HIPCHK(h, hipSetDevice(s.device));
        if (shard_total[i] > s.ex_xy_cap) {  // grow the device list (rare: a longer list)
            SYNCCHK(h, s.compute);
            if (s.ex_xy) HIPCHK(h, hipFree(s.ex_xy));
            s.ex_xy = nullptr;
            const size_t want = std::max(shard_total[i], s.ex_xy_cap * 2);
            HIPCHK(h, hipMalloc(&s.ex_xy, sizeof(int32_t) * 2 * want));
            s.ex_xy_cap = want;
        }
        HIPCHK(h, golhip::launch_extract_emit(a[i], b[i], h->pitch, s.rows * slots, h->width,
                                              s.ex_offsets, s.y0, s.rows, s.ex_xy,
                                              shard_total[i], s.compute));
        // the shard's list is slot-major; copy each slot's run to its place in the global list
        // (one shard: the shard's list IS the global list, one copy)
        if (ns == 1) {
            HIPCHK(h, hipMemcpyAsync(xy, s.ex_xy, sizeof(int32_t) * 2 * shard_total[i],
                                     hipMemcpyDeviceToHost, s.compute));
            continue;
        }
        size_t src = 0;
        for (int64_t t = 0; t < slots; ++t) {
            size_t dst = slot_base[t];
            for (size_t i2 = 0; i2 < i; ++i2) dst += cnt[i2][t];
            if (cnt[i][t])
                HIPCHK(h, hipMemcpyAsync(xy + 2 * dst, s.ex_xy + 2 * src,
                                         sizeof(int32_t) * 2 * cnt[i][t], hipMemcpyDeviceToHost,
                                         s.compute));
            src += cnt[i][t];
        }
    }
    return sync_all(h);
}

// Host <-> device byte transfer of the handle's rows, in row chunks through the shard's stage.
int transfer_bytes(golhip_t h, uint8_t *host, size_t row_stride, bool to_device) {
    if (!host) return fail(h, GOLHIP_ERR_ARG, "buffer is null");
    if (row_stride < (size_t)h->width) return fail(h, GOLHIP_ERR_ARG, "row_stride < width");
    const int64_t W = h->width;
    int64_t hrow = 0;  // host row index relative to the handle's first row
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        uint8_t *stage = s.stage;
        const int64_t cr = std::min(std::max<int64_t>(1, s.stage_bytes / W), s.rows);
        for (int64_t y = 0; y < s.rows; y += cr) {
            const int64_t nr = std::min(cr, s.rows - y);
            uint32_t *rows_dev = h->row0(s, h->cur) + y * h->pitch;
            if (to_device) {
                HIPCHK(h, hipMemcpy2DAsync(stage, (size_t)W, host + (size_t)(hrow + y) * row_stride,
                                           row_stride, (size_t)W, (size_t)nr,
                                           hipMemcpyHostToDevice, s.compute));
                HIPCHK(h, golhip::launch_pack(stage, nr, W, h->wd, rows_dev, h->pitch, s.compute));
            } else {
                HIPCHK(h, golhip::launch_unpack(rows_dev, h->pitch, nr, W, stage, s.compute));
                HIPCHK(h, hipMemcpy2DAsync(host + (size_t)(hrow + y) * row_stride, row_stride,
                                           stage, (size_t)W, (size_t)W, (size_t)nr,
                                           hipMemcpyDeviceToHost, s.compute));
            }
            SYNCCHK(h, s.compute);
        }
        hrow += s.rows;
    }
    return GOLHIP_OK;
}

int create_common(golhip_t h) {
    if (h->variant == golhip::kVariantStamp) {
        HIPCHK(h, hipSetDevice(h->shards[0].device));
        HIPCHK(h, hipMalloc(&h->stamp_buf, sizeof(uint64_t) * 4 * kStampWaves));
    }
    for (auto &s : h->shards) {
        int rc = alloc_shard(h, s);
        if (rc) return rc;
        // each launch depth is its own code object, loaded at its first launch (~1 ms): load them
        // all now, not inside the first timed or latency-sensitive step
        HIPCHK(h, golhip::warm_stencils(h->variant, s.compute));
        SYNCCHK(h, s.compute);
    }
    return GOLHIP_OK;
}

constexpr int kGraphGens = 128;      // generations per graph replay (<= count_window)
// Long runs replay larger graphs: each replay of a counting graph ends in a count finalize and a
// copy of its counts (~17 us together on a 5120^2 board, profiles/r02/small_board_timeline.txt),
// paid per 4096 generations instead of per 128 (bounded by the count window).
constexpr int kGraphGensBig = 4096;

// Graphs pay off when a launch is short (launch-bound): < ~100 us of stencil work.
bool small_board(double cells, int K) { return cells * K <= 8e9; }
bool graph_worthy(golhip_t h, int K) {
    if (h->split || h->shards.size() != 1) return false;
    if (h->graph_mode >= 0) return h->graph_mode != 0;  // golhip_set_graphs
    return small_board((double)h->L * (double)h->height, K);
}

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
    // k: the maximum depth; Kfull: the deepest depth used (graph replays), pick_k(k) unless the
    // streaming kernel's bulk depth is capped (stream_depth_cap); Kbulk: the bulk depth of long
    // runs without graphs
    // stream: the board runs the streaming kernel (no register slab/tile, no level split): its
    // graph replays use the best-rate depth too (16384^2: 64.5 vs 55.3 TCUPS at K = 12 vs 16,
    // profiles/r02/r02ae_depth_by_size.txt); the register kernels are tuned at the full depth
    LaunchPlanner(double cells_, int k, int64_t turns, bool small, bool fixed = false,
                  bool keep_last_ = false, int window = 4096, bool stream = false)
        : cells(cells_),
          Kfull(small && stream && !fixed ? best_rate_k(pick_k(k), cells_) : pick_k(k)),
          left(turns), keep_last(keep_last_) {
        M = std::max(2, (kGraphGens / Kfull) & ~1);
        Mbig = std::max(M, (std::min(kGraphGensBig, window) / Kfull) & ~1);
        graphs = small && turns >= (int64_t)M * Kfull + (keep_last ? 1 : 0);
        Kbulk = small || fixed ? Kfull : best_rate_k(Kfull, cells);
    }
    int next() {
        for (int m : {Mbig, M})
            if (graphs && left >= (int64_t)m * Kfull + (keep_last ? 1 : 0)) {
                left -= (int64_t)m * Kfull;
                last_M = m;
                return 0;
            }
        const int K = left >= 2 * (int64_t)Kbulk ? Kbulk : plan_first_k(left, Kfull, cells);
        left -= K;
        return K;
    }
};

int graph_for(golhip_t h, int K, int M, bool counting, hipGraphExec_t *out) {
    Shard &s = h->shards[0];
    const int64_t band = auto_band(h, s.rows, K, 0, counting);
    for (auto &g : h->graphs)
        if (g.K == K && g.M == M && g.cur == h->cur && g.counting == counting && g.band == band &&
            g.tail_bands == h->tail_bands && g.tail_rows == h->tail_rows) {
            *out = g.exec;
            return GOLHIP_OK;
        }
    HIPCHK(h, hipSetDevice(s.device));
    if (counting && !h->g_counts)
        HIPCHK(h, hipMalloc(&h->g_counts, sizeof(unsigned long long) * kGraphGensBig * 2));
    hipGraph_t graph = nullptr;
    HIPCHK(h, hipStreamBeginCapture(s.compute, hipStreamCaptureModeThreadLocal));
    hipError_t err = hipSuccess;
    for (int i = 0; i < M && err == hipSuccess; ++i) {
        const int c = h->cur ^ (i & 1);
        StencilParams p = make_params(h, s, K, 0, s.rows, 0, 0, 0, counting);
        err = launch_auto(h, K, h->row0(s, c), h->row0(s, c ^ 1), p,
                          counting ? s.slots + (int64_t)i * K * golhip::kCountSlots : nullptr,
                          s.compute);
    }
    if (err == hipSuccess && counting)  // one finalize for the graph's M*K generations
        err = golhip::launch_count_finalize(M * K, s.slots, h->g_counts, s.compute);
    hipError_t e2 = hipStreamEndCapture(s.compute, &graph);
    if (err != hipSuccess || e2 != hipSuccess)
        return fail(h, GOLHIP_ERR_HIP, "graph capture: %s", hipGetErrorString(err ? err : e2));
    GraphEntry g;
    g.K = K;
    g.M = M;
    g.cur = h->cur;
    g.counting = counting;
    g.band = band;
    g.tail_bands = h->tail_bands;
    g.tail_rows = h->tail_rows;
    err = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (err != hipSuccess) return fail(h, GOLHIP_ERR_HIP, "graph instantiate: %s", hipGetErrorString(err));
    h->graphs.push_back(g);
    *out = g.exec;
    return GOLHIP_OK;
}

}  // namespace

// ================================================================================ C ABI ====
extern "C" {

int golhip_version(void) { return kVersion; }

const char *golhip_strerror(int code) {
    switch (code) {
        case GOLHIP_OK: return "ok";
        case GOLHIP_ERR_ARG: return "invalid argument";
        case GOLHIP_ERR_HIP: return "HIP runtime error";
        case GOLHIP_ERR_OOM: return "out of device memory";
        case GOLHIP_ERR_CAP: return "output capacity too small";
        case GOLHIP_ERR_RCCL: return "RCCL error";
        case GOLHIP_ERR_NODEV: return "no usable gfx950 device";
        case GOLHIP_ERR_STATE: return "invalid state for this call";
        default: return "unknown error";
    }
}

int golhip_device_count(int *out) {
    if (!out) return GOLHIP_ERR_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return GOLHIP_OK;
}

int golhip_strip_bounds(int64_t height, int world_size, int rank, int64_t *y0, int64_t *rows) {
    if (height <= 0 || world_size <= 0 || rank < 0 || rank >= world_size || !y0 || !rows)
        return GOLHIP_ERR_ARG;
    strip_bounds(height, world_size, rank, *y0, *rows);
    return GOLHIP_OK;
}

int golhip_halo_plan(int64_t height, int world_size, int rank, int k, golhip_xfer *out) {
    if (height <= 0 || world_size <= 1 || rank < 0 || rank >= world_size || !out) return GOLHIP_ERR_ARG;
    if (k < 1 || k > golhip::kMaxK || height / world_size < k) return GOLHIP_ERR_ARG;
    int64_t y0, rows;
    strip_bounds(height, world_size, rank, y0, rows);
    halo_plan(world_size, rank, rows, k, out);
    return GOLHIP_OK;
}

int golhip_nccl_unique_id(uint8_t *out) {
    if (!out) return GOLHIP_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return GOLHIP_ERR_RCCL;
    static_assert(sizeof(ncclUniqueId) == GOLHIP_NCCL_ID_BYTES, "nccl id size");
    std::memcpy(out, &id, sizeof id);
    return GOLHIP_OK;
}

int golhip_create_strips(int width, int height, int nstrips, int ndevices, int k, golhip_t *out) {
    if (!out) return GOLHIP_ERR_ARG;
    *out = nullptr;
    int rc = validate_geometry(width, height, nstrips, k);
    if (rc) return rc;
    if (ndevices < 1 || ndevices > nstrips) return GOLHIP_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < ndevices) return GOLHIP_ERR_NODEV;
    golhip_t h = new golhip_engine();
    setup_engine(h, width, height, nstrips, k);
    h->shards.resize(nstrips);
    for (int r = 0; r < nstrips; ++r) {
        Shard &s = h->shards[r];
        s.device = (int)((int64_t)r * ndevices / nstrips);
        s.rank = r;
        strip_bounds(height, nstrips, r, s.y0, s.rows);
    }
    for (int d = 0; d < ndevices; ++d)
        if ((rc = check_device_arch(h, d))) goto fail;
    // peer access between neighbouring devices for the halo copies (xGMI)
    for (int d = 0; d < ndevices && ndevices > 1; ++d) {
        for (int e : {(d + 1) % ndevices, (d - 1 + ndevices) % ndevices}) {
            int can = 0;
            if (e == d || hipDeviceCanAccessPeer(&can, d, e) != hipSuccess || !can) continue;
            (void)hipSetDevice(d);
            hipError_t pe = hipDeviceEnablePeerAccess(e, 0);
            if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) {
                rc = fail(h, GOLHIP_ERR_HIP, "peer access %d->%d: %s", d, e, hipGetErrorString(pe));
                goto fail;
            }
            (void)hipGetLastError();
        }
    }
    if ((rc = create_common(h))) goto fail;
    *out = h;
    return GOLHIP_OK;
fail:
    g_create_error = h->err.empty() ? golhip_strerror(rc) : h->err;
    for (auto &s : h->shards) free_shard(s);
    delete h;
    return rc;
}

int golhip_create(int width, int height, int ngpus, int k, golhip_t *out) {
    return golhip_create_strips(width, height, ngpus, ngpus, k, out);
}

int golhip_create_rank(int width, int height, int rank, int world_size, int device, int k,
                       const uint8_t *nccl_id, golhip_t *out) {
    if (!out) return GOLHIP_ERR_ARG;
    *out = nullptr;
    int rc = validate_geometry(width, height, world_size, k);
    if (rc) return rc;
    if (rank < 0 || rank >= world_size || device < 0) return GOLHIP_ERR_ARG;
    if (world_size > 1 && !nccl_id) return GOLHIP_ERR_ARG;
    const char *rs = std::getenv("GOLHIP_RING_SELF");
    const bool ring_self = world_size == 1 && rs && std::atoi(rs) != 0;
    if (ring_self && height < k) return GOLHIP_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) return GOLHIP_ERR_NODEV;
    golhip_t h = new golhip_engine();
    setup_engine(h, width, height, world_size, k);
    h->rank_mode = true;
    // Test hook: GOLHIP_RING_SELF=1 makes a world-1 rank engine a ring of ONE halo'd strip whose
    // halos go through RCCL send/recv to itself, so the whole rank-mode path (plan, RCCL group,
    // interior/boundary overlap, count all-reduce) runs on a one-GPU box.  GOLHIP_RING_SELF=2: the
    // same ring whose every step ends in a 20 s stall of its compute stream, for the fail-fast test
    // of the deadline (tests/test_gpu_failfast.py).
    if (ring_self) {
        h->split = true;
        h->halo = k;
        h->test_ring_mode = std::atoi(rs);
    }
    h->shards.resize(1);
    Shard &s = h->shards[0];
    s.device = device;
    s.rank = rank;
    strip_bounds(height, world_size, rank, s.y0, s.rows);
    if ((rc = check_device_arch(h, device))) goto fail;
    if ((rc = create_common(h))) goto fail;
    if (h->split) {
        ncclUniqueId id;
        if (nccl_id) {
            std::memcpy(&id, nccl_id, sizeof id);
        } else if (ncclGetUniqueId(&id) != ncclSuccess) {  // ring of one: a local id
            rc = fail(h, GOLHIP_ERR_RCCL, "ncclGetUniqueId failed");
            goto fail;
        }
        (void)hipSetDevice(device);
        // non-blocking communicator: no RCCL call blocks the host, every wait on one is bounded
        // (poll_until); a rank whose peers never join fails here after the timeout
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        char desc[128];
        std::snprintf(desc, sizeof desc, "ncclCommInitRankConfig(rank %d of %d, device %d)", rank,
                      world_size, device);
        h->comm_pending = desc;
        const ncclResult_t nr = ncclCommInitRankConfig(&s.comm_nccl, world_size, id, rank, &cfg);
        if (nr != ncclSuccess && nr != ncclInProgress) {
            if (s.comm_nccl) (void)ncclCommAbort(s.comm_nccl);
            s.comm_nccl = nullptr;
            rc = fail(h, GOLHIP_ERR_RCCL, "%s: %s", desc, ncclGetErrorString(nr));
            goto fail;
        }
        if ((rc = comm_ready(h, s.comm_nccl, "the communicator's set-up (waiting for every rank)")))
            goto fail;
        h->comm_setup_done = true;
        h->comm_pending.clear();
    }
    *out = h;
    return GOLHIP_OK;
fail:
    g_create_error = h->err.empty() ? golhip_strerror(rc) : h->err;
    for (auto &sh : h->shards) free_shard(sh, h->comm_timeout_ms, h->comm_failed && h->comm_setup_done);
    delete h;
    return rc;
}

int golhip_create_rank_host(int width, int height, int rank, int world_size, int device, int k,
                            const golhip_host_comm *comm, golhip_t *out) {
    if (!out) return GOLHIP_ERR_ARG;
    *out = nullptr;
    if (!comm || !comm->exchange || !comm->allreduce_u64) return GOLHIP_ERR_ARG;
    int rc = validate_geometry(width, height, world_size, k);
    if (rc) return rc;
    if (rank < 0 || rank >= world_size || device < 0) return GOLHIP_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) return GOLHIP_ERR_NODEV;
    golhip_t h = new golhip_engine();
    setup_engine(h, width, height, world_size, k);
    h->rank_mode = true;
    h->host_comm_on = true;
    h->host_comm = *comm;
    h->shards.resize(1);
    Shard &s = h->shards[0];
    s.device = device;
    s.rank = rank;
    strip_bounds(height, world_size, rank, s.y0, s.rows);
    if ((rc = check_device_arch(h, device))) goto fail;
    if ((rc = create_common(h))) goto fail;
    if (h->split) {
        (void)hipSetDevice(device);
        const size_t bytes = (size_t)h->halo * (size_t)h->pitch * sizeof(uint32_t);
        for (void *&b : h->hc_buf) {
            const hipError_t e = hipHostMalloc(&b, bytes, hipHostMallocDefault);
            if (e != hipSuccess) {
                b = nullptr;
                rc = fail(h, GOLHIP_ERR_OOM, "pinned halo buffers: %s", hipGetErrorString(e));
                goto fail;
            }
        }
    }
    *out = h;
    return GOLHIP_OK;
fail:
    g_create_error = h->err.empty() ? golhip_strerror(rc) : h->err;
    for (auto &sh : h->shards) free_shard(sh);
    for (void *b : h->hc_buf)
        if (b) (void)hipHostFree(b);
    delete h;
    return rc;
}

int golhip_destroy(golhip_t h) {
    if (!h) return GOLHIP_ERR_ARG;
    for (auto &g : h->graphs) (void)hipGraphExecDestroy(g.exec);
    if (h->g_counts) (void)hipFree(h->g_counts);
    for (auto &tp : h->tpool) {
        (void)hipEventDestroy(tp.a);
        (void)hipEventDestroy(tp.b);
    }
    for (auto &s : h->shards) free_shard(s, rccl_waits(h) ? h->comm_timeout_ms : 0, h->comm_failed);
    for (void *b : h->hc_buf)
        if (b) (void)hipHostFree(b);
    if (h->stamp_buf) (void)hipFree(h->stamp_buf);
    delete h;
    return GOLHIP_OK;
}

#ifdef GOLHIP_TUNING
// Tuning build only (not in include/golhip.h): the per-wave stamps of the last single-strip
// launch of a GOLHIP_VARIANT=stamp handle, 4 uint64 per wave (start, end: s_memrealtime 100 MHz;
// shader cycles; HW_ID | XCC_ID << 32).  scripts/stamp_launch.py.
int golhip_tuning_stamps(golhip_t h, uint64_t *out, size_t cap_waves, size_t *n_waves) {
    if (!h || !n_waves) return GOLHIP_ERR_ARG;
    if (!h->stamp_buf) return fail(h, GOLHIP_ERR_STATE, "not a GOLHIP_VARIANT=stamp handle");
    int rc = sync_all(h);
    if (rc) return rc;
    *n_waves = (size_t)std::min<int64_t>(h->stamp_waves, kStampWaves);
    if (!out) return GOLHIP_OK;
    if (cap_waves < *n_waves) return GOLHIP_ERR_CAP;
    HIPCHK(h, hipMemcpy(out, h->stamp_buf, sizeof(uint64_t) * 4 * *n_waves, hipMemcpyDeviceToHost));
    return GOLHIP_OK;
}
// The same with the record length: words_per_wave uint64 per wave (4: gol_stencil, 8: gol_slab2's
// phase stamps -- start, rows loaded, generations done, end, cycles, HW_ID | XCC_ID << 32, group,
// wave).  cap_words / n_words count uint64.  scripts/slab_stamps.py.
int golhip_tuning_stamps_ex(golhip_t h, uint64_t *out, size_t cap_words, size_t *n_words, int *words_per_wave) {
    if (!h || !n_words || !words_per_wave) return GOLHIP_ERR_ARG;
    if (!h->stamp_buf) return fail(h, GOLHIP_ERR_STATE, "not a GOLHIP_VARIANT=stamp handle");
    int rc = sync_all(h);
    if (rc) return rc;
    *words_per_wave = h->stamp_words;
    *n_words = (size_t)std::min<int64_t>(h->stamp_waves * h->stamp_words, 4 * kStampWaves);
    if (!out) return GOLHIP_OK;
    if (cap_words < *n_words) return GOLHIP_ERR_CAP;
    HIPCHK(h, hipMemcpy(out, h->stamp_buf, sizeof(uint64_t) * *n_words, hipMemcpyDeviceToHost));
    return GOLHIP_OK;
}
#endif

const char *golhip_last_error(golhip_t h) { return h ? h->err.c_str() : g_create_error.c_str(); }

int golhip_get_info(golhip_t h, golhip_info *out) {
    if (!h || !out) return GOLHIP_ERR_ARG;
    out->width = h->width;
    out->height = h->height;
    out->torus_width = h->L;
    out->y0 = h->shards.front().y0;
    int64_t rows = 0;
    for (auto &s : h->shards) rows += s.rows;
    out->rows = rows;
    out->rank = h->shards.front().rank;
    out->world_size = h->world_size;
    out->nshards = (int32_t)h->shards.size();
    out->k = h->k;
    out->halo_rows = h->halo;
    out->band_rows = h->band_rows;
    return GOLHIP_OK;
}

int golhip_load_bytes(golhip_t h, const uint8_t *cells, size_t row_stride) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    rc = transfer_bytes(h, const_cast<uint8_t *>(cells), row_stride, true);
    if (rc) return rc;
    h->turn = 0;
    h->prev_valid = false;
    h->diff_valid = false;
    return GOLHIP_OK;
}

int golhip_store_bytes(golhip_t h, uint8_t *out, size_t row_stride) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    return transfer_bytes(h, out, row_stride, false);
}

int golhip_init_random(golhip_t h, uint64_t seed, uint32_t density_q32) {
    if (!h) return GOLHIP_ERR_ARG;
    if (h->width % 64 != 0) return fail(h, GOLHIP_ERR_ARG, "init_random needs width %% 64 == 0");
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        HIPCHK(h, golhip::launch_init_random(h->row0(s, h->cur), h->pitch, s.rows, s.y0, h->width,
                                             h->wd, seed, density_q32, s.compute));
    }
    h->turn = 0;
    h->prev_valid = false;
    h->diff_valid = false;
    return sync_all(h);
}

int golhip_store_words(golhip_t h, uint64_t *out) {
    if (!h || !out) return GOLHIP_ERR_ARG;
    if (h->width % 64 != 0) return fail(h, GOLHIP_ERR_ARG, "store_words needs width %% 64 == 0");
    int rc = sync_all(h);
    if (rc) return rc;
    const int64_t wpr = h->width / 64;
    int64_t hrow = 0;
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        uint64_t *d = reinterpret_cast<uint64_t *>(s.stage);
        const int64_t cr = std::max<int64_t>(1, s.stage_bytes / (int64_t)sizeof(uint64_t) / wpr);
        for (int64_t y = 0; y < s.rows; y += cr) {
            const int64_t nr = std::min(cr, s.rows - y);
            HIPCHK(h, golhip::launch_words_out(h->row0(s, h->cur) + y * h->pitch, h->pitch, nr,
                                               h->width, d, s.compute));
            HIPCHK(h, hipMemcpyAsync(out + (hrow + y) * wpr, d, sizeof(uint64_t) * (size_t)(nr * wpr),
                                     hipMemcpyDeviceToHost, s.compute));
            SYNCCHK(h, s.compute);
        }
        hrow += s.rows;
    }
    return GOLHIP_OK;
}

int golhip_load_words(golhip_t h, const uint64_t *in) {
    if (!h || !in) return GOLHIP_ERR_ARG;
    if (h->width % 64 != 0) return fail(h, GOLHIP_ERR_ARG, "load_words needs width %% 64 == 0");
    int rc = sync_all(h);
    if (rc) return rc;
    const int64_t wpr = h->width / 64;
    int64_t hrow = 0;
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        uint64_t *d = reinterpret_cast<uint64_t *>(s.stage);
        const int64_t cr = std::max<int64_t>(1, s.stage_bytes / (int64_t)sizeof(uint64_t) / wpr);
        for (int64_t y = 0; y < s.rows; y += cr) {
            const int64_t nr = std::min(cr, s.rows - y);
            HIPCHK(h, hipMemcpyAsync(d, in + (hrow + y) * wpr, sizeof(uint64_t) * (size_t)(nr * wpr),
                                     hipMemcpyHostToDevice, s.compute));
            HIPCHK(h, golhip::launch_words_in(d, nr, h->width, h->wd, h->row0(s, h->cur) + y * h->pitch,
                                              h->pitch, s.compute));
            SYNCCHK(h, s.compute);
        }
        hrow += s.rows;
    }
    h->turn = 0;
    h->prev_valid = false;
    h->diff_valid = false;
    return GOLHIP_OK;
}

// The body of golhip_step / golhip_step_flips.  ring: every generation is its own launch writing
// its flips into ring slot t (t = 0 .. turns-1); otherwise the launch plan, and with flips
// tracking on, the last launch writes the last generation's flips.
static int run_steps(golhip_t h, int64_t turns, uint64_t *alive_per_turn, bool ring) {
    if (!h || turns < 0) return GOLHIP_ERR_ARG;
    if (turns == 0) return GOLHIP_OK;
    if ((ring || h->track_flips) && !variant_writes_flips(h->variant))
        return fail(h, GOLHIP_ERR_STATE,
                    "flips need a production kernel variant (tuning variant %d cannot write them)",
                    h->variant);
    const bool counting = alive_per_turn != nullptr;
    if (counting) {
        // long calls keep the device buffer: their graph replays copy each replay's counts into it
        // (device to device) and one copy returns them
        const bool host_counts = h->shards.size() == 1 && !rccl_waits(h) && turns <= kPinnedCountTurns;
        for (auto &s : h->shards) {
            unsigned long long *&buf = host_counts ? s.pin_counts : s.dev_counts;
            size_t &cap = host_counts ? s.pin_counts_cap : s.dev_counts_cap;
            if (cap < (size_t)turns) {
                HIPCHK(h, hipSetDevice(s.device));
                SYNCCHK(h, s.compute);
                if (buf) HIPCHK(h, host_counts ? hipHostFree(buf) : hipFree(buf));
                buf = nullptr;
                cap = 0;
                const size_t n = (size_t)std::max<int64_t>(turns, 128);
                if (host_counts)
                    HIPCHK(h, hipHostMalloc((void **)&buf, n * sizeof(unsigned long long), hipHostMallocCoherent));
                else
                    HIPCHK(h, hipMalloc(&buf, n * sizeof(unsigned long long)));
                cap = n;
            }
            s.d_counts = buf;
            s.counts_host = host_counts;
        }
    }
    // Timing: ONE event pair around the whole call on the first strip's compute stream (per-
    // launch events would add ~10 us of idle GPU between launches); the average launch time is
    // that span / launches (the launches run back to back on the stream).
    hipEvent_t stop = nullptr;
    if (h->timing) {
        int rc = timing_begin(h, h->shards[0], &stop);
        if (rc) return rc;
    }
    int64_t done = 0;
    const int kmax = pick_k(h->k);
    const bool stream = !ring && h->shards.size() == 1 &&
                        pick_reg_kernel(h, h->shards[0].rows, kmax, counting).kind == 0 &&
                        pick_split(h, h->shards[0].rows, kmax) <= 1;
    // planned per strip (the band geometry and each GPU's launch time follow the strip), from the
    // largest strip of the board, so every rank of a rank-mode board plans the same depths
    LaunchPlanner plan((double)h->L * (double)plan_rows(h), ring ? 1 : h->k, turns,
                       !ring && graph_worthy(h, kmax), h->fixed_k || ring, h->track_flips,
                       h->count_window, stream);
    const int Kfull = plan.Kfull;
    int64_t win = 0;  // generations pending in the count window, from turn offset done - win
    while (done < turns) {
        const int K = ring ? ring_depth(h, turns - done, counting) : plan.next();
        if (K == 0) {  // one graph replay of M x Kfull generations
            const int M = plan.last_M;
            if (counting) {  // the graph finalizes its own generations from window slot 0
                int rc = flush_counts_window(h, (int)win, done - win);
                if (rc) return rc;
                win = 0;
            }
            hipGraphExec_t exec = nullptr;
            int rc = graph_for(h, Kfull, M, counting, &exec);
            if (rc) return rc;
            Shard &s = h->shards[0];
            HIPCHK(h, hipGraphLaunch(exec, s.compute));
            if (counting)
                HIPCHK(h, hipMemcpyAsync(s.d_counts + done, h->g_counts,
                                         sizeof(unsigned long long) * (size_t)M * Kfull,
                                         s.counts_host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice,
                                         s.compute));
            done += (int64_t)M * Kfull;
            h->turn += (int64_t)M * Kfull;
            h->prev_valid = (Kfull == 1);
            h->diff_valid = false;
            if (h->timing) {
                h->tlaunches += M;
                h->tgens += (int64_t)M * Kfull;
            }
            continue;
        }
        if (counting && win + K > h->count_window) {
            int rc = flush_counts_window(h, (int)win, done - win);
            if (rc) return rc;
            win = 0;
        }
        const int64_t diff_slot = ring                                      ? done
                                  : (h->track_flips && done + K == turns) ? kDiffLast
                                                                          : kDiffNone;
        int rc = step_block(h, K, counting ? win : -1, diff_slot);
        if (rc) return rc;
        done += K;
        if (counting) win += K;
    }
    if (counting) {
        int rc = flush_counts_window(h, (int)win, done - win);
        if (rc) return rc;
    }
    if (h->test_ring_mode == 2 && rccl_waits(h))  // test hook (GOLHIP_RING_SELF=2): a stalled rank
        HIPCHK(h, hipLaunchHostFunc(h->shards[0].compute,
                                    [](void *) { std::this_thread::sleep_for(std::chrono::seconds(20)); },
                                    nullptr));
    if (stop) {
        HIPCHK(h, hipSetDevice(h->shards[0].device));
        HIPCHK(h, hipEventRecord(stop, h->shards[0].compute));
        if (h->tused >= 1024) {
            int rc = timing_collect(h);
            if (rc) return rc;
        }
    }
    if (counting) {
        std::vector<unsigned long long *> bufs;
        for (auto &s : h->shards) bufs.push_back(s.d_counts);
        int rc = reduce_u64(h, bufs, (size_t)turns, alive_per_turn);
        if (rc) return rc;
        const uint64_t rep = (uint64_t)h->rep();
        if (rep > 1)
            for (int64_t i = 0; i < turns; ++i) alive_per_turn[i] /= rep;
    }
    return GOLHIP_OK;
}

int golhip_step(golhip_t h, int64_t turns, uint64_t *alive_per_turn) {
    return run_steps(h, turns, alive_per_turn, false);
}

// Ring slots per golhip_step_flips call: as many turns' flips boards as fit in ~1 GiB per strip
// (5120^2: 319 turns; 512^2: 1024; 65536^2: 2).  Every rank of a rank-mode board gets the same
// capacity (that of the largest strip, plan_rows), so a call that fits on one rank fits on all and
// no rank fails alone while the others block in the halo exchange.
static int64_t ring_capacity(golhip_t h) {
    int64_t rows = std::max<int64_t>(1, plan_rows(h));
    for (auto &s : h->shards) rows = std::max(rows, s.rows);
    const int64_t board = rows * h->pitch * 4;
    return std::max<int64_t>(1, std::min<int64_t>(1024, ((int64_t)1 << 30) / board));
}

int golhip_flips_ring_capacity(golhip_t h, int64_t *out) {
    if (!h || !out) return GOLHIP_ERR_ARG;
    *out = ring_capacity(h);
    return GOLHIP_OK;
}

// The per-turn flips ring: allocated once per engine (ring_capacity turns of strip-sized slots).
static int ensure_ring(golhip_t h, int64_t rc_cap) {
    if (h->ring_cap < rc_cap) {
        for (auto &s : h->shards) {
            HIPCHK(h, hipSetDevice(s.device));
            SYNCCHK(h, s.compute);
            if (s.ring) HIPCHK(h, hipFree(s.ring));
            s.ring = nullptr;
            HIPCHK(h, hipMalloc(&s.ring, sizeof(uint32_t) * (size_t)(rc_cap * s.rows * h->pitch)));
            int rc = ensure_extract_scratch(h, s, rc_cap * s.rows, rc_cap);
            if (rc) return rc;
        }
        h->ring_cap = rc_cap;
    }
    return GOLHIP_OK;
}

int golhip_step_flips(golhip_t h, int64_t turns, int32_t *xy, size_t cap, size_t *n,
                      uint64_t *flips_per_turn, uint64_t *alive_per_turn) {
    if (!h || turns < 0 || !n) return GOLHIP_ERR_ARG;
    const int64_t rc_cap = ring_capacity(h);
    if (turns > rc_cap)
        return fail(h, GOLHIP_ERR_ARG, "%lld turns exceed the flips ring (%lld turns)",
                    (long long)turns, (long long)rc_cap);
    *n = 0;
    if (turns == 0) return GOLHIP_OK;
    int rc = ensure_ring(h, rc_cap);
    if (rc) return rc;
    rc = run_steps(h, turns, alive_per_turn, true);
    if (rc) return rc;
    h->ring_turns = turns;
    std::vector<const uint32_t *> a, b(h->shards.size(), nullptr);
    for (auto &s : h->shards) a.push_back(s.ring);
    return extract_cells(h, a, b, turns, xy, cap, n, flips_per_turn);
}

int golhip_flips_fetch(golhip_t h, int32_t *xy, size_t cap, size_t *n, uint64_t *flips_per_turn) {
    if (!h || !n) return GOLHIP_ERR_ARG;
    if (h->ring_turns == 0)
        return fail(h, GOLHIP_ERR_STATE, "no golhip_step_flips call holds flips in the ring");
    int rc = sync_all(h);
    if (rc) return rc;
    std::vector<const uint32_t *> a, b(h->shards.size(), nullptr);
    for (auto &s : h->shards) a.push_back(s.ring);
    return extract_cells(h, a, b, h->ring_turns, xy, cap, n, flips_per_turn);
}

// The flips ring as x-only rows (golhip_step_flips_rows / golhip_flips_fetch_rows): one strip
// per handle, width <= 65536.  row_offsets (slots * rows + 1 entries) = the exclusive scan of the
// ring's row counts, copied straight from the extraction scan; x = the cells' x as uint16 in the
// same order: 2 bytes per flip instead of the 8 of an (x, y) pair.
int extract_rows(golhip_t h, int64_t slots, uint16_t *x, size_t cap, size_t *n,
                 uint64_t *row_offsets) {
    Shard &s = h->shards[0];
    const int64_t rows = s.rows * slots;
    int rc = ensure_extract_scratch(h, s, rows, slots);
    if (rc) return rc;
    HIPCHK(h, hipSetDevice(s.device));
    HIPCHK(h, golhip::launch_extract_count(s.ring, nullptr, h->pitch, rows, h->width, s.ex_rowcounts,
                                           s.ex_offsets, s.ex_block_sums, s.compute));
    HIPCHK(h, hipMemcpyAsync(row_offsets, s.ex_offsets, sizeof(uint64_t) * (size_t)(rows + 1),
                             hipMemcpyDeviceToHost, s.compute));
    SYNCCHK(h, s.compute);
    const size_t total = (size_t)row_offsets[rows];
    *n = total;
    if (total > cap) return fail(h, GOLHIP_ERR_CAP, "%zu cells do not fit in cap %zu", total, cap);
    if (total == 0) return GOLHIP_OK;
    if (!x) return fail(h, GOLHIP_ERR_ARG, "x is null");
    if (total > s.ex_xy_cap) {  // the (x, y) list's device buffer holds 4x as many x-only cells
        if (s.ex_xy) HIPCHK(h, hipFree(s.ex_xy));
        s.ex_xy = nullptr;
        const size_t want = std::max(total, s.ex_xy_cap * 2);
        HIPCHK(h, hipMalloc(&s.ex_xy, sizeof(int32_t) * 2 * want));
        s.ex_xy_cap = want;
    }
    uint16_t *dx = reinterpret_cast<uint16_t *>(s.ex_xy);
    HIPCHK(h, golhip::launch_extract_emit_x16(s.ring, nullptr, h->pitch, rows, h->width, s.ex_offsets,
                                              dx, total, s.compute));
    HIPCHK(h, hipMemcpyAsync(x, dx, sizeof(uint16_t) * total, hipMemcpyDeviceToHost, s.compute));
    SYNCCHK(h, s.compute);
    return GOLHIP_OK;
}

static int rows_api_check(golhip_t h, uint64_t *row_offsets, size_t *n) {
    if (!h || !n || !row_offsets) return GOLHIP_ERR_ARG;
    if (h->shards.size() != 1)
        return fail(h, GOLHIP_ERR_STATE, "flips rows: one strip per handle (%zu here)", h->shards.size());
    if (h->width > 65536)
        return fail(h, GOLHIP_ERR_ARG, "flips rows: x is uint16, width %lld > 65536", (long long)h->width);
    return GOLHIP_OK;
}

int golhip_step_flips_rows(golhip_t h, int64_t turns, uint16_t *x, size_t cap, size_t *n,
                           uint64_t *row_offsets, uint64_t *alive_per_turn) {
    int rc = rows_api_check(h, row_offsets, n);
    if (rc) return rc;
    if (turns < 0) return GOLHIP_ERR_ARG;
    const int64_t rc_cap = ring_capacity(h);
    if (turns > rc_cap)
        return fail(h, GOLHIP_ERR_ARG, "%lld turns exceed the flips ring (%lld turns)",
                    (long long)turns, (long long)rc_cap);
    *n = 0;
    row_offsets[0] = 0;
    if (turns == 0) return GOLHIP_OK;
    rc = ensure_ring(h, rc_cap);
    if (rc) return rc;
    rc = run_steps(h, turns, alive_per_turn, true);
    if (rc) return rc;
    h->ring_turns = turns;
    return extract_rows(h, turns, x, cap, n, row_offsets);
}

int golhip_flips_fetch_rows(golhip_t h, uint16_t *x, size_t cap, size_t *n, uint64_t *row_offsets) {
    int rc = rows_api_check(h, row_offsets, n);
    if (rc) return rc;
    if (h->ring_turns == 0)
        return fail(h, GOLHIP_ERR_STATE, "no golhip_step_flips call holds flips in the ring");
    rc = sync_all(h);
    if (rc) return rc;
    return extract_rows(h, h->ring_turns, x, cap, n, row_offsets);
}

int golhip_track_flips(golhip_t h, int enable) {
    if (!h) return GOLHIP_ERR_ARG;
    if (enable && !variant_writes_flips(h->variant))
        return fail(h, GOLHIP_ERR_STATE,
                    "flips need a production kernel variant (tuning variant %d cannot write them)",
                    h->variant);
    h->track_flips = enable != 0;
    if (h->track_flips)
        for (auto &s : h->shards)
            if (!s.diffbuf) {
                HIPCHK(h, hipSetDevice(s.device));
                HIPCHK(h, hipMalloc(&s.diffbuf, sizeof(uint32_t) * (size_t)(s.rows * h->pitch)));
            }
    return GOLHIP_OK;
}

// ---- checkpoint (the broker's paused worldSave/turn/size, broker/broker.go:124-155) ----------
// File: a 64-byte little-endian header, then the handle's rows as packed bits, LSB-first
// (bit b of byte i of a row is x = 8i + b; the bits past `width` in a row's last byte are 0).
struct CkptHeader {
    char magic[8];  // "GOLCKPT1"
    uint32_t version, header_bytes;
    int64_t width, height, y0, rows, turn;
    uint64_t row_bytes;
};
static_assert(sizeof(CkptHeader) == 64, "checkpoint header layout");
static const char kCkptMagic[8] = {'G', 'O', 'L', 'C', 'K', 'P', 'T', '1'};

static int read_ckpt_header(FILE *f, CkptHeader *hd) {
    if (std::fread(hd, sizeof *hd, 1, f) != 1) return GOLHIP_ERR_ARG;
    if (std::memcmp(hd->magic, kCkptMagic, 8) != 0 || hd->version != 1 ||
        hd->header_bytes != sizeof *hd || hd->width <= 0 || hd->height <= 0 || hd->rows <= 0 ||
        hd->row_bytes != (uint64_t)((hd->width + 7) / 8) || hd->turn < 0)
        return GOLHIP_ERR_ARG;
    return GOLHIP_OK;
}

int golhip_checkpoint_info(const char *path, int64_t *width, int64_t *height, int64_t *turn) {
    if (!path) return GOLHIP_ERR_ARG;
    FILE *f = std::fopen(path, "rb");
    if (!f) return GOLHIP_ERR_ARG;
    CkptHeader hd;
    const int rc = read_ckpt_header(f, &hd);
    std::fclose(f);
    if (rc) return rc;
    if (width) *width = hd.width;
    if (height) *height = hd.height;
    if (turn) *turn = hd.turn;
    return GOLHIP_OK;
}

// Rows [y, y + nr) of a shard <-> packed host rows (row_bytes each).  Widths that are a multiple
// of 128 are the torus rows themselves (one 2-D copy); other widths go through the byte codec,
// which also restores the horizontal replication of the torus on load.
static int ckpt_rows(golhip_t h, Shard &s, int64_t y, int64_t nr, uint8_t *host, bool to_device) {
    const int64_t W = h->width, rb = (W + 7) / 8;
    uint32_t *dev = h->row0(s, h->cur) + y * h->pitch;
    HIPCHK(h, hipSetDevice(s.device));
    if (W % 128 == 0) {
        if (to_device)
            HIPCHK(h, hipMemcpy2DAsync(dev, (size_t)h->pitch * 4, host, (size_t)rb, (size_t)rb,
                                       (size_t)nr, hipMemcpyHostToDevice, s.compute));
        else
            HIPCHK(h, hipMemcpy2DAsync(host, (size_t)rb, dev, (size_t)h->pitch * 4, (size_t)rb,
                                       (size_t)nr, hipMemcpyDeviceToHost, s.compute));
        SYNCCHK(h, s.compute);
        return GOLHIP_OK;
    }
    // the byte codec in row chunks through the shard's stage
    const int64_t cr = std::max<int64_t>(1, s.stage_bytes / W);
    std::vector<uint8_t> bytes((size_t)(std::min(cr, nr) * W));
    uint8_t *stage = s.stage;
    for (int64_t y0 = 0; y0 < nr; y0 += cr) {
        const int64_t n = std::min(cr, nr - y0);
        const size_t nb = (size_t)(n * W);
        uint8_t *hrows = host + y0 * rb;
        uint32_t *drows = dev + y0 * h->pitch;
        if (to_device) {
            for (int64_t r = 0; r < n; ++r)
                for (int64_t x = 0; x < W; ++x)
                    bytes[(size_t)(r * W + x)] = (hrows[r * rb + x / 8] >> (x % 8)) & 1 ? 255 : 0;
            HIPCHK(h, hipMemcpyAsync(stage, bytes.data(), nb, hipMemcpyHostToDevice, s.compute));
            HIPCHK(h, golhip::launch_pack(stage, n, W, h->wd, drows, h->pitch, s.compute));
            SYNCCHK(h, s.compute);
        } else {
            HIPCHK(h, golhip::launch_unpack(drows, h->pitch, n, W, stage, s.compute));
            HIPCHK(h, hipMemcpyAsync(bytes.data(), stage, nb, hipMemcpyDeviceToHost, s.compute));
            SYNCCHK(h, s.compute);
            std::memset(hrows, 0, (size_t)(n * rb));
            for (int64_t r = 0; r < n; ++r)
                for (int64_t x = 0; x < W; ++x)
                    if (bytes[(size_t)(r * W + x)]) hrows[r * rb + x / 8] |= (uint8_t)(1u << (x % 8));
        }
    }
    return GOLHIP_OK;
}

int golhip_checkpoint_save(golhip_t h, const char *path) {
    if (!h || !path) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    const std::string tmp = std::string(path) + ".tmp";
    FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f) return fail(h, GOLHIP_ERR_ARG, "cannot write %s", tmp.c_str());
    CkptHeader hd{};
    std::memcpy(hd.magic, kCkptMagic, 8);
    hd.version = 1;
    hd.header_bytes = sizeof hd;
    hd.width = h->width;
    hd.height = h->height;
    hd.y0 = h->shards.front().y0;
    hd.rows = 0;
    for (auto &s : h->shards) hd.rows += s.rows;
    hd.turn = h->turn;
    hd.row_bytes = (uint64_t)((h->width + 7) / 8);
    bool ok = std::fwrite(&hd, sizeof hd, 1, f) == 1;
    const int64_t chunk = std::max<int64_t>(1, (64ll << 20) / (int64_t)hd.row_bytes);
    std::vector<uint8_t> buf;
    for (auto &s : h->shards)
        for (int64_t y = 0; ok && y < s.rows; y += chunk) {
            const int64_t nr = std::min(chunk, s.rows - y);
            buf.resize((size_t)(nr * (int64_t)hd.row_bytes));
            if ((rc = ckpt_rows(h, s, y, nr, buf.data(), false))) break;
            ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
        }
    ok = (std::fclose(f) == 0) && ok;
    if (rc || !ok) {
        std::remove(tmp.c_str());
        return rc ? rc : fail(h, GOLHIP_ERR_ARG, "short write to %s", tmp.c_str());
    }
    if (std::rename(tmp.c_str(), path) != 0) {  // atomic replace: never a half-written checkpoint
        std::remove(tmp.c_str());
        return fail(h, GOLHIP_ERR_ARG, "cannot rename %s to %s", tmp.c_str(), path);
    }
    return GOLHIP_OK;
}

int golhip_checkpoint_load(golhip_t h, const char *path) {
    if (!h || !path) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    FILE *f = std::fopen(path, "rb");
    if (!f) return fail(h, GOLHIP_ERR_ARG, "cannot read %s", path);
    CkptHeader hd;
    if ((rc = read_ckpt_header(f, &hd))) {
        std::fclose(f);
        return fail(h, rc, "%s is not a golhip checkpoint", path);
    }
    int64_t rows = 0;
    for (auto &s : h->shards) rows += s.rows;
    if (hd.width != h->width || hd.height != h->height || hd.y0 != h->shards.front().y0 ||
        hd.rows != rows) {
        std::fclose(f);
        return fail(h, GOLHIP_ERR_STATE,
                    "checkpoint holds rows [%lld, %lld) of a %lldx%lld board, this handle rows "
                    "[%lld, %lld) of %lldx%lld",
                    (long long)hd.y0, (long long)(hd.y0 + hd.rows), (long long)hd.width,
                    (long long)hd.height, (long long)h->shards.front().y0,
                    (long long)(h->shards.front().y0 + rows), (long long)h->width,
                    (long long)h->height);
    }
    const int64_t chunk = std::max<int64_t>(1, (64ll << 20) / (int64_t)hd.row_bytes);
    std::vector<uint8_t> buf;
    bool ok = true;
    for (auto &s : h->shards)
        for (int64_t y = 0; ok && y < s.rows; y += chunk) {
            const int64_t nr = std::min(chunk, s.rows - y);
            buf.resize((size_t)(nr * (int64_t)hd.row_bytes));
            ok = std::fread(buf.data(), 1, buf.size(), f) == buf.size();
            if (ok && (rc = ckpt_rows(h, s, y, nr, buf.data(), true))) break;
        }
    std::fclose(f);
    if (rc) return rc;
    if (!ok) return fail(h, GOLHIP_ERR_ARG, "%s is truncated", path);
    h->turn = hd.turn;
    h->prev_valid = false;
    h->diff_valid = false;
    return GOLHIP_OK;
}

int golhip_launch_kind(golhip_t h, int k, int *kind, int *param) {
    return golhip_launch_kind_counts(h, k, 0, kind, param);
}

int golhip_launch_kind_counts(golhip_t h, int k, int counting, int *kind, int *param) {
    if (!h || !kind || !param || k < 1 || k > golhip::kMaxK) return GOLHIP_ERR_ARG;
    *kind = 0;
    *param = 0;
    if (h->split) return GOLHIP_OK;  // strips: the streaming kernel around the halo exchange
    const int64_t rows = h->shards[0].rows;
    if (const RegKernel rk = pick_reg_kernel(h, rows, k, counting != 0); rk.kind) {
        *kind = rk.kind;
        *param = rk.kind == 2 ? rk.T : (rk.NC != 4 ? rk.NC * 10000 : 0) + rk.W * 100 + rk.S;
    } else if (const int S = pick_split(h, rows, k); S > 1) {
        *kind = 1;
        *param = S;
    }
    return GOLHIP_OK;
}

int golhip_launch_plan(int64_t width, int64_t height, int strips, int k, int64_t turns,
                       int32_t *depths, size_t cap, size_t *n) {
    if (width <= 0 || height <= 0 || strips <= 0 || k < 1 || k > golhip::kMaxK || turns < 0 || !n)
        return GOLHIP_ERR_ARG;
    const double cells = (double)lcm64(width, 128) * (double)height;
    const double strip_cells = (double)lcm64(width, 128) * (double)strip_plan_rows(height, strips);
    const int Kfull = pick_k(k);
    // the engine's automatic choice for one strip: the register slab where the streaming kernel
    // would have at most kSlabMaxWaves1PerCu minimal-band waves per CU (256 CUs), else streaming
    // (pick_reg_kernel)
    const int64_t wd = lcm64(width, 128) / 32;
    const int64_t per = golhip::chunk_words(Kfull, golhip::kVariantProd);
    const int64_t waves1 = (height + std::max(Kfull, 8) - 1) / std::max(Kfull, 8) * ((wd + per - 1) / per);
    const bool stream = strips > 1 || !golhip::stencil_slab_supported(Kfull, 8, Kfull == 16 ? 12 : 8,
                                                                       Kfull == 16 ? 9 : 4) ||
                        waves1 > kSlabMaxWaves1PerCu * 256;
    LaunchPlanner plan(strip_cells, k, turns, strips == 1 && small_board(cells, Kfull), false, false,
                       4096, stream);
    size_t cnt = 0;
    while (plan.left > 0) {
        const int K = plan.next();
        if (depths && cnt < cap) depths[cnt] = K == 0 ? -(plan.last_M * plan.Kfull) : K;
        ++cnt;
    }
    *n = cnt;
    return cnt > cap && depths ? GOLHIP_ERR_CAP : GOLHIP_OK;
}

int golhip_alive_count(golhip_t h, uint64_t *out) {
    if (!h || !out) return GOLHIP_ERR_ARG;
    std::vector<unsigned long long *> bufs;
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        HIPCHK(h, hipMemsetAsync(s.scratch_u64, 0, sizeof(unsigned long long), s.compute));
        HIPCHK(h, golhip::launch_popcount(h->row0(s, h->cur), h->pitch, s.rows, h->wd,
                                          s.scratch_u64, s.compute));
        bufs.push_back(s.scratch_u64);
    }
    uint64_t v = 0;
    int rc = reduce_u64(h, bufs, 1, &v);
    if (rc) return rc;
    *out = v / (uint64_t)h->rep();
    return GOLHIP_OK;
}

int golhip_alive_cells(golhip_t h, int32_t *xy, size_t cap, size_t *n) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    std::vector<const uint32_t *> a, b(h->shards.size(), nullptr);
    for (auto &s : h->shards) a.push_back(h->row0(s, h->cur));
    return extract_cells(h, a, b, 1, xy, cap, n, nullptr);
}

int golhip_flips(golhip_t h, int32_t *xy, size_t cap, size_t *n) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    std::vector<const uint32_t *> a, b(h->shards.size(), nullptr);
    if (h->diff_valid) {  // written by the last launch beside its output
        for (auto &s : h->shards) a.push_back(s.diffbuf);
    } else if (h->prev_valid) {  // a one-generation launch: XOR with the buffer it read
        b.clear();
        for (auto &s : h->shards) {
            a.push_back(h->row0(s, h->cur));
            b.push_back(h->row0(s, h->cur ^ 1));
        }
    } else {
        if (n) *n = 0;
        return fail(h, GOLHIP_ERR_STATE,
                    "flips of the last generation are not held: enable golhip_track_flips (or "
                    "step by 1 turn) before stepping");
    }
    return extract_cells(h, a, b, 1, xy, cap, n, nullptr);
}

int golhip_turn(golhip_t h, int64_t *out) {
    if (!h || !out) return GOLHIP_ERR_ARG;
    *out = h->turn;
    return GOLHIP_OK;
}

int golhip_set_turn(golhip_t h, int64_t turn) {
    if (!h || turn < 0) return GOLHIP_ERR_ARG;
    h->turn = turn;
    return GOLHIP_OK;
}

int golhip_set_k(golhip_t h, int k) {
    if (!h) return GOLHIP_ERR_ARG;
    if (k < 1 || k > golhip::kMaxK) return fail(h, GOLHIP_ERR_ARG, "k must be 1..%d", golhip::kMaxK);
    if (h->split && k > h->halo)
        return fail(h, GOLHIP_ERR_ARG, "k=%d exceeds the %d halo rows allocated at create", k,
                    h->halo);
    h->k = k;
    return GOLHIP_OK;
}

int golhip_set_fixed_k(golhip_t h, int fixed) {
    if (!h) return GOLHIP_ERR_ARG;
    h->fixed_k = fixed != 0;
    return GOLHIP_OK;
}

int golhip_set_band_rows(golhip_t h, int band_rows) {
    if (!h || band_rows < 0) return GOLHIP_ERR_ARG;
    h->band_rows = band_rows;
    return GOLHIP_OK;
}

int golhip_set_graphs(golhip_t h, int mode) {
    if (!h || mode < -1 || mode > 1) return GOLHIP_ERR_ARG;
    h->graph_mode = mode;
    return GOLHIP_OK;
}

int golhip_set_count_window(golhip_t h, int generations) {
    if (!h || generations < kCountWindowMin) return GOLHIP_ERR_ARG;
    if (generations == h->count_window) return GOLHIP_OK;
    int rc = sync_all(h);
    if (rc) return rc;
    // the slots are zero between calls (every finalize re-zeroes what it summed); captured counting
    // graphs bake the old slot array in, so they go
    for (auto &g : h->graphs) (void)hipGraphExecDestroy(g.exec);
    h->graphs.clear();
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        if (s.slots) HIPCHK(h, hipFree(s.slots));
        s.slots = nullptr;
        const size_t bytes = sizeof(unsigned long long) * (size_t)generations * golhip::kCountSlots;
        HIPCHK(h, hipMalloc(&s.slots, bytes));
        HIPCHK(h, hipMemsetAsync(s.slots, 0, bytes, s.compute));
        SYNCCHK(h, s.compute);
    }
    h->count_window = generations;
    return GOLHIP_OK;
}

int golhip_set_comm_timeout(golhip_t h, int64_t ms) {
    if (ms <= 0) return GOLHIP_ERR_ARG;
    if (h)
        h->comm_timeout_ms = ms;
    else
        g_comm_timeout_ms.store(ms);
    return GOLHIP_OK;
}

int golhip_set_tail_bands(golhip_t h, int bands, int rows) {
    if (!h || bands < 0 || rows < 0) return GOLHIP_ERR_ARG;
    h->tail_bands = bands;
    h->tail_rows = rows;
    return GOLHIP_OK;
}

int golhip_sync(golhip_t h) {
    if (!h) return GOLHIP_ERR_ARG;
    return sync_all(h);
}

int golhip_timing(golhip_t h, int enable) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = timing_collect(h);
    if (rc) return rc;
    h->timing = enable != 0;
    h->tms = 0.0;
    h->tlaunches = 0;
    h->tgens = 0;
    // create the event pairs now: a hipEventCreate inside the first timed golhip_step call would
    // add its host cost to a caller's timed region (a 20-turn region is ~0.75 ms)
    if (h->timing) {
        HIPCHK(h, hipSetDevice(h->shards[0].device));
        while (h->tpool.size() < 4) {
            TimingPair tp;
            HIPCHK(h, hipEventCreate(&tp.a));
            HIPCHK(h, hipEventCreate(&tp.b));
            h->tpool.push_back(tp);
        }
    }
    return GOLHIP_OK;
}

int golhip_kernel_time(golhip_t h, double *total_ms, int64_t *launches, int64_t *generations) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = timing_collect(h);
    if (rc) return rc;
    if (total_ms) *total_ms = h->tms;
    if (launches) *launches = h->tlaunches;
    if (generations) *generations = h->tgens;
    return GOLHIP_OK;
}

}  // extern "C"
