// golhip_engine.hip -- the core of libgolhip's host side: handles and their device memory, the step
// loop behind golhip_step (one K-block per launch, interior / boundary bands of split boards,
// captured graph replays of small boards), per-call timing and the setters of the C ABI
// (include/golhip.h).  The planner, the exchange, cell extraction and host I/O live in
// engine_plan.hip / engine_comm.hip / engine_cells.hip / engine_io.hip (golhip_engine.hpp).
//
// Reference role: gol/distributor.go:45-67 (Call: one Broker.Publish RPC per turn, the whole world
// out and back) -> golhip_step(h, n): n turns device-side, the board resident in HBM.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>

#include "golhip_engine.hpp"

namespace golhip {

thread_local std::string g_create_error;

namespace {
const EngineHooks *g_hooks = nullptr;  // set by the tuning library's TU when it loads
}  // namespace

const EngineHooks *engine_hooks() { return g_hooks; }
void set_engine_hooks(const EngineHooks *hooks) { g_hooks = hooks; }

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

int64_t lcm64(int64_t a, int64_t b) { return a / std::gcd(a, b) * b; }

int check_device_arch(golhip_t h, int device) {
    hipDeviceProp_t prop;
    HIPCHK(h, hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(h, GOLHIP_ERR_NODEV, "device %d is %s, libgolhip is built for gfx950", device, prop.gcnArchName);
    return GOLHIP_OK;
}

namespace {

int alloc_shard(golhip_t h, Shard &s) {
    HIPCHK(h, hipSetDevice(s.device));
    HIPCHK(h, hipStreamCreateWithFlags(&s.compute, hipStreamNonBlocking));
    // comm and edge streams at the default priority: high-priority queues for them (so the bands'
    // few workgroups dispatch ahead of the interior's) ran the 65536^2 ring of one 16 % SLOWER over
    // 1000 turns (r04g vs r04f, profiles/r04/r04h_edge_ab_p*.log); a tuning selector (edge_prio)
    int lo_prio = 0, hi_prio = 0;
    HIPCHK(h, hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
    const int edge_prio = h->edge_prio ? hi_prio : lo_prio;
    HIPCHK(h, hipStreamCreateWithPriority(&s.comm, hipStreamNonBlocking, edge_prio));
    HIPCHK(h, hipStreamCreateWithPriority(&s.edge, hipStreamNonBlocking, edge_prio));
    HIPCHK(h, hipEventCreateWithFlags(&s.ev_ready, hipEventDisableTiming));
    HIPCHK(h, hipEventCreateWithFlags(&s.ev_halo, hipEventDisableTiming));
    HIPCHK(h, hipEventCreateWithFlags(&s.ev_edge, hipEventDisableTiming));
    const size_t words = (size_t)(s.rows + 2 * (int64_t)h->halo) * (size_t)h->pitch;
    for (int i = 0; i < 2; ++i) {
        HIPCHK(h, hipMalloc(&s.buf[i], words * sizeof(uint32_t)));
        HIPCHK(h, hipMemsetAsync(s.buf[i], 0, words * sizeof(uint32_t), s.compute));
    }
    HIPCHK(h, hipMalloc(&s.slots, sizeof(unsigned long long) * h->count_window * kCountSlots));
    HIPCHK(h, hipMemsetAsync(s.slots, 0, sizeof(unsigned long long) * h->count_window * kCountSlots, s.compute));
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

}  // namespace

void free_shard(Shard &s, int64_t drain_ms, bool comm_failed) {
    (void)hipSetDevice(s.device);
    // a failed communicator is aborted first: ncclCommAbort makes the RCCL kernels still spinning on
    // a transfer that will never complete (and the ones queued behind them) exit, so the streams
    // can drain.  Measured on two real RCCL ranks with a receive whose send never comes and three
    // RCCL operations in flight: abort 0.5 s, drain 10 ms, no GPU fault, the next process on the
    // GPU bit-exact (profiles/r05/r05d_stuck_rccl_receive_abort.log)
    // one deadline for the abort and all of the shard's streams: after a real peer hang every one of
    // them can be stuck, and destroy must not wait 3 x the comm timeout
    const Clock::time_point end = Clock::now() + std::chrono::milliseconds(std::max<int64_t>(0, drain_ms));
    if (comm_failed && s.comm_nccl) {
        const bool aborted = comm_abort_within(s.comm_nccl, std::max<int64_t>(1, drain_ms));
        s.comm_nccl = nullptr;
        if (!aborted) {  // something other than RCCL holds the device: leave it all to the teardown
            s = Shard{};
            return;
        }
    }
    bool drained = true;
    for (hipStream_t st : {s.compute, s.comm, s.edge}) {
        if (!st) continue;
        if (drain_ms <= 0) {
            (void)hipStreamSynchronize(st);
            continue;
        }
        hipError_t e;
        while ((e = hipStreamQuery(st)) == hipErrorNotReady && Clock::now() < end)
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        drained = drained && e != hipErrorNotReady;
    }
    // a stream still stuck keeps what it may touch (and its communicator)
    if (s.comm_nccl && drained) (void)ncclCommDestroy(s.comm_nccl);
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
                    (void *)s.ex_slot_counts, (void *)s.ex_xy, (void *)s.stage, (void *)s.ex_block_sums,
                    (void *)s.act, (void *)s.act_stats, (void *)s.pflags, (void *)s.psave})
        if (q) (void)hipFree(q);
    if (s.ev_ready) (void)hipEventDestroy(s.ev_ready);
    if (s.ev_halo) (void)hipEventDestroy(s.ev_halo);
    if (s.ev_edge) (void)hipEventDestroy(s.ev_edge);
    if (s.compute) (void)hipStreamDestroy(s.compute);
    if (s.comm) (void)hipStreamDestroy(s.comm);
    if (s.edge) (void)hipStreamDestroy(s.edge);
    s = Shard{};
}

int validate_geometry(int width, int height, int world, int k) {
    if (width <= 0 || height <= 0 || world <= 0) return GOLHIP_ERR_ARG;
    if (k < 1 || k > kMaxK) return GOLHIP_ERR_ARG;
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
    // the tuning library's A/B selectors (read at create); the production library has no hooks and
    // reads none of them: a stray variable cannot change its kernels
    if (const EngineHooks *hk = engine_hooks(); hk && hk->configure) hk->configure(h);
    return GOLHIP_OK;
}

int create_common(golhip_t h) {
    if (const EngineHooks *hk = engine_hooks(); hk && hk->create) {
        int rc = hk->create(h);
        if (rc) return rc;
    }
    for (auto &s : h->shards) {
        int rc = alloc_shard(h, s);
        if (rc) return rc;
        // each launch depth is its own code object, loaded at its first launch (~1 ms): load them
        // all now, not inside the first timed or latency-sensitive step
        HIPCHK(h, warm_stencils(h->variant, s.compute));
        SYNCCHK(h, s.compute);
    }
    return GOLHIP_OK;
}

namespace {

// calls up to this many turns return their counts pinned, if their plan replays no graph: a
// replayed graph copies its counts per replay, and into pinned memory that copy cost more than the
// one device-to-host copy it saves (pinned counts up to 4096 turns: 1600 turns at 512^2 0.570 ->
// 0.705 us/turn, profiles/r04/r04pk2_depths.log; 127 turns: r04pw_narrow.log).  The plan decides,
// not the turn count alone: at K = 12 / 14 a graph is 120 / 112 generations (round-4 advice).
constexpr int64_t kPinnedCountTurns = 127;

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

// The next event pair of the edge-join timing (grown on demand; reused after timing_collect).
int edge_pair(golhip_t h, TimingPair **out) {
    if (h->tedge_used == h->tedge.size()) {
        TimingPair tp;
        HIPCHK(h, hipEventCreate(&tp.a));
        HIPCHK(h, hipEventCreate(&tp.b));
        h->tedge.push_back(tp);
    }
    *out = &h->tedge[h->tedge_used++];
    return GOLHIP_OK;
}

int timing_collect(golhip_t h) {
    for (size_t i = 0; i < h->tedge_used; ++i) {  // recorded before the call's stop event
        const hipEvent_t ev = h->tedge[i].b;
        if (rccl_waits(h)) {
            int rc = poll_until(h, "a timed boundary-band join behind the RCCL transfers", [&]() -> int {
                const hipError_t e = hipEventQuery(ev);
                return e == hipSuccess ? 0
                       : e == hipErrorNotReady
                           ? 1
                           : fail(h, GOLHIP_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(e));
            });
            if (rc) return rc;
        }
        HIPCHK(h, hipEventSynchronize(ev));
        float ms = 0.f;
        HIPCHK(h, hipEventElapsedTime(&ms, h->tedge[i].a, ev));
        h->tedge_ms += ms;
        h->tedge_blocks += 1;
    }
    h->tedge_used = 0;
    if (h->tused == 0) return GOLHIP_OK;
    HIPCHK(h, hipSetDevice(h->shards[0].device));
    for (size_t i = 0; i < h->tused; ++i) {
        if (rccl_waits(h)) {
            const hipEvent_t ev = h->tpool[i].b;
            int rc = poll_until(h, "a timed launch behind the RCCL transfers", [&]() -> int {
                const hipError_t e = hipEventQuery(ev);
                return e == hipSuccess ? 0
                       : e == hipErrorNotReady
                           ? 1
                           : fail(h, GOLHIP_ERR_HIP, "hipEventQuery: %s", hipGetErrorString(e));
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

// One K-generation block on every shard.  slot_gen >= 0: count the K generations into the count
// window at generation slot_gen (finalized later by flush_counts_window), -1: no counts.
// diff_slot: kDiffNone no flips, kDiffLast the last generation's flips into diffbuf, t >= 0 into
// flips ring slot t (the launch's last generation's flips are written beside its output).
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
    const EngineHooks *hk = engine_hooks();
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        unsigned long long *slots = slot_gen >= 0 ? s.slots + slot_gen * kCountSlots : nullptr;
        const uint32_t *in = h->row0(s, h->cur);
        uint32_t *out = h->row0(s, nxt);
        uint32_t *diff = diff_slot == kDiffLast ? s.diffbuf
                         : diff_slot >= 0      ? s.ring + diff_slot * s.rows * h->pitch
                                               : nullptr;
        if (!h->split) {
            StencilParams p = make_params(h, s, K, 0, s.rows, 0, 0, 0, slots != nullptr);
            p.diff = diff;
            if (hk && hk->launch_params) hk->launch_params(h, s, K, slots != nullptr, p);  // tuning: stamps
            // a K-deep ring launch (ring_depth: a production register slab) writes the flips of
            // each of its K generations into K consecutive ring slots
            p.diff_stride = diff_slot >= 0 && K > 1 ? s.rows * h->pitch : 0;
            if (!diff) {  // stable-slab skipping: its flags (allocated here, outside any capture)
                int rc = ensure_activity(h, s, K, slots != nullptr);
                if (rc) return rc;
            }
            HIPCHK(h, launch_auto(h, K, in, out, p, slots, s.compute, &s, h->cur));
        } else if (s.rows >= 3 * K) {
            h->act_valid = false;
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
                HIPCHK(h, launch_stencil(K, h->variant, in, out, pi, slots, s.compute));
                int rc = exchange_halos(h, K, false);
                if (rc) return rc;
            } else if (!h->edge_first) {
                HIPCHK(h, launch_stencil(K, h->variant, in, out, pi, slots, s.compute));
            }
            HIPCHK(h, hipStreamWaitEvent(s.edge, s.ev_ready, 0));
            HIPCHK(h, hipStreamWaitEvent(s.edge, s.ev_halo, 0));
            HIPCHK(h, launch_stencil(K, h->variant, in, out, pb, slots, s.edge));
            HIPCHK(h, hipEventRecord(s.ev_edge, s.edge));
            if (h->edge_first) HIPCHK(h, launch_stencil(K, h->variant, in, out, pi, slots, s.compute));
            TimingPair *tp = nullptr;  // timing: the join's wait on the compute stream
            if (h->timing && &s == &h->shards[0]) {
                int rc = edge_pair(h, &tp);
                if (rc) return rc;
                HIPCHK(h, hipEventRecord(tp->a, s.compute));
            }
            HIPCHK(h, hipStreamWaitEvent(s.compute, s.ev_edge, 0));
            if (tp) HIPCHK(h, hipEventRecord(tp->b, s.compute));
            h->edge_k = K;
        } else {
            h->act_valid = false;
            h->edge_k = 0;
            HIPCHK(h, hipStreamWaitEvent(s.compute, s.ev_halo, 0));
            StencilParams p = make_params(h, s, K, 0, s.rows, 0, 0, 0, slots != nullptr);
            p.diff = diff;
            HIPCHK(h, launch_stencil(K, h->variant, in, out, p, slots, s.compute));
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

// One K-generation launch of the whole-board kernel (stencil_board.hip): the step_block of boards
// that fit one workgroup.  slot_gen / diff_slot as step_block's (no flips ring).
int board_block(golhip_t h, int K, int W, int R, int64_t slot_gen, int64_t diff_slot) {
    Shard &s = h->shards[0];
    HIPCHK(h, hipSetDevice(s.device));
    StencilParams p{};
    p.pitch = h->pitch;
    p.wd = h->wd;
    p.r0e = s.rows;
    p.wrap_rows = h->height;
    p.hi = s.rows;
    p.nchunks = 1;
    p.diff = diff_slot == kDiffLast ? s.diffbuf : nullptr;
    unsigned long long *slots = slot_gen >= 0 ? s.slots + slot_gen * kCountSlots : nullptr;
    HIPCHK(h, launch_stencil_board(K, W, R, h->row0(s, h->cur), h->row0(s, h->cur ^ 1), p, slots, s.compute));
    if (h->timing) {
        h->tlaunches += 1;
        h->tgens += K;
    }
    h->queued_s += (double)h->L * (double)h->height * K / 5e10 + kLaunchOverheadUs * 1e-6;
    h->cur ^= 1;
    h->turn += K;
    h->prev_valid = (K == 1);
    h->diff_valid = diff_slot == kDiffLast;
    h->act_valid = false;
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
        if (rk.kind == 3 && stencil_slab_flips_every_gen(K, rk.W, rk.S, rk.NC)) return K;
    }
    return 1;
}

// Per-generation counts of the first n window generations -> s.d_counts[off, off + n), one
// finalize launch per window (it re-zeroes the slots) instead of one per K-generation block.
int flush_counts_window(golhip_t h, int n, int64_t off) {
    if (n <= 0) return GOLHIP_OK;
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        HIPCHK(h, launch_count_finalize(n, s.slots, s.d_counts + off, s.compute));
    }
    return GOLHIP_OK;
}

// Graphs pay off when a launch is short (launch-bound): single-strip small boards.
bool graph_worthy(golhip_t h, int K) {
    if (h->split || h->shards.size() != 1) return false;
    if (h->graph_mode >= 0) return h->graph_mode != 0;  // golhip_set_graphs
    return small_board((double)h->L * (double)h->height, K);
}

int graph_for(golhip_t h, int K, int M, bool counting, hipGraphExec_t *out) {
    Shard &s = h->shards[0];
    const int64_t band = auto_band(h, s.rows, K, 0, counting);
    for (auto &g : h->graphs)
        if (g.K == K && g.M == M && g.cur == h->cur && g.counting == counting && g.band == band &&
            g.tail_bands == h->tail_bands && g.tail_rows == h->tail_rows) {
            *out = g.exec;
            h->act_valid = g.act_after;  // the flags as the replay leaves them
            std::copy(g.act_key_after, g.act_key_after + 3, h->act_key);
            return GOLHIP_OK;
        }
    HIPCHK(h, hipSetDevice(s.device));
    {
        int rc = ensure_activity(h, s, K, counting);
        if (rc) return rc;
    }
    if (counting && !h->g_counts) HIPCHK(h, hipMalloc(&h->g_counts, sizeof(unsigned long long) * kGraphGensBig * 2));
    hipGraph_t graph = nullptr;
    HIPCHK(h, hipStreamBeginCapture(s.compute, hipStreamCaptureModeThreadLocal));
    hipError_t err = hipSuccess;
    for (int i = 0; i < M && err == hipSuccess; ++i) {
        const int c = h->cur ^ (i & 1);
        StencilParams p = make_params(h, s, K, 0, s.rows, 0, 0, 0, counting);
        // the first launch of a replay recomputes the stable-slab flags (a replay must not trust
        // flags another state left)
        err = launch_auto(h, K, h->row0(s, c), h->row0(s, c ^ 1), p,
                          counting ? s.slots + (int64_t)i * K * kCountSlots : nullptr, s.compute, &s, c,
                          i == 0);
    }
    if (err == hipSuccess && counting)  // one finalize for the graph's M*K generations
        err = launch_count_finalize(M * K, s.slots, h->g_counts, s.compute);
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
    g.act_after = h->act_valid;
    std::copy(h->act_key, h->act_key + 3, g.act_key_after);
    err = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (err != hipSuccess) return fail(h, GOLHIP_ERR_HIP, "graph instantiate: %s", hipGetErrorString(err));
    h->graphs.push_back(g);
    *out = g.exec;
    return GOLHIP_OK;
}

}  // namespace

// The body of golhip_step / golhip_step_flips.  ring: every generation is its own launch writing
// its flips into ring slot t (t = 0 .. turns-1); otherwise the launch plan, and with flips
// tracking on, the last launch writes the last generation's flips.
int run_steps(golhip_t h, int64_t turns, uint64_t *alive_per_turn, bool ring) {
    if (!h || turns < 0) return GOLHIP_ERR_ARG;
    if (turns == 0) return GOLHIP_OK;
    if ((ring || h->track_flips) && !variant_writes_flips(h->variant))
        return fail(h, GOLHIP_ERR_STATE, "flips need a production kernel variant (tuning variant %d cannot write them)",
                    h->variant);
    const bool counting = alive_per_turn != nullptr;
    int bw = 0, br = 0;  // the whole-board kernel: W waves x R rows per segment
    const bool board = !ring && board_applies(h, &bw, &br);
    const int kmax = pick_k(h->k);
    const bool reg = !ring && !h->split && h->shards.size() == 1 &&
                     pick_reg_kernel(h, h->shards[0].rows, kmax, counting).kind != 0;
    const bool stream = !ring && h->shards.size() == 1 && !reg && pick_split(h, h->shards[0].rows, kmax) <= 1;
    // planned per strip (the band geometry and each GPU's launch time follow the strip), from the
    // largest strip of the board, so every rank of a rank-mode board plans the same depths.  A
    // register-slab board runs its tuned full depth (reg: fixed; best_rate_k's rates are the
    // streaming kernel's), also without graphs, where only full-depth slabs skip stable slabs
    LaunchPlanner plan((double)h->L * (double)plan_rows(h), ring ? 1 : h->k, turns, !ring && graph_worthy(h, kmax),
                       h->fixed_k || ring || reg, h->track_flips, h->count_window, stream, reg && !h->fixed_k);
    if (counting) {
        // pinned host counts for calls that replay no graph (their graph replays would copy each
        // replay's counts into it); the others keep the device buffer and one copy returns them
        // (the whole-board kernel replays no graph: one finalize per count window writes them)
        const bool host_counts = h->shards.size() == 1 && !rccl_waits(h) &&
                                 (board || (turns <= kPinnedCountTurns && !plan.replays()));
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
    const int Kfull = plan.Kfull;
    int64_t win = 0;  // generations pending in the count window, from turn offset done - win
    while (done < turns) {
        if (board) {  // one launch per count window (or kBoardMaxK generations)
            if (counting && win >= h->count_window) {
                int rc = flush_counts_window(h, (int)win, done - win);
                if (rc) return rc;
                win = 0;
            }
            int64_t K = std::min<int64_t>(turns - done, kBoardMaxK);
            if (counting) K = std::min<int64_t>(K, h->count_window - win);
            const int64_t diff_slot = h->track_flips && done + K == turns ? kDiffLast : kDiffNone;
            int rc = board_block(h, (int)K, bw, br, counting ? win : -1, diff_slot);
            if (rc) return rc;
            done += K;
            if (counting) win += K;
            continue;
        }
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
                HIPCHK(h, hipMemcpyAsync(s.d_counts + done, h->g_counts, sizeof(unsigned long long) * (size_t)M * Kfull,
                                         s.counts_host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice, s.compute));
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
    if (const EngineHooks *hk = engine_hooks(); hk && hk->after_steps) {  // tuning: fault injection
        int rc = hk->after_steps(h);
        if (rc) return rc;
    }
    if (stop) {
        HIPCHK(h, hipSetDevice(h->shards[0].device));
        HIPCHK(h, hipEventRecord(stop, h->shards[0].compute));
        if (h->tused >= 1024 || h->tedge_used >= 4096) {
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

}  // namespace golhip

using namespace golhip;

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

int golhip_destroy(golhip_t h) {
    if (!h) return GOLHIP_ERR_ARG;
    for (auto &g : h->graphs) (void)hipGraphExecDestroy(g.exec);
    if (h->g_counts) (void)hipFree(h->g_counts);
    for (auto *pool : {&h->tpool, &h->tedge})
        for (auto &tp : *pool) {
            (void)hipEventDestroy(tp.a);
            (void)hipEventDestroy(tp.b);
        }
    for (auto &s : h->shards) free_shard(s, rccl_waits(h) ? h->comm_timeout_ms : 0, h->comm_failed);
    release_rccl_ops(h);
    for (void *b : h->hc_buf)
        if (b) (void)hipHostFree(b);
    if (const EngineHooks *hk = engine_hooks(); hk && hk->destroy) hk->destroy(h);
    delete h;
    return GOLHIP_OK;
}

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

int golhip_step(golhip_t h, int64_t turns, uint64_t *alive_per_turn) {
    return run_steps(h, turns, alive_per_turn, false);
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
    if (k < 1 || k > kMaxK) return fail(h, GOLHIP_ERR_ARG, "k must be 1..%d", kMaxK);
    if (h->split && k > h->halo)
        return fail(h, GOLHIP_ERR_ARG, "k=%d exceeds the %d halo rows allocated at create", k, h->halo);
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
        const size_t bytes = sizeof(unsigned long long) * (size_t)generations * kCountSlots;
        HIPCHK(h, hipMalloc(&s.slots, bytes));
        HIPCHK(h, hipMemsetAsync(s.slots, 0, bytes, s.compute));
        SYNCCHK(h, s.compute);
    }
    h->count_window = generations;
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
    h->tedge_ms = 0.0;
    h->tedge_blocks = 0;
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

int golhip_edge_wait(golhip_t h, double *total_ms, int64_t *blocks) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = timing_collect(h);
    if (rc) return rc;
    if (total_ms) *total_ms = h->tedge_ms;
    if (blocks) *blocks = h->tedge_blocks;
    return GOLHIP_OK;
}

int golhip_set_activity(golhip_t h, int enable) {
    if (!h) return GOLHIP_ERR_ARG;
    if (enable < -1 || enable > 1) return GOLHIP_ERR_ARG;
    if (enable != h->activity && !h->graphs.empty()) {
        // captured replays bake the slab kernel (with or without skipping) in: recapture
        int rc = sync_all(h);
        if (rc) return rc;
        for (auto &g : h->graphs) (void)hipGraphExecDestroy(g.exec);
        h->graphs.clear();
    }
    h->activity = enable;
    h->act_valid = false;
    return GOLHIP_OK;
}

int golhip_activity_stats(golhip_t h, int64_t *computed, int64_t *skipped) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    unsigned long long v[2] = {0, 0};
    for (auto &s : h->shards)
        if (s.act_stats) {
            unsigned long long t[2 * kActStatSlots];
            HIPCHK(h, hipSetDevice(s.device));
            HIPCHK(h, hipMemcpy(t, s.act_stats, sizeof t, hipMemcpyDeviceToHost));
            for (int i = 0; i < 2 * kActStatSlots; ++i) v[i / kActStatSlots] += t[i];
        }
    if (computed) *computed = (int64_t)v[0];
    if (skipped) *skipped = (int64_t)v[1];
    return GOLHIP_OK;
}

int golhip_set_board_kernel(golhip_t h, int enable) {
    if (!h) return GOLHIP_ERR_ARG;
    if (enable < -1 || enable > 1) return GOLHIP_ERR_ARG;
    h->board_kernel = enable;
    return GOLHIP_OK;
}

}  // extern "C"
