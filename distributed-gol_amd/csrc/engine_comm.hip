// engine_comm.hip -- row strips over ranks: the halo exchange (RCCL send/recv, peer copies, or the
// caller's host transport), count reductions, the RCCL fail-fast waits and the rank-mode creates.
//
// Reference roles: broker/broker.go:37-56 (publish: the strip split), :58-84 (subscriberLoop: one
// RPC per server per turn, the full world out and a strip back), :168-174 (the stitch).  Here only
// K halo rows per strip edge move per K generations, and a stuck transfer fails the call at a
// deadline instead of stalling the controller forever (a dead server blocks Broker.Publish in the
// reference).
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>

#include "golhip_engine.hpp"

namespace golhip {

std::atomic<int64_t> g_comm_timeout_ms{120000};

// ---- RCCL fail-fast --------------------------------------------------------------------------
// True when device work of this handle can wait on an RCCL transfer (rank mode over RCCL: the
// boundary bands wait for the halo event, the compute stream for the boundary bands, counts for
// the all-reduce).  Only then do host waits poll; everything else synchronises directly.
bool rccl_waits(golhip_t h) { return h->rank_mode && h->split && !h->host_comm_on; }

namespace {

// Record an event behind the RCCL operation just enqueued on `st` (retiring the completed ones at
// the front first), so a failed wait can name the first incomplete operation.
int track_rccl_op(golhip_t h, hipStream_t st) {
    while (!h->rccl_ops.empty() && hipEventQuery(h->rccl_ops.front().first) == hipSuccess) {
        h->rccl_ev_pool.push_back(h->rccl_ops.front().first);
        h->rccl_ops.pop_front();
    }
    hipEvent_t ev = nullptr;
    if (!h->rccl_ev_pool.empty()) {
        ev = h->rccl_ev_pool.back();
        h->rccl_ev_pool.pop_back();
    } else {
        HIPCHK(h, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    HIPCHK(h, hipEventRecord(ev, st));
    h->rccl_ops.emplace_back(ev, h->comm_pending);
    return GOLHIP_OK;
}

// "the first incomplete of the N RCCL operations in flight: <desc>", or the last one enqueued.
std::string pending_desc(golhip_t h) {
    size_t n = 0;
    const std::string *first = nullptr;
    for (auto &op : h->rccl_ops)
        if (hipEventQuery(op.first) != hipSuccess) {
            if (!first) first = &op.second;
            ++n;
        }
    if (!first) return h->comm_pending.empty() ? "no RCCL operation pending" : h->comm_pending;
    char head[96];
    std::snprintf(head, sizeof head, "the first incomplete of %zu RCCL operations in flight: ", n);
    return head + *first;
}

// Fail the call with the pending operation named; the handle refuses device work afterwards
// (comm_failed).  Before the communicator's set-up has completed nothing of it runs on the device,
// and ncclCommAbort stops its bootstrap.  After it, the communicator is left in place until the
// caller calls golhip_comm_abort or golhip_destroy (both ncclCommAbort it: RCCL aborts the
// operations still running on the device; profiles/r05/r05d_stuck_rccl_receive_abort.log) or ends
// the process.
int comm_abort(golhip_t h, const char *why, ncclResult_t state) {
    const bool before_setup = !h->comm_setup_done;
    if (before_setup)
        for (auto &s : h->shards)
            if (s.comm_nccl) {
                (void)ncclCommAbort(s.comm_nccl);
                s.comm_nccl = nullptr;
            }
    h->comm_failed = true;
    const std::string pending = pending_desc(h);
    return fail(h, GOLHIP_ERR_RCCL, "rank %d of %d: %s: %s (communicator state: %s); %s",
                h->shards.empty() ? -1 : h->shards[0].rank, h->world_size, why, pending.c_str(),
                ncclGetErrorString(state),
                before_setup ? "communicator aborted"
                             : "communicator left in place: golhip_comm_abort / golhip_destroy abort it, "
                               "or end the process (RCCL work may still be queued)");
}

// Deadline of a wait: the handle's timeout plus 10x the modelled time of the stencil work the host
// queued since the last full sync (a long golhip_step of a big board is not a hang).
int64_t wait_budget_ms(golhip_t h) {
    return (int64_t)std::min((double)h->comm_timeout_ms + 10.0 * h->queued_s * 1e3, 3.6e6);
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

// An RCCL call on a non-blocking communicator: ncclInProgress is not an error (comm_ready waits).
#define NCCLCALL(h, what, expr)                                                                   \
    do {                                                                                          \
        ncclResult_t r_ = (expr);                                                                 \
        if (r_ != ncclSuccess && r_ != ncclInProgress) return comm_abort((h), (what), r_);        \
    } while (0)

// The 4 transfers of a K-row exchange for one strip (toroidal ring of strips).  Order matters
// when up == down (world 2): sends to `down` first and receives from `up` first, so the i-th send
// of one rank to a peer matches the i-th receive of that peer (RCCL per-peer ordering).
void halo_plan(int world, int rank, int64_t rows, int K, golhip_xfer out[4]) {
    const int up = (rank - 1 + world) % world, down = (rank + 1) % world;
    out[0] = {0, down, rows - K, K};   // my last K rows -> the top halo of the strip below
    out[1] = {0, up, 0, K};            // my first K rows -> the bottom halo of the strip above
    out[2] = {1, up, -(int64_t)K, K};  // top halo <- last K rows of the strip above
    out[3] = {1, down, rows, K};       // bottom halo <- first K rows of the strip below
}

}  // namespace

int poll_until_fn(golhip_t h, const char *what, int (*done)(void *), void *ctx) {
    const int64_t budget_ms = wait_budget_ms(h);
    const Clock::time_point deadline = Clock::now() + std::chrono::milliseconds(budget_ms);
    int spins = 0;
    for (;;) {
        const int r = done(ctx);
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

bool comm_abort_within(ncclComm_t comm, int64_t ms) {
    struct State {
        std::mutex m;
        std::condition_variable cv;
        bool done = false;
    };
    auto st = std::make_shared<State>();
    std::thread t([comm, st] {
        (void)ncclCommAbort(comm);
        std::lock_guard<std::mutex> g(st->m);
        st->done = true;
        st->cv.notify_all();
    });
    std::unique_lock<std::mutex> lk(st->m);
    const bool done = st->cv.wait_for(lk, std::chrono::milliseconds(std::max<int64_t>(1, ms)), [&] { return st->done; });
    lk.unlock();
    if (done)
        t.join();
    else
        t.detach();  // still inside ncclCommAbort: the process teardown ends it
    return done;
}

int copy_to_host(golhip_t h, void *dst, const void *src, size_t bytes, hipStream_t st) {
    if (rccl_waits(h)) SYNCCHK(h, st);
    HIPCHK(h, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    return GOLHIP_OK;
}

void strip_bounds(int64_t height, int world, int rank, int64_t &y0, int64_t &rows) {
    // balanced contiguous split (the reference's publish() splits ImageSize/numServers and hands
    // the remainder to the first strips, broker/broker.go:38-46; same coverage here, any height)
    y0 = height * rank / world;
    rows = height * (rank + 1) / world - y0;
}

// Exchange K halo rows between neighbouring strips on the comm streams.
//  * rank mode (one process per GPU): RCCL send/recv over xGMI, the plan above in one group;
//  * single process (golhip_create / golhip_create_strips): every strip pulls its two halos from
//    its neighbours' rows with peer copies (xGMI between devices, a D2D copy on one device).
// record_ready = false: the caller recorded ev_ready (the end of the previous block) itself, before
// enqueueing this block's interior (step_block's interior-first order).
int exchange_halos(golhip_t h, int K, bool record_ready) {
    const size_t bytes = (size_t)K * (size_t)h->pitch * sizeof(uint32_t);
    if (record_ready)
        for (auto &s : h->shards) {
            HIPCHK(h, hipSetDevice(s.device));
            HIPCHK(h, hipEventRecord(s.ev_ready, s.compute));
        }
    ++h->exchanges;
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
        char desc[288];
        std::snprintf(desc, sizeof desc,
                      "halo exchange #%lld of K = %d rows (%zu bytes per transfer): send rows "
                      "[%lld, +%d) -> rank %d, rows [0, +%d) -> rank %d; receive rows [-%d, ...) <- "
                      "rank %d, [%lld, ...) <- rank %d",
                      (long long)h->exchanges, K, bytes, (long long)(s.rows - K), K, plan[0].peer, K,
                      plan[1].peer, K, plan[2].peer, (long long)s.rows, plan[3].peer);
        h->comm_pending = desc;
        uint32_t *r0 = h->row0(s, h->cur);
        const EngineHooks *hk = engine_hooks();
        NCCLCALL(h, "ncclGroupStart", ncclGroupStart());
        for (int i = 0; i < 4; ++i) {
            const golhip_xfer &x = plan[i];
            if (hk && hk->skip_xfer && hk->skip_xfer(h, x, i)) continue;  // tuning: fault injection
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
        if ((rc = track_rccl_op(h, s.comm))) return rc;
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

// The events of the tracked RCCL operations (golhip_destroy).
void release_rccl_ops(golhip_t h) {
    for (auto &op : h->rccl_ops) (void)hipEventDestroy(op.first);
    for (hipEvent_t ev : h->rccl_ev_pool) (void)hipEventDestroy(ev);
    h->rccl_ops.clear();
    h->rccl_ev_pool.clear();
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
        if ((rc = track_rccl_op(h, s.compute))) return rc;
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
        int rc = copy_to_host(h, i == 0 ? out : tmp.data(), bufs[i], n * sizeof(uint64_t), s.compute);
        if (rc) return rc;
        SYNCCHK(h, s.compute);
        if (i > 0)
            for (size_t j = 0; j < n; ++j) out[j] += tmp[j];
    }
    if (h->host_comm_on && h->split && h->host_comm.allreduce_u64(h->host_comm.ctx, out, n) != 0)
        return fail(h, GOLHIP_ERR_RCCL, "host transport: all-reduce of %zu counts failed", n);
    return GOLHIP_OK;
}

}  // namespace golhip

using namespace golhip;

// ================================================================================ C ABI ====
extern "C" {

int golhip_strip_bounds(int64_t height, int world_size, int rank, int64_t *y0, int64_t *rows) {
    if (height <= 0 || world_size <= 0 || rank < 0 || rank >= world_size || !y0 || !rows)
        return GOLHIP_ERR_ARG;
    strip_bounds(height, world_size, rank, *y0, *rows);
    return GOLHIP_OK;
}

int golhip_halo_plan(int64_t height, int world_size, int rank, int k, golhip_xfer *out) {
    if (height <= 0 || world_size <= 1 || rank < 0 || rank >= world_size || !out) return GOLHIP_ERR_ARG;
    if (k < 1 || k > kMaxK || height / world_size < k) return GOLHIP_ERR_ARG;
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
    // interior/boundary overlap, count all-reduce) runs on a one-GPU box.
    if (ring_self) {
        h->split = true;
        h->halo = k;
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

int golhip_comm_abort(golhip_t h) {
    if (!h) return GOLHIP_ERR_ARG;
    if (!h->comm_failed) return fail(h, GOLHIP_ERR_STATE, "golhip_comm_abort: the communicator has not failed");
    bool all = true;
    for (auto &s : h->shards)
        if (s.comm_nccl) {
            (void)hipSetDevice(s.device);
            all = comm_abort_within(s.comm_nccl, h->comm_timeout_ms) && all;
            s.comm_nccl = nullptr;
        }
    if (!all)
        return fail(h, GOLHIP_ERR_RCCL,
                    "ncclCommAbort did not return within %lld ms (device work that is not RCCL's is stuck); "
                    "end the process", (long long)h->comm_timeout_ms);
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

}  // extern "C"
