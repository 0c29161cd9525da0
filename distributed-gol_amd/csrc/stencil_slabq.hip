// stencil_slabq.hip -- gol_slabq, a PERSISTENT gol_slab2 (counting, end flush) that runs a whole
// count window of K-generation blocks in one launch: golhip_step_persistent, an opt-in call
// (`gol_slabq`).  At configs[1] / configs[4] every slab has its own CU and ~3.3 us of
// every 16-generation launch is its boundary (ramp, row loads, tail); here a slab waits only for the
// 3 x 3 neighbourhood of slabs (the ones whose rows its next block reads, and that read its rows) to
// finish the previous block, instead of for a launch boundary.
//
// Hand-off, two forms (golhip_set_persistent_handoff).  Both: every board store is an `sc1`
// (write-through) buffer store, every storing wave waits vmcnt(0), a workgroup barrier, then lane 0
// stores the slab's block counter (relaxed, agent scope); the consumer's wave 0 polls its
// neighbours' counters (relaxed), a workgroup barrier, and every board load is an `sc1` buffer load.
//   GOLHIP_HANDOFF_FENCED (default): the memory model's own pairing on top -- lane 0 issues an
//     agent-scope RELEASE fence and an asm vmcnt(0) (the compiler may drop its own wait after the
//     write-back: /opt/skills/guides/MI355X_MICROARCH.md "Compiler hazard") before the counter
//     store, and the poller ONE agent-scope ACQUIRE fence + vmcnt(0) before the barrier.
//   GOLHIP_HANDOFF_SC1: without the two fences -- the guide's measured hand-off (its "Valid forms"
//     table, row 1: all stores and loads `sc1`, drained before one lane's flag), round 5's form;
//     measured, not an architectural guarantee, so it is an explicit opt-in.
// The fences cost ~2.7 us per 16-generation block (configs[4]'s board: 0.650 -> 0.818 us/turn, slower
// than the launch path's 0.680: profiles/r06/r06c_persistent_handoff_ab.log).
// Residency: the grid is one workgroup per slab (rounded up to a multiple of the 8 XCDs; the
// surplus workgroups exit at once) and the host refuses the call, before touching the board, unless
// the occupancy query puts the whole grid on the chip at once and the slabs fit the caller's limit
// (golhip_set_persistent_limit).  Still, another process or stream can take CUs: a poll that waits
// longer than kSpinTicks (or sees another slab's failure) sets *err and the workgroup leaves, every
// later window's workgroups leave at entry, and the host restores the board it saved before the
// call -- a failed call leaves the board and turn as they were (GOLHIP_ERR_STATE), never half
// advanced.
#include "golhip_engine.hpp"
#include "stencil_tile.hpp"

namespace golhip {
namespace {

constexpr int kCpSc1 = 16;                  // cache policy: sc1 (buffer load / store aux operand)
constexpr uint64_t kSpinTicks = 20000000;   // 200 ms of s_memrealtime (100 MHz)

template <int K, int W, int S, bool FENCED>
__global__ __launch_bounds__(64 * W) void gol_slabq(uint32_t *buf0, uint32_t *buf1, StencilParams p,
                                                    unsigned long long *slots, uint32_t *flags, int nblocks,
                                                    uint32_t *err, int stall_group) {
    constexpr int T = W * S - 2 * K;
    static_assert(T >= 1 && K >= 2 && K <= 16 && W >= 2 && S >= 3, "slab geometry");
    __shared__ uint32_t ex[2][W + 2][4][64];
    __shared__ uint32_t cnt_lds[K][W][64];
    __shared__ uint32_t quit;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t ngroups = p.nbands * (int64_t)p.nchunks;
    const int64_t per_xcd = (ngroups + kXcds - 1) / kXcds;
    const int64_t group = (int64_t)(blockIdx.x % kXcds) * per_xcd + blockIdx.x / kXcds;
    if (group >= ngroups) return;  // whole workgroup; never waited for
    // an earlier window of this call failed: touch nothing (the host restores the board)
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    const int nb = (int)p.nbands, nc = (int)p.nchunks;
    const int bi = (int)group / nc, ci = (int)group - bi * nc;
    int ya, yb;
    band_rows(p, bi, ya, yb);
    const int nrows = yb - ya;
    const int colraw = ci * kTileChunkWords + lane - 1;
    const int col = (colraw + p.wd) % p.wd;
    const int rowbytes = (int)(p.pitch * 4);
    const LaneStore ls = lane_store<false>(lane, colraw, col, p.wd);
    const bool count_lane = lane >= 2 && colraw <= p.wd;
    const int o0 = w * S - K;  // output row of c[1]
    // the slabs whose rows this one's blocks read (and that read its rows): bands within K rows
    // (one more beyond a short last band), x the adjacent chunks; lanes 0..14 poll one each
    auto wrap = [](int v, int n) {
        v = v < 0 ? v + n : v;
        v = v < 0 ? v + n : v;
        v = v >= n ? v - n : v;
        return v >= n ? v - n : v;
    };
    const bool short_last = (int)(p.r0e - (int64_t)(nb - 1) * p.band) < K;
    const int bm1 = wrap(bi - 1, nb), bp1 = wrap(bi + 1, nb);
    const int pl = lane < 15 ? lane : 0;
    const int pi = pl / 3, pj = pl % 3;
    const int pband = pi == 0 ? (short_last && bm1 == nb - 1 ? wrap(bi - 2, nb) : bi)
                    : pi == 1 ? bm1 : pi == 2 ? bi : pi == 3 ? bp1
                                              : (short_last && bp1 == nb - 1 ? wrap(bi + 2, nb) : bi);
    uint32_t *const pflag = flags + (pband * nc + wrap(ci + pj - 1, nc));
    if (w == 0)
        for (int par = 0; par < 2; ++par)
            for (int i = 0; i < 4; ++i) ex[par][0][i][lane] = ex[par][W + 1][i][lane] = 0u;
    uint32_t *const ex_base0 = &ex[0][w][0][lane];
    constexpr int kExPar = (W + 2) * 4 * 64;
    uint32_t *const cnt_my = &cnt_lds[0][w][lane];
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    const bool full = o0 >= 0 && o0 + S <= nrows;
    const bool halo = o0 + S <= 0 || o0 >= nrows;
    const int base_row = 0, span_rows = (int)p.wrap_rows;

#pragma clang loop unroll(disable)
    for (int blk = 0; blk < nblocks; ++blk) {
        const uint32_t *in = (blk & 1) ? buf1 : buf0;
        uint32_t *out = (blk & 1) ? buf0 : buf1;
        if (blk > 0) {  // the neighbourhood has finished block blk - 1 (its stores drained)
            if (w == 0) {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                uint32_t stop = 0;
                for (;;) {
                    // lanes 0..14: the neighbourhood's block counters; lane 15: the error word
                    const uint32_t f = lane < 15 ? __hip_atomic_load(pflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : lane == 15 ? __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                  : (uint32_t)blk;
                    if (__builtin_amdgcn_ballot_w64(lane == 15 && f != 0u) != 0) {
                        stop = 1;  // another slab failed: nothing this one computes is kept
                        break;
                    }
                    if (__builtin_amdgcn_ballot_w64(lane < 15 && f < (uint32_t)blk) == 0) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
                        stop = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if constexpr (FENCED) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (lane == 0) {
                    quit = stop;
                    if (stop) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            __syncthreads();
            if (quit) return;
        }
        uint32_t c[S + 2];
        c[0] = c[S + 1] = 0;
        {
            const __amdgpu_buffer_rsrc_t irsrc = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint32_t *>(in + (int64_t)base_row * p.pitch), 0, span_rows * rowbytes, kBufferRsrcWord3);
            RowStream rows(p, ya - K + w * S);
#pragma unroll
            for (int r = 0; r < S; ++r) {
                c[1 + r] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(irsrc, col * 4,
                                                                          (rows.ly - base_row) * rowbytes, kCpSc1);
                rows.advance();
            }
        }
        const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
            out + (int64_t)ya * p.pitch, 0, nrows * rowbytes, kBufferRsrcWord3);
        for (int j = 0; j < K; ++j) cnt_lds[j][w][lane] = 0;
        unsigned long long *const bslots = slots + (int64_t)blk * K * kCountSlots;
        auto cnt_sum = [&](int j) {
            uint32_t a = 0;
#pragma unroll
            for (int ww = 0; ww < W; ++ww) a += cnt_lds[j][ww][lane];
            return count_lane ? a : 0u;
        };
        auto gen = [&](auto last_c, auto full_c, auto cnt_c, int g) {
            constexpr bool LAST = decltype(last_c)::value, FULL = decltype(full_c)::value;
            constexpr bool CNT = decltype(cnt_c)::value;
            const int gi = g - 1;
            uint32_t cnt = 0;
            auto emit = [&](int r, uint32_t nx) {
                const int o = o0 + r - 1;
                const bool mine = FULL || (o >= 0 && o < nrows);
                if (CNT) cnt = bcnt_acc(mine ? nx : 0u, cnt);
                if constexpr (LAST) {  // sc1 stores: the neighbours read them in the next block
                    const uint32_t v = realign_drift<K>(nx);
                    __builtin_amdgcn_raw_buffer_store_b32((int)v, orsrc, ls.off_full + (mine ? o * rowbytes : kOutOfRange),
                                                          0, kCpSc1);
                }
            };
            uint32_t x[S], s[S], cy[S], ctr[S];
#pragma unroll
            for (int i = 0; i < S; ++i) x[i] = c[i + 1];
            sums_om<S>(x, s, cy, ctr);
            uint32_t *const b = ex_base0 + (g & 1) * kExPar;
            b[256] = s[0];
            b[320] = cy[0];
            b[384] = s[S - 1];
            b[448] = cy[S - 1];
            {
                constexpr int NI = S - 2;
                uint32_t as[NI], acy[NI], ms[NI], mcy[NI], mc[NI], bs[NI], bcy[NI], nx[NI];
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    as[i] = s[i], acy[i] = cy[i];
                    ms[i] = s[i + 1], mcy[i] = cy[i + 1], mc[i] = ctr[i + 1];
                    bs[i] = s[i + 2], bcy[i] = cy[i + 2];
                }
                life_om<NI>(as, acy, ms, mcy, mc, bs, bcy, nx, AllRows{});
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    emit(i + 2, nx[i]);
                    if constexpr (!LAST) c[i + 2] = nx[i];
                }
            }
            lds_barrier();
            const uint32_t ts = b[128], tcy = b[192];
            const uint32_t bts = b[512], btcy = b[576];
            {
                uint32_t as[2] = {ts, s[S - 2]}, acy[2] = {tcy, cy[S - 2]};
                uint32_t ms[2] = {s[0], s[S - 1]}, mcy[2] = {cy[0], cy[S - 1]}, mc[2] = {ctr[0], ctr[S - 1]};
                uint32_t bs[2] = {s[1], bts}, bcy[2] = {cy[1], btcy}, nx[2];
                life_om<2>(as, acy, ms, mcy, mc, bs, bcy, nx, AllRows{});
                emit(1, nx[0]);
                emit(S, nx[1]);
                if constexpr (!LAST) {
                    c[1] = nx[0];
                    c[S] = nx[1];
                }
            }
            if constexpr (CNT) cnt_my[gi * (W * 64)] = cnt;
        };
        auto idle = [&](int g) {
            uint32_t x2[2] = {c[1], c[S]}, s2[2], cy2[2], c2[2];
            sums_om<2>(x2, s2, cy2, c2);
            uint32_t *const b = ex_base0 + (g & 1) * kExPar;
            b[256] = s2[0];
            b[320] = cy2[0];
            b[384] = s2[1];
            b[448] = cy2[1];
            lds_barrier();
        };
        using No = std::false_type;
        using Yes = std::true_type;
        if (halo) {
            const int g_end = std::min(std::min(w * S + S, W * S - w * S), K);
            int g = 1;
#pragma clang loop unroll(disable)
            for (; g < g_end; ++g) gen(No{}, No{}, No{}, g);
#pragma clang loop unroll(disable)
            for (; g <= K; ++g) idle(g);
        } else if (full) {
#pragma clang loop unroll(disable)
            for (int g = 1; g < K; ++g) gen(No{}, Yes{}, Yes{}, g);
            gen(Yes{}, Yes{}, Yes{}, K);
        } else {
#pragma clang loop unroll(disable)
            for (int g = 1; g < K; ++g) gen(No{}, No{}, Yes{}, g);
            gen(Yes{}, No{}, Yes{}, K);
        }
        // publish: this workgroup's board stores have drained, a release, then its block counter;
        // the count atomics go after it, off the neighbours' critical path (only the finalize
        // after the launch reads them)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // also: every generation's per-wave counts are in LDS
        if (w == 0 && lane == 0 && !(group == stall_group && blk == 0)) {  // stall_group: fault injection
            if constexpr (FENCED) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __hip_atomic_store(flags + group, (uint32_t)(blk + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        for (int j = w; j < K; j += W) {
            uint32_t acc[1] = {cnt_sum(j)};
            flush_counts<1>(acc, j, lane, group, bslots);
        }
    }
}

template <int W, int S>
const void *slabq_fn(bool fenced) {
    return fenced ? reinterpret_cast<const void *>(&gol_slabq<16, W, S, true>)
                  : reinterpret_cast<const void *>(&gol_slabq<16, W, S, false>);
}

// Workgroups of slab shape `shape` (W * 100 + S) the device holds at once (occupancy x CUs).
int slabq_resident(golhip_t h, int shape, bool fenced, int64_t *out) {
    const void *fn = shape == 1207 ? slabq_fn<12, 7>(fenced) : shape == 1606 ? slabq_fn<16, 6>(fenced)
                   : shape == 1208 ? slabq_fn<12, 8>(fenced) : slabq_fn<16, 4>(fenced);
    int per_cu = 0;
    HIPCHK(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * (shape / 100), 0));
    *out = (int64_t)per_cu * h->cus;
    return GOLHIP_OK;
}

template <int W, int S>
hipError_t launch_slabq(bool fenced, uint32_t *b0, uint32_t *b1, const StencilParams &q, unsigned long long *slots,
                        uint32_t *flags, int nblocks, uint32_t *err, int stall_group, hipStream_t s) {
    const int64_t ngroups = q.nbands * (int64_t)q.nchunks;
    const unsigned blocks = (unsigned)((ngroups + kXcds - 1) / kXcds * kXcds);
    if (fenced)
        hipLaunchKernelGGL((gol_slabq<16, W, S, true>), dim3(blocks), dim3(64 * W), 0, s, b0, b1, q, slots, flags,
                           nblocks, err, stall_group);
    else
        hipLaunchKernelGGL((gol_slabq<16, W, S, false>), dim3(blocks), dim3(64 * W), 0, s, b0, b1, q, slots, flags,
                           nblocks, err, stall_group);
    return hipGetLastError();
}

}  // namespace
}  // namespace golhip

using namespace golhip;

extern "C" {

// golhip_step_persistent (include/golhip.h): golhip_step with per-turn counts through gol_slabq on
// single-strip boards whose counting launch is a production gol_slab2 shape with one slab per CU.
// Refuses (GOLHIP_ERR_STATE, nothing enqueued) unless every slab can be resident at once; saves the
// board first and restores it when a window fails, so a failed call leaves board and turn unchanged.
int golhip_step_persistent(golhip_t h, int64_t turns, uint64_t *alive_per_turn) {
    if (!h || !alive_per_turn || turns < 0) return GOLHIP_ERR_ARG;
    if (turns == 0) return GOLHIP_OK;
    constexpr int K = 16;
    if (h->split || h->shards.size() != 1 || h->k < K || h->variant != kVariantProd)
        return fail(h, GOLHIP_ERR_STATE, "golhip_step_persistent: a single-strip board of the production kernels, k >= 16");
    if (h->track_flips)  // gol_slabq writes no flips board
        return fail(h, GOLHIP_ERR_STATE, "golhip_step_persistent: flip tracking is on (use golhip_step)");
    Shard &s = h->shards[0];
    const RegKernel rk = pick_reg_kernel(h, s.rows, K, true);
    const int shape = rk.kind == 3 && rk.NC == kSlab2E ? rk.W * 100 + rk.S : 0;
    if (shape != 1207 && shape != 1606 && shape != 1208 && shape != 1604)
        return fail(h, GOLHIP_ERR_STATE,
                    "golhip_step_persistent: the board's counting launch is not a gol_slab2 12x7 / 16x6 / 12x8 / 16x4 slab");
    StencilParams q = make_params(h, s, K, 0, s.rows, 0, 0, 0, true);
    const int T = rk.W * rk.S - 2 * K;
    q.band = T;
    q.band2 = q.nbig0 = 0;
    q.nbands0 = q.nbands = (s.rows + T - 1) / T;
    q.nchunks = (int32_t)((h->wd + kTileChunkWords - 1) / kTileChunkWords);
    const int64_t ngroups = q.nbands * (int64_t)q.nchunks;
    const int64_t grid = (ngroups + kXcds - 1) / kXcds * kXcds;
    if (ngroups > h->cus || q.wrap_rows <= 0 || q.nbands < 3)
        return fail(h, GOLHIP_ERR_STATE, "golhip_step_persistent: %lld slabs (more than the %d CUs, or under 3 bands)",
                    (long long)ngroups, h->cus);
    HIPCHK(h, hipSetDevice(s.device));
    // co-residency, before anything is enqueued: the whole grid on the chip at once (occupancy
    // query), and the slabs within the CUs the caller says it owns (golhip_set_persistent_limit)
    int64_t resident = 0;
    const bool fenced = h->persistent_handoff == GOLHIP_HANDOFF_FENCED;
    if (int rc = slabq_resident(h, shape, fenced, &resident)) return rc;
    if (grid > resident || (h->persistent_limit > 0 && ngroups > h->persistent_limit))
        return fail(h, GOLHIP_ERR_STATE,
                    "golhip_step_persistent: %lld slabs (grid %lld) cannot all be resident: the device holds %lld "
                    "such workgroups at once, the handle's limit is %d (golhip_set_persistent_limit); board unchanged",
                    (long long)ngroups, (long long)grid, (long long)resident, h->persistent_limit);
    if (s.pflags_cap < ngroups + 1) {
        SYNCCHK(h, s.compute);
        if (s.pflags) HIPCHK(h, hipFree(s.pflags));
        s.pflags = nullptr;
        s.pflags_cap = 0;
        HIPCHK(h, hipMalloc(&s.pflags, sizeof(uint32_t) * (ngroups + 1)));
        s.pflags_cap = ngroups + 1;
    }
    const size_t board_bytes = sizeof(uint32_t) * (size_t)s.rows * (size_t)h->pitch;
    if (!s.psave) HIPCHK(h, hipMalloc(&s.psave, board_bytes));  // the board's size is fixed per handle
    if (s.dev_counts_cap < (size_t)turns) {
        SYNCCHK(h, s.compute);
        if (s.dev_counts) HIPCHK(h, hipFree(s.dev_counts));
        s.dev_counts = nullptr;
        s.dev_counts_cap = 0;
        HIPCHK(h, hipMalloc(&s.dev_counts, sizeof(unsigned long long) * (size_t)std::max<int64_t>(turns, 128)));
        s.dev_counts_cap = (size_t)std::max<int64_t>(turns, 128);
    }
    uint32_t *const err = s.pflags + ngroups;
    const int cur0 = h->cur;
    const int64_t turn0 = h->turn;
    HIPCHK(h, hipMemcpyAsync(s.psave, h->row0(s, cur0), board_bytes, hipMemcpyDeviceToDevice, s.compute));
    HIPCHK(h, hipMemsetAsync(err, 0, sizeof(uint32_t), s.compute));
    const int stall_group = h->fault == Fault::slab_stall ? 0 : -1;  // tuning library's fault injection
    // the 16-generation blocks, one launch per count window; a tail under 16 turns: golhip_step
    const int64_t body = turns / K * K;
    for (int64_t done = 0; done < body;) {
        const int64_t n = std::min<int64_t>(body - done, h->count_window / K * K);
        HIPCHK(h, hipMemsetAsync(s.pflags, 0, sizeof(uint32_t) * ngroups, s.compute));
        uint32_t *b0 = h->row0(s, h->cur), *b1 = h->row0(s, h->cur ^ 1);
        const int nblocks = (int)(n / K);
        hipError_t e = hipErrorInvalidValue;
        if (shape == 1207) e = launch_slabq<12, 7>(fenced, b0, b1, q, s.slots, s.pflags, nblocks, err, stall_group, s.compute);
        if (shape == 1606) e = launch_slabq<16, 6>(fenced, b0, b1, q, s.slots, s.pflags, nblocks, err, stall_group, s.compute);
        if (shape == 1208) e = launch_slabq<12, 8>(fenced, b0, b1, q, s.slots, s.pflags, nblocks, err, stall_group, s.compute);
        if (shape == 1604) e = launch_slabq<16, 4>(fenced, b0, b1, q, s.slots, s.pflags, nblocks, err, stall_group, s.compute);
        if (e != hipSuccess) {  // undo the windows that did run
            SYNCCHK(h, s.compute);
            HIPCHK(h, hipMemcpy(h->row0(s, cur0), s.psave, board_bytes, hipMemcpyDeviceToDevice));
            h->cur = cur0;
            h->turn = turn0;
            return fail(h, GOLHIP_ERR_HIP, "gol_slabq: %s (board restored to turn %lld)", hipGetErrorString(e),
                        (long long)turn0);
        }
        HIPCHK(h, launch_count_finalize((int)n, s.slots, s.dev_counts + done, s.compute));
        h->cur ^= (nblocks & 1);
        h->turn += n;
        done += n;
    }
    h->prev_valid = h->diff_valid = h->act_valid = false;
    uint32_t errv = 0;
    HIPCHK(h, hipMemcpyAsync(alive_per_turn, s.dev_counts, sizeof(uint64_t) * (size_t)body, hipMemcpyDeviceToHost,
                             s.compute));
    HIPCHK(h, hipMemcpyAsync(&errv, err, sizeof errv, hipMemcpyDeviceToHost, s.compute));
    SYNCCHK(h, s.compute);
    if (errv) {  // a slab gave up waiting: put the saved board back, as of before the call
        HIPCHK(h, hipMemcpyAsync(h->row0(s, cur0), s.psave, board_bytes, hipMemcpyDeviceToDevice, s.compute));
        SYNCCHK(h, s.compute);
        h->cur = cur0;
        h->turn = turn0;
        return fail(h, GOLHIP_ERR_STATE,
                    "golhip_step_persistent: a slab waited over 200 ms for its neighbours (the GPU is shared?); the "
                    "board and turn are restored to turn %lld (use golhip_step)", (long long)turn0);
    }
    const int64_t rep = h->rep();
    if (rep > 1)
        for (int64_t i = 0; i < body; ++i) alive_per_turn[i] /= (uint64_t)rep;
    if (body < turns) return run_steps(h, turns - body, alive_per_turn + body, false);
    return GOLHIP_OK;
}

// golhip_set_persistent_handoff (include/golhip.h)
int golhip_set_persistent_handoff(golhip_t h, int mode) {
    if (!h || (mode != GOLHIP_HANDOFF_FENCED && mode != GOLHIP_HANDOFF_SC1)) return GOLHIP_ERR_ARG;
    h->persistent_handoff = mode;
    return GOLHIP_OK;
}

// golhip_set_persistent_limit (include/golhip.h)
int golhip_set_persistent_limit(golhip_t h, int max_groups) {
    if (!h || max_groups < 0) return GOLHIP_ERR_ARG;
    h->persistent_limit = max_groups;
    return GOLHIP_OK;
}

}  // extern "C"
