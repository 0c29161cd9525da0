// stencil_tile.hpp -- the register kernels for small boards (gol_tile, gol_slab, gol_slab2, gol_slabp,
// gol_slab3) and their launch templates, shared by the production TU stencil_tile.hip and the tuning
// library's tuning/stencil_tile_tuning.hip.
//
// Why a second kernel: gol_stencil streams a band of rows through a chain of K generation levels.
// Each wave is one long dependency chain (row after row, level after level) whose pipeline fill
// costs 2K rows, so it needs tall bands and many waves.  A small board cannot give it both.  At
// 5120^2 a K = 16 launch ran 23.7 us, about 12x the VALU time of its useful work
// (profiles/r02/small_board_timeline_split_k16.txt): short bands, about one wave per SIMD, and every step
// waiting on the previous level.
//
// gol_tile turns the loop around.  A wave loads a whole tile into VGPRs: R = T + 2K rows of its
// 64-lane column chunk, the same 62-word chunk geometry as gol_stencil (lanes 0 and 63 are halo).
// It then runs the K generations over the tile in place.  Generation g recomputes rows
// [g, R - g): the K-row trapezoid of temporal blocking, with the halo rows going stale from the
// tile edges inward.  All rows of a generation are independent, so a wave carries R-way ILP
// instead of one chain.  Finally it stores the T middle rows.  There are no LDS, barriers or
// pipeline fill.  The cost is the trapezoid: K(R - K - 1) row updates for T useful rows per
// generation.
//
// The row update is gol_stencil's drifting-sum form (row_sum3_drift + life_next): 12 VALU per
// word per generation (1 DPP, 2 v_alignbit, 9 v_bitop3).  Generation g sits g bits east of the
// board frame; the stored rows move back with realign_drift<K>.  Counts use the same whole-word
// window as the 62-word drift geometry.  Rows load through a raw-buffer descriptor with the row
// offset in an SGPR: one VGPR offset per lane for every row.
#pragma once
#include "golhip_stencil.hpp"

namespace golhip {
namespace {

// Independent row chains per wave (segments advanced op-major).
constexpr int kTileChains = 4;
constexpr int kXcds = 8;  // MI355X: 8 XCDs, workgroups dealt round-robin

// Drifting 3-cell sums (row_sum3_drift) of N rows, op-major: each op for every row before the
// next op, so the N dependency chains interleave.  Rows with use(i) false are skipped.
struct AllRows {
    constexpr bool operator()(int) const { return true; }
};
template <int N, class U = AllRows>
__device__ __forceinline__ void sums_om(const uint32_t (&x)[N], uint32_t (&s)[N], uint32_t (&cy)[N],
                                        uint32_t (&ctr)[N], U use = U{}) {
    uint32_t wl[N], w2[N];
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) wl[i] = lane_from_west(x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) ctr[i] = __builtin_amdgcn_alignbit(x[i], wl[i], 31);  // cell x-1 onto x
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) w2[i] = __builtin_amdgcn_alignbit(x[i], wl[i], 30);  // cell x-2 onto x
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) s[i] = GOL_BOP3(w2[i], ctr[i], x[i], kXor3);
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) cy[i] = GOL_BOP3(w2[i], ctr[i], x[i], kMaj);
}

// life_next of N rows, op-major (same circuit: 7 v_bitop3 per row).
template <int N, class U>
__device__ __forceinline__ void life_om(const uint32_t (&as)[N], const uint32_t (&acy)[N],
                                        const uint32_t (&ms)[N], const uint32_t (&mcy)[N],
                                        const uint32_t (&mc)[N], const uint32_t (&bs)[N],
                                        const uint32_t (&bcy)[N], uint32_t (&out)[N], U use) {
    uint32_t o[N], k[N], pp[N], q[N], u[N], v[N];
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) o[i] = GOL_BOP3(as[i], ms[i], bs[i], kXor3);
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) k[i] = GOL_BOP3(as[i], ms[i], bs[i], kMaj);
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) pp[i] = GOL_BOP3(acy[i], mcy[i], bcy[i], kXor3);
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) q[i] = GOL_BOP3(acy[i], mcy[i], bcy[i], kMaj);
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) u[i] = GOL_BOP3(k[i], pp[i], q[i], kTwosEven);
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) v[i] = GOL_BOP3(o[i], q[i], mc[i], kOddSelect);
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (use(i)) out[i] = GOL_BOP3(v[i], o[i], u[i], GOL_TT(a & (b ^ c)));
}

// Segment geometry of one generation step i: NS segments over rows [LO, LO + N), segment sg =
// [first(sg), first(sg + 1)); active: it has a row at step I; fresh: that row's successor needs
// new sums (not the segment's last row before a next segment, whose first m is saved).
// Segment geometry of one generation step I: NS segments over rows [LO, LO + N), segment sg =
// [first(sg), first(sg + 1)), walked top-down -- except segment 0 when REV0, walked bottom-up, so
// that the row above the range (an LDS hand-off in gol_slab) is needed only at its LAST step.
// fresh_row: the row whose sums step I takes fresh, -1 when it takes the saved sums of the next
// segment's first row (a top-down segment's last row: that row may be overwritten already).
template <int LO, int N, int NS, bool REV0, int I>
struct TileStep {
    static constexpr int first(int sg) { return LO + (N * sg) / NS; }
    static constexpr bool rev(int sg) { return REV0 && sg == 0; }
    static constexpr bool active(int sg) { return first(sg) + I < first(sg + 1); }
    static constexpr int row(int sg) { return rev(sg) ? first(sg + 1) - 1 - I : first(sg) + I; }
    static constexpr int fresh_row(int sg) {
        return !active(sg)                                          ? -1
               : rev(sg)                                            ? row(sg) - 1
               : (row(sg) + 1 == first(sg + 1) && sg + 1 < NS) ? -1
                                                                    : row(sg) + 1;
    }
    struct Active {
        constexpr bool operator()(int sg) const { return active(sg); }
    };
    struct Fresh {
        constexpr bool operator()(int sg) const { return fresh_row(sg) >= 0; }
    };
};

// Row sums handed to gen_rows instead of computed from c[] (gol_slab's exchange): NoPre computes
// every row; SlabPre<S> supplies rows 0 and S + 1 (the neighbour waves' edge rows: sums and carries
// only, they are never a centre row) and rows 1 and S (this wave's own edge rows, computed once
// before the exchange that publishes them: sums, carries and centre cells).
struct NoPre {
    static constexpr bool has(int) { return false; }
    template <int R>
    __device__ __forceinline__ void get(std::integral_constant<int, R>, uint32_t &, uint32_t &,
                                        uint32_t &) const {}
};
template <int S>
struct SlabPre {
    uint32_t ts, tcy;            // row 0 (above): the upper neighbour wave's last row
    uint32_t fs, fcy, fctr;      // row 1: this wave's first row
    uint32_t ls, lcy, lctr;      // row S: this wave's last row
    uint32_t bs, bcy;            // row S + 1 (below): the lower neighbour wave's first row
    static constexpr bool has(int r) { return r == 0 || r == 1 || r == S || r == S + 1; }
    template <int R>
    __device__ __forceinline__ void get(std::integral_constant<int, R>, uint32_t &s, uint32_t &cy,
                                        uint32_t &ctr) const {
        if constexpr (R == 0) s = ts, cy = tcy, ctr = 0u;
        else if constexpr (R == 1) s = fs, cy = fcy, ctr = fctr;
        else if constexpr (R == S) s = ls, cy = lcy, ctr = lctr;
        else if constexpr (R == S + 1) s = bs, cy = bcy, ctr = 0u;
    }
};

// One generation over rows [LO, LO + N) of c (compile time) from the previous generation's rows
// [LO - 1, LO + N].  The rows are cut into NS segments that advance together, op-major (one op
// of every segment, then the next op): NS independent dependency chains per wave.  A segment
// walks its rows holding the sums of the rows on both sides of the current row: (o) the one
// already passed and (m) the row itself; each step takes the sums of the next row, writes the
// row's new cells (WRITE) and rotates o <- m <- new.  The rule is symmetric in the rows above
// and below, so top-down and bottom-up segments run the same code.  Every sum comes from the
// previous generation: the first o/m of every segment are taken before any row is written, and a
// top-down segment's last row takes the next segment's first m (saved then).
// emit(integral_constant<r>, next, centre) sees every new row and the centre cells it replaces
// (same drifted frame: the last generation's flips are next ^ centre).
template <int LO, int N, bool WRITE, int NC = kTileChains, bool REV0 = false, int R, class F,
          class P = NoPre>
__device__ __forceinline__ void gen_rows(uint32_t (&c)[R], F &&emit, const P &pre = P{}) {
    constexpr int NS = N < NC ? N : NC;
    using TS0 = TileStep<LO, N, NS, REV0, 0>;
    static_assert(!REV0 || !P::has(LO - 1), "precomputed sums: top-down segments only");
    constexpr int L = (N + NS - 1) / NS;
    uint32_t os[NS], ocy[NS], ms[NS], mcy[NS], mc[NS], ss[NS], scy[NS];
    {
        // the initial (o, m) rows of every segment; rows the provider holds are not recomputed
        auto init_row = [](int i) constexpr {
            const int sg = i / 2;
            return (i & 1) ? (TS0::rev(sg) ? TS0::first(sg + 1) - 1 : TS0::first(sg))
                           : (TS0::rev(sg) ? TS0::first(sg + 1) : TS0::first(sg) - 1);
        };
        struct Need {
            constexpr bool operator()(int i) const {
                const int sg = i / 2;
                const int r = (i & 1) ? (TS0::rev(sg) ? TS0::first(sg + 1) - 1 : TS0::first(sg))
                                      : (TS0::rev(sg) ? TS0::first(sg + 1) : TS0::first(sg) - 1);
                return !P::has(r);
            }
        };
        uint32_t x[2 * NS], s2[2 * NS], cy2[2 * NS], c2[2 * NS];
#pragma unroll
        for (int i = 0; i < 2 * NS; ++i) x[i] = c[init_row(i)];
        sums_om<2 * NS>(x, s2, cy2, c2, Need{});
        static_for(std::make_integer_sequence<int, 2 * NS>{}, [&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int r = init_row(i);
            if constexpr (P::has(r)) pre.get(std::integral_constant<int, r>{}, s2[i], cy2[i], c2[i]);
        });
#pragma unroll
        for (int sg = 0; sg < NS; ++sg) {
            os[sg] = s2[2 * sg], ocy[sg] = cy2[2 * sg];
            ms[sg] = ss[sg] = s2[2 * sg + 1], mcy[sg] = scy[sg] = cy2[2 * sg + 1];
            mc[sg] = c2[2 * sg + 1];
        }
    }
    static_for(std::make_integer_sequence<int, L>{}, [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        using TS = TileStep<LO, N, NS, REV0, i>;
        constexpr typename TS::Active active{};
        constexpr typename TS::Fresh fresh{};
        struct Compute {  // fresh rows whose sums are not precomputed
            constexpr bool operator()(int sg) const {
                return TS::fresh_row(sg) >= 0 && !P::has(TS::fresh_row(sg));
            }
        };
        uint32_t x[NS], bs[NS], bcy[NS], bc[NS], nx[NS];
#pragma unroll
        for (int sg = 0; sg < NS; ++sg) x[sg] = fresh(sg) ? c[TS::fresh_row(sg)] : 0u;
        sums_om<NS>(x, bs, bcy, bc, Compute{});
        static_for(std::make_integer_sequence<int, NS>{}, [&](auto sgc) {
            constexpr int sg = decltype(sgc)::value;
            constexpr int fr = TS::fresh_row(sg);
            if constexpr (fr >= 0 && P::has(fr))
                pre.get(std::integral_constant<int, fr>{}, bs[sg], bcy[sg], bc[sg]);
        });
#pragma unroll
        for (int sg = 0; sg < NS; ++sg)
            if (active(sg) && !fresh(sg)) bs[sg] = ss[sg + 1], bcy[sg] = scy[sg + 1], bc[sg] = 0u;
        life_om<NS>(os, ocy, ms, mcy, mc, bs, bcy, nx, active);
        static_for(std::make_integer_sequence<int, NS>{}, [&](auto sgc) {
            constexpr int sg = decltype(sgc)::value;
            if constexpr (TS::active(sg)) {
                constexpr int r = TS::row(sg);
                emit(std::integral_constant<int, r>{}, nx[sg], mc[sg]);
                if constexpr (WRITE) c[r] = nx[sg];
                os[sg] = ms[sg], ocy[sg] = mcy[sg];
                ms[sg] = bs[sg], mcy[sg] = bcy[sg], mc[sg] = bc[sg];
            }
        });
    });
}

// Input rows through one raw-buffer descriptor over the rows the stream can address (the torus
// [0, wrap) or the halo'd strip [lo, hi)); the row offset goes in soffset (SGPR), the column in
// voffset.  Loads c[first .. first + n) from stream row `row0` on.
template <int FIRST, int NROWS, int R>
__device__ __forceinline__ void load_rows(uint32_t (&c)[R], const uint32_t *in, const StencilParams &p,
                                          int row0, int col) {
    const int rowbytes = (int)(p.pitch * 4);
    const int base_row = p.wrap_rows > 0 ? 0 : (int)p.lo;
    const int span_rows = p.wrap_rows > 0 ? (int)p.wrap_rows : (int)(p.hi - p.lo);
    const __amdgpu_buffer_rsrc_t irsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t *>(in + (int64_t)base_row * p.pitch), 0, span_rows * rowbytes,
        kBufferRsrcWord3);
    RowStream rows(p, row0);
    const int voff = col * 4;
#pragma unroll
    for (int r = 0; r < NROWS; ++r) {
        c[FIRST + r] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(irsrc, voff,
                                                                      (rows.ly - base_row) * rowbytes, 0);
        rows.advance();
    }
}

template <int K, int T, bool COUNT, bool LD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 4))) void gol_tile(
    const uint32_t *__restrict__ in, uint32_t *__restrict__ out, StencilParams p,
    unsigned long long *__restrict__ slots) {
    constexpr int R = T + 2 * K;  // tile rows: T output rows with K halo rows above and below
    static_assert(T >= 1 && K >= 2 && K <= 32, "tile geometry");
    const int lane = threadIdx.x & 63;
    const int64_t wave =
        (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t chunk = wave % p.nchunks;
    const int64_t bandi = wave / p.nchunks;
    if (bandi >= p.nbands) return;  // wave-uniform
    int ya, yb;
    band_rows(p, bandi, ya, yb);  // yb - ya <= T (the host sets p.band = T)
    const int nrows = yb - ya;
    const int colraw = (int)chunk * kTileChunkWords + lane - 1;
    const int col = (colraw + p.wd) % p.wd;
    const int rowbytes = (int)(p.pitch * 4);
    // per-generation counts parked per lane in LDS (runtime generation index), reduced at the end
    __shared__ uint32_t cnt_lds[4][COUNT ? K : 1][64];
    const int wl = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    uint32_t c[R];
    load_rows<0, R>(c, in, p, ya - K, col);
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)ya * p.pitch, 0, nrows * rowbytes, kBufferRsrcWord3);
    __amdgpu_buffer_rsrc_t drsrc = orsrc;
    if constexpr (LD)
        drsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + (int64_t)ya * p.pitch, 0,
                                                  nrows * rowbytes, kBufferRsrcWord3);
    const LaneStore ls = lane_store<false>(lane, colraw, col, p.wd);
    // the 62-word drift count window: lanes 2..63 with colraw <= wd (gol_stencil, count_lane)
    const bool count_lane = lane >= 2 && colraw <= p.wd;

    // generation `gen` (0-based) over rows [LO, LO + N); LAST: the output rows, stored
    auto pass = [&](auto lo_c, auto n_c, auto last_c, int gen) {
        constexpr int LO = decltype(lo_c)::value, N = decltype(n_c)::value;
        constexpr bool LAST = decltype(last_c)::value;
        uint32_t cnt = 0;
        gen_rows<LO, N, !LAST>(c, [&](auto rc, uint32_t nx, uint32_t centre) {
            constexpr int r = decltype(rc)::value;
            constexpr bool out_row = r >= K && r < K + T;
            // rows past the band's end (a short last band) are not the band's
            const bool mine = out_row && r - K < nrows;
            if (COUNT && out_row) cnt += __builtin_popcount(mine ? nx : 0u);
            if constexpr (LAST && out_row) {
                const int rowoff = mine ? (r - K) * rowbytes : kOutOfRange;
                Words<1> v;
                v.w[0] = realign_drift<K>(nx);
                golhip::store_row<1, false>(orsrc, ls, v, rowoff);
                if constexpr (LD) {  // the last generation's flips, same (drifted) frame
                    Words<1> dv;
                    dv.w[0] = realign_drift<K>(nx ^ centre);
                    golhip::store_row<1, false>(drsrc, ls, dv, rowoff);
                }
            }
        });
        if constexpr (COUNT) cnt_lds[wl][gen][lane] = count_lane ? cnt : 0u;
    };
    // Generation g (1..K) must produce rows [g, R - g).  The generations run as a loop (one
    // generation's code is reused from the instruction cache), in two phases of fixed row ranges:
    // generations 1..H over [1, R - 1), H+1..K-1 over [H+1, R-H-1) (garbage rows outside
    // [g, R - g) are harmless: they were garbage already), then the last generation over the T
    // output rows, with the stores.
    constexpr int H = K / 2;
    using One = std::integral_constant<int, 1>;
    using No = std::false_type;
#pragma clang loop unroll(disable)
    for (int g = 1; g <= H; ++g) pass(One{}, std::integral_constant<int, R - 2>{}, No{}, g - 1);
    if constexpr (K - 1 > H) {
#pragma clang loop unroll(disable)
        for (int g = H + 1; g <= K - 1; ++g)
            pass(std::integral_constant<int, H + 1>{}, std::integral_constant<int, R - 2 * (H + 1)>{}, No{},
                 g - 1);
    }
    pass(std::integral_constant<int, K>{}, std::integral_constant<int, T>{}, std::true_type{}, K - 1);
    if constexpr (COUNT) {
        uint32_t acc[K];
#pragma unroll
        for (int j = 0; j < K; ++j) acc[j] = cnt_lds[wl][j][lane];
        flush_counts<K>(acc, 0, lane, wave, slots);
    }
}

// A drifted row of generation g (0-based; g + 1 bits east of the board frame) moved back, for
// runtime g: the lane's word takes its upper 31 - g bits and the east lane's low g + 1 bits.
__device__ __forceinline__ uint32_t realign_drift_rt(uint32_t v, int g) {
    return __builtin_amdgcn_alignbit(lane_from_east(v), v, (uint32_t)(g + 1));
}

// popcount(x) + acc as ONE v_bcnt_u32_b32 (the compiler splits a row sum of popcounts into
// v_bcnt(x, 0) + v_add3 trees: 3 extra VALU per 8 rows)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

// gol_slab: the register tile spread over the W waves of a workgroup.  Wave w holds S rows of the
// slab's W*S (a 62-word column chunk, rows ya - K + wS ...) in c[1..S]; each generation the waves
// swap their edge rows through LDS (c[0] = the row above, c[S+1] = the row below, double-buffered
// by generation parity: one barrier per generation) and update their S rows.  The trapezoid is
// paid once per slab (2K rows of W*S) instead of once per wave, with S-row waves: more waves per
// SIMD at the same work.  Output: the T = W*S - 2K middle rows.
// LD: 0 no flips, 1 the last generation's flips to p.diff, 2 EVERY generation's flips to
// p.diff + g * p.diff_stride (golhip_step_flips: one K-deep launch fills K slots of the per-turn
// flips ring; the output rows are valid at every generation of the trapezoid, and each
// generation's new row and the centre cells it replaces sit in the same drifted frame).
template <int K, int W, int S, bool COUNT, int LD, int NC = kTileChains>
__global__ __launch_bounds__(64 * W) void gol_slab(const uint32_t *__restrict__ in,
                                                   uint32_t *__restrict__ out, StencilParams p,
                                                   unsigned long long *__restrict__ slots) {
    constexpr int T = W * S - 2 * K;
    static_assert(T >= 1 && K >= 2 && K <= 32 && W >= 2 && S >= 2, "slab geometry");
    // the waves' edge-row SUMS (3-cell sum bits and carries of the first and last row), not the
    // rows: a row's sums are computed once, by the wave that owns it, instead of also by the
    // neighbour that needs them (2 of every S + 2 row sums per wave and generation).  Wave w's
    // block is ex[par][w + 1]; blocks 0 and W + 1 stay zero, so the first and last wave read their
    // missing neighbour's sums from there without a branch, and every address of a wave's exchange
    // is one base (its upper neighbour's block) plus an immediate offset.
    __shared__ uint32_t ex[2][W + 2][4][64];
    // per-generation alive counts of the slab, per lane (summed over the waves by LDS adds; one
    // global atomic per generation per slab at the end)
    // per-generation alive counts, one slot per wave and lane (plain LDS stores; twelve waves'
    // atomic adds to ONE slot per lane serialised in the LDS pipe in front of every barrier),
    // summed over the waves by the flushing wave
    __shared__ uint32_t cnt_lds[COUNT ? K : 1][COUNT ? W : 1][64];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // XCD-aware order: the dispatcher deals workgroups round-robin over the 8 XCDs (each with its
    // own L2), so workgroup b runs on XCD b % 8.  Give XCD x a contiguous range of slabs (all
    // column chunks of consecutive bands): the halo rows and halo lanes a slab reads were written
    // by its neighbours in the previous launch on the SAME XCD, i.e. they hit that L2, except at
    // the 8 range seams.
    const int64_t ngroups = p.nbands * (int64_t)p.nchunks;
    const int64_t per_xcd = (ngroups + kXcds - 1) / kXcds;
    const int64_t group = (int64_t)(blockIdx.x % kXcds) * per_xcd + blockIdx.x / kXcds;
    if (group >= ngroups) return;  // whole workgroup (grid padded to whole XCD rounds)
    const int64_t chunk = group % p.nchunks;
    const int64_t bandi = group / p.nchunks;
    int ya, yb;
    band_rows(p, bandi, ya, yb);  // yb - ya <= T (the host sets p.band = T)
    const int nrows = yb - ya;
    const int colraw = (int)chunk * kTileChunkWords + lane - 1;
    const int col = (colraw + p.wd) % p.wd;
    const int rowbytes = (int)(p.pitch * 4);
    uint32_t c[S + 2];
    c[0] = c[S + 1] = 0;  // never read: their sums come from the neighbour waves (pre)
    load_rows<1, S>(c, in, p, ya - K + w * S, col);
    SlabPre<S> pre{};
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)ya * p.pitch, 0, nrows * rowbytes, kBufferRsrcWord3);
    __amdgpu_buffer_rsrc_t drsrc = orsrc;
    if constexpr (LD == 1)
        drsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + (int64_t)ya * p.pitch, 0,
                                                  nrows * rowbytes, kBufferRsrcWord3);
    const LaneStore ls = lane_store<false>(lane, colraw, col, p.wd);
    const bool count_lane = lane >= 2 && colraw <= p.wd;
    // slab row of c[1]: output row o = w*S + (r - 1) - K is this band's if 0 <= o < nrows
    const int o0 = w * S - K;
    if constexpr (COUNT)
        for (int j = 0; j < K; ++j) cnt_lds[j][w][lane] = 0;  // halo waves never write theirs
    if (w == 0)  // the zero neighbour blocks (ordered before any read by the first exchange's barrier)
        for (int par = 0; par < 2; ++par)
            for (int i = 0; i < 4; ++i) ex[par][0][i][lane] = ex[par][W + 1][i][lane] = 0u;
    // exchange addressing: parity 0's base and the distance to parity 1 (words)
    uint32_t *const ex_base0 = &ex[0][w][0][lane];
    constexpr int kExPar = (W + 2) * 4 * 64;
    // this wave's per-generation count slot: cnt_my[gen * W * 64] (unmasked; the flusher masks the
    // lanes outside the count window once per generation)
    uint32_t *const cnt_my = &cnt_lds[0][w][lane];
    // LDS-only barrier: the waves' global stores and count atomics stay in flight (a
    // __syncthreads() would also drain vmcnt every generation)
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    auto cnt_sum = [&](int j) {
        uint32_t a = 0;
#pragma unroll
        for (int ww = 0; ww < W; ++ww) a += cnt_lds[j][ww][lane];
        return count_lane ? a : 0u;
    };
    auto exchange = [&](int g) {
        const int par = g & 1;
        {  // this wave's edge rows' sums: published below and used by its own pass
            uint32_t xr[2] = {c[1], c[S]}, s2[2], cy2[2], c2[2];
            sums_om<2>(xr, s2, cy2, c2);
            pre.fs = s2[0], pre.fcy = cy2[0], pre.fctr = c2[0];
            pre.ls = s2[1], pre.lcy = cy2[1], pre.lctr = c2[1];
        }
        uint32_t *const b = ex_base0 + par * kExPar;  // block w (the upper neighbour's)
        b[256] = pre.fs;  // own block w + 1
        b[320] = pre.fcy;
        b[384] = pre.ls;
        b[448] = pre.lcy;
        lds_barrier();
        pre.ts = b[128];  // the upper neighbour's last row (zero block above wave 0)
        pre.tcy = b[192];
        pre.bs = b[512];  // the lower neighbour's first row (zero block below wave W - 1)
        pre.bcy = b[576];
        if constexpr (COUNT && 2 * S <= K) {
            // Generation g - 2 (0-based) is complete in LDS after this barrier.  With 2S <= K,
            // waves 0 and W - 1 hold only halo rows, dead from generation S on (g_end below),
            // i.e. for at least half the launch: they take turns summing and flushing one
            // complete generation per exchange while the other waves compute, instead of every
            // generation's flush queueing at the end of the launch.  (Measured: with S = 12 of
            // K = 16 the same scheme is slower than the end flush, and so is letting the two
            // waves flush in batches once idle: profiles/r02/r02aa_slab_flush.txt.)
            if (g >= 2 && w == ((g & 1) ? W - 1 : 0)) {
                uint32_t acc[1] = {cnt_sum(g - 2)};
                flush_counts<1>(acc, g - 2, lane, group, slots);
            }
        }
    };
    // FULL: every row of this wave is an output row of the band (interior waves): the counts need
    // no per-row mask (one v_bcnt per row instead of a select and a v_bcnt)
    const bool full = o0 >= 0 && o0 + S <= nrows;
    // HALO: no row of this wave is an output row of the band (the slab's K-row halos, or rows past
    // a short last band): it never counts and never stores, so it skips the last generation, and
    // any generation at which all its rows are already outside the trapezoid [g, W*S - g)
    const bool halo = o0 + S <= 0 || o0 >= nrows;
    auto pass = [&](auto last_c, auto full_c, auto cnt_c, int gen) {
        constexpr bool LAST = decltype(last_c)::value, FULL = decltype(full_c)::value;
        constexpr bool CNT = COUNT && decltype(cnt_c)::value;
        uint32_t cnt = 0;
        __amdgpu_buffer_rsrc_t grsrc = orsrc;  // LD == 2: this generation's flips ring slot
        if constexpr (LD == 2)
            grsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + gen * p.diff_stride + (int64_t)ya * p.pitch,
                                                      0, nrows * rowbytes, kBufferRsrcWord3);
        // (segment 0 bottom-up, REV0 -- the hand-off row above needed only at its last step --
        // measured 3-7 % slower: profiles/r02/small_boards.txt)
        gen_rows<1, S, !LAST, NC>(c, [&](auto rc, uint32_t nx, uint32_t centre) {
            constexpr int r = decltype(rc)::value;
            const int o = o0 + r - 1;
            const bool mine = FULL || (o >= 0 && o < nrows);  // wave-uniform
            if (CNT) cnt = bcnt_acc(mine ? nx : 0u, cnt);
            if constexpr (LD == 2) {  // every generation's flips (output rows only)
                Words<1> dv;
                dv.w[0] = realign_drift_rt(nx ^ centre, gen);
                golhip::store_row<1, false>(grsrc, ls, dv, mine ? o * rowbytes : kOutOfRange);
            }
            if constexpr (LAST) {
                const int rowoff = mine ? o * rowbytes : kOutOfRange;
                Words<1> v;
                v.w[0] = realign_drift<K>(nx);
                golhip::store_row<1, false>(orsrc, ls, v, rowoff);
                if constexpr (LD == 1) {
                    Words<1> dv;
                    dv.w[0] = realign_drift<K>(nx ^ centre);
                    golhip::store_row<1, false>(drsrc, ls, dv, rowoff);
                }
            }
        }, pre);
        if constexpr (CNT) cnt_my[gen * (W * 64)] = cnt;
    };
    using No = std::false_type;
    using Yes = std::true_type;
    // One generation loop per wave kind, each with a single pass body (a branch between pass
    // variants inside the loop makes the allocator reconcile c[] with v_movs every generation).
    // Slab rows [w*S, w*S + S) of this wave; generation g is valid on [g, W*S - g), so from
    // generation g_end = min(w*S + S, W*S - w*S) on all of a wave's rows are outside it.
    if constexpr (LD == 2) {
        // every generation's flips: halo waves run their dead generations too (they store
        // nothing: no output rows), so every wave runs one loop of one pass body
        if (full) {
#pragma clang loop unroll(disable)
            for (int g = 1; g < K; ++g) {
                exchange(g);
                pass(No{}, Yes{}, Yes{}, g - 1);
            }
        } else {
#pragma clang loop unroll(disable)
            for (int g = 1; g < K; ++g) {
                exchange(g);
                pass(No{}, No{}, Yes{}, g - 1);
            }
        }
        exchange(K);
        pass(Yes{}, No{}, Yes{}, K - 1);
    } else if constexpr (!COUNT) {
        // without counts every wave runs every generation: measured faster than skipping the
        // halo waves' dead generations (0.815 vs 0.847 us/turn at 5120^2, profiles/r02/r02z_slab_ab.txt)
#pragma clang loop unroll(disable)
        for (int g = 1; g < K; ++g) {
            exchange(g);
            pass(No{}, No{}, No{}, g - 1);
        }
        exchange(K);
        pass(Yes{}, No{}, No{}, K - 1);
    } else if (halo) {
        const int g_end = std::min(std::min(w * S + S, W * S - w * S), K);
        int g = 1;
#pragma clang loop unroll(disable)
        for (; g < g_end; ++g) {
            exchange(g);
            pass(No{}, No{}, No{}, g - 1);
        }
#pragma clang loop unroll(disable)
        for (; g <= K; ++g) exchange(g);  // its edge rows are garbage: nothing reads them as valid
    } else {
        if (COUNT && full) {
#pragma clang loop unroll(disable)
            for (int g = 1; g < K; ++g) {
                exchange(g);
                pass(No{}, Yes{}, Yes{}, g - 1);
            }
        } else {
#pragma clang loop unroll(disable)
            for (int g = 1; g < K; ++g) {
                exchange(g);
                pass(No{}, No{}, Yes{}, g - 1);
            }
        }
        exchange(K);
        pass(Yes{}, No{}, Yes{}, K - 1);
    }
    if constexpr (COUNT) {  // the generations not flushed yet
        lds_barrier();
        if constexpr (2 * S <= K) {
            if (w == ((K & 1) ? 0 : W - 1)) {  // K - 1 (K - 2 went in exchange(K))
                uint32_t acc[1] = {cnt_sum(K - 1)};
                flush_counts<1>(acc, K - 1, lane, group, slots);
            }
        } else {
            for (int j = w; j < K; j += W) {
                uint32_t acc[1] = {cnt_sum(j)};
                flush_counts<1>(acc, j, lane, group, slots);
            }
        }
    }
}

// gol_slab2: gol_slab with the edge-row hand-off taken OFF the critical path.  gol_slab's waves
// wait at each generation's barrier, then read their neighbours' edge-row sums from LDS, then
// update their rows in NC rolling segments: the barrier and the LDS round trip sit in front of
// every generation's work, and two segments per wave leave a SIMD with two waves on it short of
// independent instructions (PMC, configs[1] 5120^2: VALU active 31 % of the wave cycles, parked at
// barrier/waitcnt 45 %, profiles/r04/).  Here a generation is:
//   1. the 3-cell sums of ALL S own rows, op-major (S independent chains);
//   2. publish the two edge rows' sums to LDS;
//   3. the new cells of the S - 2 interior rows, op-major -- they need only the wave's own sums,
//      so they run while the neighbours are still publishing;
//   4. the barrier, the neighbours' edge sums from LDS, and the two edge rows.
// Only step 4's short tail (an LDS read and two 7-op rules) waits on the other waves.
// FM, where the per-generation counts are flushed (tuning A/B): 0 (production) the pure-halo waves
// flush generation g - 2 after every barrier when there are two per side (2S <= K), else every
// generation at the end of the launch; 1 (NC = 11) in the loop whenever there is one per side
// (S <= K); 2 (NC = 12) always at the end.
// YP (tuning A/B, NC = 13: with FM = 2): the second-dispatched half of the workgroup's waves -- the
// arbitration losers on every SIMD after each barrier (MI355X_MICROARCH.md "Two waves per SIMD"
// items 4 and 6) -- run at s_setprio 1 for the whole launch.
//
// ACT (StencilParams::act, production shapes without flips): stable-slab skipping.  A slab whose 3 x 3
// neighbourhood of slabs (bands and chunks wrap on the torus) did not change in the last generation
// of the previous launch is constant for this launch's K generations: the Life update of a cell
// depends on its radius-1 ball only, so a region of radius K around the slab that equals itself one
// generation earlier keeps the slab fixed for K generations (every band but the torus's last has
// T >= K rows -- the host checks -- and the band beyond a short last band is checked too; a chunk is
// >= 1 word wide, more than the K <= 16 bits the region reaches sideways).  Such a slab
// copies its input to its output once (then both buffers agree: `same`), adds its cached alive
// count to every generation's count slot and ends; the others compute as usual and record whether
// their output changed in the last generation, and its alive count.  Bit-exact by construction;
// on settled boards (configs[4]: ~2 600 live cells on 4096^2 for most of its 1e6 turns) nearly
// every slab is skipped.
//
// PF (tuning A/B, NC = 15: with FM = 2): the generation's workgroup barrier replaced by point-to-point
// LDS flags.  A wave waits only for its two neighbour waves, not for all W: after step 3 it waits
// lgkmcnt(0) (its edge sums are in LDS) and stores its generation number in its flag; in step 4 it
// polls its neighbours' flags until both reached the generation, then reads their sums (LDS
// operations are processed in order, so a flag seen means the sums before it are there).  The
// double-buffered exchange stays safe: a wave writes parity g & 1 again at g + 2 only after passing
// g + 1's wait, i.e. after both readers of generation g's block finished generation g.  Waves then
// drift up to one generation per wave apart, so in-loop count flushes (FM 0 / 1) are out.
template <int K, int W, int S, bool COUNT, int LD, int FM = 0, bool YP = false, bool ST = false,
          bool ACT = false, bool PF = false>
__global__ __launch_bounds__(64 * W) void gol_slab2(const uint32_t *__restrict__ in,
                                                    uint32_t *__restrict__ out, StencilParams p,
                                                    unsigned long long *__restrict__ slots) {
    constexpr int T = W * S - 2 * K;
    static_assert(T >= 1 && K >= 2 && K <= 32 && W >= 2 && S >= 3, "slab geometry");
    static_assert(!ACT || (LD == 0 && !ST), "stable-slab skipping: no flips, no stamps");
    static_assert(!PF || FM == 2, "neighbour flags: counts flushed at the end only");
    __shared__ uint32_t ex[2][W + 2][4][64];  // as gol_slab: wave w's block is ex[par][w + 1]
    __shared__ int flg[PF ? W + 2 : 1];  // PF: wave w's flag is flg[w + 1]; flg[0], flg[W + 1] never wait
    __shared__ uint32_t cnt_lds[COUNT ? K : 1][COUNT ? W : 1][64];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // XCD-aware order (gol_slab): XCD b % 8 gets a contiguous range of slabs
    const int64_t ngroups = p.nbands * (int64_t)p.nchunks;
    const int64_t per_xcd = (ngroups + kXcds - 1) / kXcds;
    const int64_t group = (int64_t)(blockIdx.x % kXcds) * per_xcd + blockIdx.x / kXcds;
    if (group >= ngroups) return;  // whole workgroup
    uint32_t act_chg = 0, act_pop = 0;  // ACT: this lane's changed bits / count at the last generation
    if constexpr (YP)
        if (w >= W / 2) __builtin_amdgcn_s_setprio(1);
    // ST (the tuning library's stamp kernels), p.stamp: phase stamps of every wave (start, rows loaded, generations done, end;
    // s_memrealtime 100 MHz), its shader cycles and HW_ID / XCC_ID
    uint64_t st_t0 = 0, st_c0 = 0, st_t1 = 0, st_t2 = 0;
    if constexpr (ST)
        if (p.stamp) st_t0 = __builtin_amdgcn_s_memrealtime(), st_c0 = __builtin_amdgcn_s_memtime();
    const int64_t chunk = group % p.nchunks;
    const int64_t bandi = group / p.nchunks;
    int ya, yb;
    band_rows(p, bandi, ya, yb);
    const int nrows = yb - ya;
    const int colraw = (int)chunk * kTileChunkWords + lane - 1;
    const int col = (colraw + p.wd) % p.wd;
    const int rowbytes = (int)(p.pitch * 4);
    // ACT: the changed bytes of the slabs within K rows, loaded before the rows (one round trip,
    // no branch or division in between): the adjacent bands, and the next one beyond an adjacent
    // band shorter than K rows (the short last band of the torus; every other band has T >= K
    // rows), x the adjacent chunks; 16 bytes (one per wave) per slab, lanes 0..59 one dword each
    uint32_t act_f = 0;
    if constexpr (ACT) {
        const int nb = (int)p.nbands, nc = (int)p.nchunks;
        const int bi = (int)bandi, ci = (int)chunk;
        const bool short_last = (int)(p.r0e - (int64_t)(nb - 1) * p.band) < K;  // slab_params: uniform bands
        auto wrap = [](int v, int n) {  // |v| < 3 n
            v = v < 0 ? v + n : v;
            v = v < 0 ? v + n : v;
            v = v >= n ? v - n : v;
            return v >= n ? v - n : v;
        };
        const int bm1 = wrap(bi - 1, nb), bp1 = wrap(bi + 1, nb);
        const int l = lane < 60 ? lane : 0;  // every lane loads (lanes 60..63 masked below)
        const int i = l / 12, j = (l >> 2) % 3, d = l & 3;
        const int bb = i == 0 ? (short_last && bm1 == nb - 1 ? wrap(bi - 2, nb) : bi)
                     : i == 1 ? bm1 : i == 2 ? bi : i == 3 ? bp1
                                               : (short_last && bp1 == nb - 1 ? wrap(bi + 2, nb) : bi);
        act_f = p.act[act_chg_off(p.act_par, ngroups) + (int64_t)(bb * nc + wrap(ci + j - 1, nc)) * 4 + d];
    }
    uint32_t c[S + 2];  // rows 1..S of this wave (c[0], c[S + 1] unused)
    c[0] = c[S + 1] = 0;
    load_rows<1, S>(c, in, p, ya - K + w * S, col);
    if constexpr (ST)
        if (p.stamp) {
            __builtin_amdgcn_s_waitcnt(0);  // the rows are in (stamp runs only)
            st_t1 = __builtin_amdgcn_s_memrealtime();
        }
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)ya * p.pitch, 0, nrows * rowbytes, kBufferRsrcWord3);
    __amdgpu_buffer_rsrc_t drsrc = orsrc;
    if constexpr (LD == 1)
        drsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + (int64_t)ya * p.pitch, 0,
                                                  nrows * rowbytes, kBufferRsrcWord3);
    const LaneStore ls = lane_store<false>(lane, colraw, col, p.wd);
    const bool count_lane = lane >= 2 && colraw <= p.wd;
    const int o0 = w * S - K;  // output row of c[1]
    if constexpr (ACT) {
        uint32_t *const same = p.act + act_same_off(ngroups);
        const uint32_t *const pop = p.act + act_pop_off(ngroups) + group * 16;  // one count per wave
        // first use of the flags after the row loads are issued (the wait is vmcnt(S), not 0)
        const int nbytes = W - 4 * (lane & 3);  // this dword's bytes that belong to waves of this shape
        const uint32_t mask = lane >= 60 || nbytes <= 0 ? 0u : nbytes >= 4 ? ~0u : (1u << (8 * nbytes)) - 1u;
        if (!p.act_reset && __builtin_amdgcn_ballot_w64((act_f & mask) != 0u) == 0) {
            // stable for K generations: output = input, every generation counts the slab's alive cells
            if (same[group] == 0) {  // the output buffer still holds an older generation: store the
                                     // rows just loaded (this wave's rows of the band) once
#pragma unroll
                for (int r = 1; r <= S; ++r) {
                    const int o = o0 + r - 1;
                    Words<1> v;
                    v.w[0] = c[r];
                    golhip::store_row<1, false>(orsrc, ls, v, o >= 0 && o < nrows ? o * rowbytes : kOutOfRange);
                }
            }
            if (w == 0) {  // vector stores / atomics from lanes, never the scalar path
                if constexpr (COUNT) {
                    const uint32_t n = __builtin_amdgcn_readlane(wave_sum_dpp(lane < W ? pop[lane] : 0u), 63);
                    if (lane < K && n)
                        __hip_atomic_fetch_add(&slots[lane * kCountSlots + (int)(group & (kCountSlots - 1))],
                                               (unsigned long long)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (lane < 4) p.act[act_chg_off(p.act_par ^ 1, ngroups) + group * 4 + lane] = 0u;
                if (lane == 0) {
                    same[group] = 1u;
                    if (p.act_stats)
                        __hip_atomic_fetch_add(&p.act_stats[kActStatSlots + (int)(group & (kActStatSlots - 1))], 1ull,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            return;
        }
        // computed: the two buffers now differ on this slab; every wave writes its changed byte and
        // count at its end (plain stores: no clearing, no atomics on the flags)
        if (w == 0 && lane == 0) {
            same[group] = 0u;
            if (p.act_stats)
                __hip_atomic_fetch_add(&p.act_stats[(int)(group & (kActStatSlots - 1))], 1ull, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if constexpr (COUNT)
        for (int j = 0; j < K; ++j) cnt_lds[j][w][lane] = 0;
    if (w == 0)
        for (int par = 0; par < 2; ++par)
            for (int i = 0; i < 4; ++i) ex[par][0][i][lane] = ex[par][W + 1][i][lane] = 0u;
    uint32_t *const ex_base0 = &ex[0][w][0][lane];
    constexpr int kExPar = (W + 2) * 4 * 64;
    uint32_t *const cnt_my = &cnt_lds[0][w][lane];
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    // PF: publish generation g (the edge sums stored before are complete first), then wait for both
    // neighbours to have published it (wave-uniform: every lane reads the same two words)
    auto publish_flag = [&](int g) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(&flg[w + 1], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto wait_neighbours = [&](int g) {
        for (;;) {
            const int up = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&flg[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            const int dn = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&flg[w + 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (up >= g && dn >= g) break;
        }
        asm volatile("" ::: "memory");  // the neighbours' sums are read after the flags
    };
    if constexpr (PF) {  // the flags and the zero blocks before any wave polls or reads them
        if (lane == 0) {
            flg[w + 1] = 0;
            if (w == 0) flg[0] = flg[W + 1] = 1 << 30;
        }
        lds_barrier();
    }
    auto cnt_sum = [&](int j) {
        uint32_t a = 0;
#pragma unroll
        for (int ww = 0; ww < W; ++ww) a += cnt_lds[j][ww][lane];
        return count_lane ? a : 0u;
    };
    // with 2S <= K the two halo waves take turns flushing the generation that is complete after
    // generation g's barrier (g - 2, 0-based), as gol_slab does
    auto flush_after_barrier = [&](int g) {
        if constexpr (COUNT && (FM == 0 ? 2 * S <= K : FM == 1 ? S <= K : false)) {
            if (g >= 2 && w == ((g & 1) ? W - 1 : 0)) {
                uint32_t acc[1] = {cnt_sum(g - 2)};
                flush_counts<1>(acc, g - 2, lane, group, slots);
            }
        }
    };
    const bool full = o0 >= 0 && o0 + S <= nrows;
    const bool halo = o0 + S <= 0 || o0 >= nrows;
    // generation g (1-based) of this wave's rows
    auto gen = [&](auto last_c, auto full_c, auto cnt_c, int g) {
        constexpr bool LAST = decltype(last_c)::value, FULL = decltype(full_c)::value;
        constexpr bool CNT = COUNT && decltype(cnt_c)::value;
        const int gi = g - 1;
        uint32_t cnt = 0;
        __amdgpu_buffer_rsrc_t grsrc = orsrc;
        if constexpr (LD == 2)
            grsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + gi * p.diff_stride + (int64_t)ya * p.pitch,
                                                      0, nrows * rowbytes, kBufferRsrcWord3);
        auto emit = [&](int r, uint32_t nx, uint32_t centre) {  // r: 1..S (compile time after unroll)
            const int o = o0 + r - 1;
            const bool mine = FULL || (o >= 0 && o < nrows);  // wave-uniform
            if (CNT) cnt = bcnt_acc(mine ? nx : 0u, cnt);
            if constexpr (LD == 2) {
                Words<1> dv;
                dv.w[0] = realign_drift_rt(nx ^ centre, gi);
                golhip::store_row<1, false>(grsrc, ls, dv, mine ? o * rowbytes : kOutOfRange);
            }
            if constexpr (LAST) {
                const int rowoff = mine ? o * rowbytes : kOutOfRange;
                Words<1> v;
                v.w[0] = realign_drift<K>(nx);
                golhip::store_row<1, false>(orsrc, ls, v, rowoff);
                if constexpr (LD == 1) {
                    Words<1> dv;
                    dv.w[0] = realign_drift<K>(nx ^ centre);
                    golhip::store_row<1, false>(drsrc, ls, dv, rowoff);
                }
                if constexpr (ACT) {  // the stored cells: changed since the previous generation? count
                    const uint32_t own = mine ? ls.own_mask : 0u;
                    act_chg |= realign_drift<K>(nx ^ centre) & own;
                    act_pop += (uint32_t)__builtin_popcount(v.w[0] & own);
                }
            }
        };
        // 1. sums of all S rows (independent chains, op-major)
        uint32_t x[S], s[S], cy[S], ctr[S];
#pragma unroll
        for (int i = 0; i < S; ++i) x[i] = c[i + 1];
        sums_om<S>(x, s, cy, ctr);
        // 2. publish the edge rows' sums
        uint32_t *const b = ex_base0 + (g & 1) * kExPar;  // block w (the upper neighbour's)
        b[256] = s[0];
        b[320] = cy[0];
        b[384] = s[S - 1];
        b[448] = cy[S - 1];
        // 3. the interior rows 2..S-1 (c[2..S-1]) from the wave's own sums
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
                emit(i + 2, nx[i], mc[i]);
                if constexpr (!LAST) c[i + 2] = nx[i];
            }
        }
        // 4. the neighbours' edge sums, then the two edge rows
        if constexpr (PF) {
            publish_flag(g);
            wait_neighbours(g);
        } else {
            lds_barrier();
        }
        const uint32_t ts = b[128], tcy = b[192];  // the upper neighbour's last row
        const uint32_t bts = b[512], btcy = b[576];  // the lower neighbour's first row
        flush_after_barrier(g);
        {
            uint32_t as[2] = {ts, s[S - 2]}, acy[2] = {tcy, cy[S - 2]};
            uint32_t ms[2] = {s[0], s[S - 1]}, mcy[2] = {cy[0], cy[S - 1]}, mc[2] = {ctr[0], ctr[S - 1]};
            uint32_t bs[2] = {s[1], bts}, bcy[2] = {cy[1], btcy}, nx[2];
            life_om<2>(as, acy, ms, mcy, mc, bs, bcy, nx, AllRows{});
            emit(1, nx[0], mc[0]);
            emit(S, nx[1], mc[1]);
            if constexpr (!LAST) {
                c[1] = nx[0];
                c[S] = nx[1];
            }
        }
        if constexpr (CNT) cnt_my[gi * (W * 64)] = cnt;
    };
    // a generation this wave sits out (all its rows dead from now on): it still publishes its edge
    // rows' sums -- at g_end its edge row is the last generation's, still read as valid by the
    // neighbour -- and keeps the barrier count
    // (PF: the same sums go to both parities in its first two idle generations; from then on nothing
    // it publishes changes, so it posts the last generation's flag and leaves the loop -- idle
    // returns true)
    auto idle = [&](int g, int g_end) {
        uint32_t x[2] = {c[1], c[S]}, s2[2], cy2[2], c2[2];
        sums_om<2>(x, s2, cy2, c2);
        uint32_t *const b = ex_base0 + (g & 1) * kExPar;
        b[256] = s2[0];
        b[320] = cy2[0];
        b[384] = s2[1];
        b[448] = cy2[1];
        if constexpr (PF) {
            if (g > g_end) {
                publish_flag(K);
                return true;
            }
            publish_flag(g);
            wait_neighbours(g);
            return false;
        } else {
            lds_barrier();
            flush_after_barrier(g);
            return false;
        }
    };
    using No = std::false_type;
    using Yes = std::true_type;
    if constexpr (LD == 2 || !COUNT) {
#pragma clang loop unroll(disable)
        for (int g = 1; g < K; ++g) gen(No{}, No{}, Yes{}, g);
        gen(Yes{}, No{}, Yes{}, K);
    } else if (halo) {
        const int g_end = std::min(std::min(w * S + S, W * S - w * S), K);
        int g = 1;
#pragma clang loop unroll(disable)
        for (; g < g_end; ++g) gen(No{}, No{}, No{}, g);
#pragma clang loop unroll(disable)
        for (; g <= K; ++g)
            if (idle(g, g_end)) break;
    } else if (full) {
#pragma clang loop unroll(disable)
        for (int g = 1; g < K; ++g) gen(No{}, Yes{}, Yes{}, g);
        gen(Yes{}, Yes{}, Yes{}, K);
    } else {
#pragma clang loop unroll(disable)
        for (int g = 1; g < K; ++g) gen(No{}, No{}, Yes{}, g);
        gen(Yes{}, No{}, Yes{}, K);
    }
    if constexpr (ST)
        if (p.stamp) st_t2 = __builtin_amdgcn_s_memrealtime();
    if constexpr (COUNT) {  // the generations not flushed yet
        lds_barrier();
        if constexpr (FM == 0 ? 2 * S <= K : FM == 1 ? S <= K : false) {
            if (w == ((K & 1) ? 0 : W - 1)) {
                uint32_t acc[1] = {cnt_sum(K - 1)};
                flush_counts<1>(acc, K - 1, lane, group, slots);
            }
        } else {
            flush_counts_strided<(K + W - 1) / W>(w, W, K, lane, group, slots, cnt_sum);
        }
    }
    if constexpr (ST)
        if (p.stamp) {
            __builtin_amdgcn_s_waitcnt(0);  // the stores and count atomics have left the wave
            const uint64_t t3 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
            const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
            const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
            if (lane == 0) {
                uint64_t *r = p.stamp + 8 * (group * W + w);
                r[0] = st_t0, r[1] = st_t1, r[2] = st_t2, r[3] = t3;
                r[4] = c1 - st_c0, r[5] = (uint64_t)hw | ((uint64_t)xcc << 32);
                r[6] = (uint64_t)group, r[7] = (uint64_t)w;
            }
        }
    if constexpr (ACT) {  // this wave's share of the slab's flags for the next launch
        const bool chg = __builtin_amdgcn_ballot_w64(act_chg != 0u) != 0;
        const uint32_t cnt = wave_sum_dpp(act_pop);
        if (lane == 63) {
            reinterpret_cast<uint8_t *>(p.act + act_chg_off(p.act_par ^ 1, ngroups) + group * 4)[w] = chg ? 1 : 0;
            p.act[act_pop_off(ngroups) + group * 16 + w] = cnt;
        }
    }
}

// gol_slabp: gol_slab2 for NARROW boards (wd <= 30 words: 960 cells or fewer), P = 64 / (wd + 2)
// sub-chunks packed into each wave.  gol_slab2 gives a wave one chunk of up to 62 words; at wd = 16
// (configs[0] 512^2) 46 of its 64 lanes carry nothing, and the launch is a chain of barrier-bound
// generations over a few workgroups (about 1 us per turn whatever the shape, profiles/r04).  Here
// lane l of a wave is column k = l % L (L = wd + 2: the west halo word, the wd words, the east halo
// word) of sub-chunk j = l / L, and sub-chunk j holds the wave's S-row segment w * P + j: a
// workgroup of W waves covers W * P * S rows, P times gol_slab2's, with the same instructions per
// wave and generation.  The segments' edge rows go through LDS with per-lane addresses (the
// segment above is the lanes L lower in the same wave, or the previous wave's last sub-chunk), and
// every count is flushed at the end of the launch (gol_slab2 FM = 2).  Lanes past P * L compute
// and discard.  The west-only drift of row_sum3 keeps a sub-chunk's garbage west neighbour (the
// east halo of the sub-chunk before) to its halo lane's low bits, as at lane 0 of gol_slab2.
template <int K, int W, int S, bool COUNT, int LD>
__global__ __launch_bounds__(64 * W) void gol_slabp(const uint32_t *__restrict__ in,
                                                    uint32_t *__restrict__ out, StencilParams p,
                                                    unsigned long long *__restrict__ slots) {
    static_assert(K >= 2 && K <= 16 && W >= 1 && S >= 3, "packed slab geometry");
    __shared__ uint32_t ex[2][W + 2][4][64];  // wave w's block is ex[par][w + 1]; 0 / W + 1 zero
    __shared__ uint32_t cnt_lds[COUNT ? K : 1][COUNT ? W : 1][64];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t ngroups = p.nbands;  // one chunk (wd <= 30)
    const int64_t per_xcd = (ngroups + kXcds - 1) / kXcds;
    const int64_t group = (int64_t)(blockIdx.x % kXcds) * per_xcd + blockIdx.x / kXcds;
    if (group >= ngroups) return;  // whole workgroup
    int ya, yb;
    band_rows(p, group, ya, yb);
    const int nrows = yb - ya;
    const int wd = (int)p.wd;
    const int L = wd + 2, P = 64 / L;
    const int j = lane / L, k = lane - j * L;
    const bool live = j < P;
    const int colraw = k - 1;
    const int col = (colraw + wd) % wd;
    const int rowbytes = (int)(p.pitch * 4);
    const int seg = w * P + j;
    const int o0 = seg * S - K;  // output row of c[1]
    uint32_t c[S + 2];
    c[0] = c[S + 1] = 0;
    {  // this lane's rows: per-lane row offsets in voffset
        const int base_row = p.wrap_rows > 0 ? 0 : (int)p.lo;
        const int span_rows = p.wrap_rows > 0 ? (int)p.wrap_rows : (int)(p.hi - p.lo);
        const __amdgpu_buffer_rsrc_t irsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t *>(in + (int64_t)base_row * p.pitch), 0, span_rows * rowbytes,
            kBufferRsrcWord3);
        RowStream rows(p, ya + o0);
#pragma unroll
        for (int r = 0; r < S; ++r) {
            c[r + 1] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
                irsrc, col * 4 + (rows.ly - base_row) * rowbytes, 0, 0);
            rows.advance();
        }
    }
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)ya * p.pitch, 0, nrows * rowbytes, kBufferRsrcWord3);
    __amdgpu_buffer_rsrc_t drsrc = orsrc;
    if constexpr (LD == 1)
        drsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + (int64_t)ya * p.pitch, 0,
                                                  nrows * rowbytes, kBufferRsrcWord3);
    LaneStore ls;
    if (live && k >= 1 && k <= wd) ls.off_full = col * 4, ls.own_mask = ~0u;
    const bool count_lane = live && k >= 2 && k <= wd + 1;
    if constexpr (COUNT)
        for (int g = 0; g < K; ++g) cnt_lds[g][w][lane] = 0;
    if (w == 0)
        for (int par = 0; par < 2; ++par)
            for (int i = 0; i < 4; ++i) ex[par][0][i][lane] = ex[par][W + 1][i][lane] = 0u;
    // LDS word offsets within one parity: publish at block w + 1; read the segment above's last row
    // ([2], [3]) and the segment below's first row ([0], [1])
    const int pub = (w + 1) * 256 + lane;
    const int top = j > 0 ? (w + 1) * 256 + 128 + lane - L : w * 256 + 128 + lane + (P - 1) * L;
    const int bot = j < P - 1 ? (w + 1) * 256 + lane + L : (w + 2) * 256 + lane - (P - 1) * L;
    constexpr int kExPar = (W + 2) * 4 * 64;
    uint32_t *const exf = &ex[0][0][0][0];
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    auto gen = [&](auto last_c, int g) {
        constexpr bool LAST = decltype(last_c)::value;
        const int gi = g - 1;
        uint32_t cnt = 0;
        __amdgpu_buffer_rsrc_t grsrc = orsrc;
        if constexpr (LD == 2)
            grsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + gi * p.diff_stride + (int64_t)ya * p.pitch,
                                                      0, nrows * rowbytes, kBufferRsrcWord3);
        auto emit = [&](int r, uint32_t nx, uint32_t centre) {
            const int o = o0 + r - 1;
            const bool mine = o >= 0 && o < nrows;  // per lane
            if (COUNT) cnt = bcnt_acc(mine ? nx : 0u, cnt);
            if constexpr (LD == 2) {
                Words<1> dv;
                dv.w[0] = realign_drift_rt(nx ^ centre, gi);
                golhip::store_row<1, false>(grsrc, ls, dv, mine ? o * rowbytes : kOutOfRange);
            }
            if constexpr (LAST) {
                const int rowoff = mine ? o * rowbytes : kOutOfRange;
                Words<1> v;
                v.w[0] = realign_drift<K>(nx);
                golhip::store_row<1, false>(orsrc, ls, v, rowoff);
                if constexpr (LD == 1) {
                    Words<1> dv;
                    dv.w[0] = realign_drift<K>(nx ^ centre);
                    golhip::store_row<1, false>(drsrc, ls, dv, rowoff);
                }
            }
        };
        uint32_t x[S], s[S], cy[S], ctr[S];
#pragma unroll
        for (int i = 0; i < S; ++i) x[i] = c[i + 1];
        sums_om<S>(x, s, cy, ctr);
        uint32_t *const e = exf + (g & 1) * kExPar;
        e[pub] = s[0];
        e[pub + 64] = cy[0];
        e[pub + 128] = s[S - 1];
        e[pub + 192] = cy[S - 1];
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
                emit(i + 2, nx[i], mc[i]);
                if constexpr (!LAST) c[i + 2] = nx[i];
            }
        }
        lds_barrier();
        const uint32_t ts = e[top], tcy = e[top + 64];
        const uint32_t bts = e[bot], btcy = e[bot + 64];
        {
            uint32_t as[2] = {ts, s[S - 2]}, acy[2] = {tcy, cy[S - 2]};
            uint32_t ms[2] = {s[0], s[S - 1]}, mcy[2] = {cy[0], cy[S - 1]}, mc[2] = {ctr[0], ctr[S - 1]};
            uint32_t bs[2] = {s[1], bts}, bcy[2] = {cy[1], btcy}, nx[2];
            life_om<2>(as, acy, ms, mcy, mc, bs, bcy, nx, AllRows{});
            emit(1, nx[0], mc[0]);
            emit(S, nx[1], mc[1]);
            if constexpr (!LAST) {
                c[1] = nx[0];
                c[S] = nx[1];
            }
        }
        if constexpr (COUNT) cnt_lds[gi][w][lane] = cnt;
    };
#pragma clang loop unroll(disable)
    for (int g = 1; g < K; ++g) gen(std::false_type{}, g);
    gen(std::true_type{}, K);
    if constexpr (COUNT) {
        lds_barrier();
        flush_counts_strided<(K + W - 1) / W>(w, W, K, lane, group, slots, [&](int g) {
            uint32_t a = 0;
#pragma unroll
            for (int ww = 0; ww < W; ++ww) a += cnt_lds[g][ww][lane];
            return count_lane ? a : 0u;
        });
    }
}

// gol_slab3: gol_slab2 software-pipelined across generations.  The phase stamps of gol_slab2
// (profiles/r04/r04n_slab_stamps.log: configs[1] 5120^2 with every count, 14.4 us per 16-turn
// launch, 10.5 of them in the generation loop, 0.66 us per generation for ~0.4 us of VALU issue)
// put the loss inside the loop: after each generation's barrier a wave reads its neighbours' edge
// sums from LDS and must wait for them, then updates only its two edge rows -- two dependency
// chains per wave, two waves per SIMD.  Here the work after the barrier starts with independent
// rows: iteration g (after barrier g) issues the LDS reads of the neighbours' sums of generation
// g - 1, computes the sums of the S - 2 interior rows of generation g (which were finished before
// the barrier) while the reads are in flight, then the two edge rows of generation g, their sums
// and their publication for barrier g + 1, and the interior rows of generation g + 1.  The same
// instructions as gol_slab2 in another order; the LDS round trip and the short edge chains overlap
// S - 2 rows of independent work.
template <int K, int W, int S, bool COUNT, int LD, bool ST = false>
__global__ __launch_bounds__(64 * W) void gol_slab3(const uint32_t *__restrict__ in,
                                                    uint32_t *__restrict__ out, StencilParams p,
                                                    unsigned long long *__restrict__ slots) {
    constexpr int T = W * S - 2 * K;
    static_assert(T >= 1 && K >= 3 && K <= 32 && W >= 2 && S >= 4, "slab geometry");
    __shared__ uint32_t ex[2][W + 2][4][64];  // as gol_slab: wave w's block is ex[par][w + 1]
    __shared__ uint32_t cnt_lds[COUNT ? K : 1][COUNT ? W : 1][64];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t ngroups = p.nbands * (int64_t)p.nchunks;
    const int64_t per_xcd = (ngroups + kXcds - 1) / kXcds;
    const int64_t group = (int64_t)(blockIdx.x % kXcds) * per_xcd + blockIdx.x / kXcds;
    if (group >= ngroups) return;  // whole workgroup
    uint64_t st_t0 = 0, st_c0 = 0, st_t1 = 0, st_t2 = 0;
    if constexpr (ST)
        if (p.stamp) st_t0 = __builtin_amdgcn_s_memrealtime(), st_c0 = __builtin_amdgcn_s_memtime();
    const int64_t chunk = group % p.nchunks;
    const int64_t bandi = group / p.nchunks;
    int ya, yb;
    band_rows(p, bandi, ya, yb);
    const int nrows = yb - ya;
    const int colraw = (int)chunk * kTileChunkWords + lane - 1;
    const int col = (colraw + p.wd) % p.wd;
    const int rowbytes = (int)(p.pitch * 4);
    uint32_t c[S + 2];  // rows 1..S of this wave (c[0], c[S + 1] unused)
    c[0] = c[S + 1] = 0;
    load_rows<1, S>(c, in, p, ya - K + w * S, col);
    if constexpr (ST)
        if (p.stamp) {
            __builtin_amdgcn_s_waitcnt(0);
            st_t1 = __builtin_amdgcn_s_memrealtime();
        }
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)ya * p.pitch, 0, nrows * rowbytes, kBufferRsrcWord3);
    __amdgpu_buffer_rsrc_t drsrc = orsrc;
    if constexpr (LD == 1)
        drsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + (int64_t)ya * p.pitch, 0,
                                                  nrows * rowbytes, kBufferRsrcWord3);
    const LaneStore ls = lane_store<false>(lane, colraw, col, p.wd);
    const bool count_lane = lane >= 2 && colraw <= p.wd;
    const int o0 = w * S - K;  // output row of c[1]
    if constexpr (COUNT)
        for (int j = 0; j < K; ++j) cnt_lds[j][w][lane] = 0;
    if (w == 0)
        for (int par = 0; par < 2; ++par)
            for (int i = 0; i < 4; ++i) ex[par][0][i][lane] = ex[par][W + 1][i][lane] = 0u;
    uint32_t *const ex_base0 = &ex[0][w][0][lane];
    constexpr int kExPar = (W + 2) * 4 * 64;
    uint32_t *const cnt_my = &cnt_lds[0][w][lane];
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    auto cnt_sum = [&](int j) {
        uint32_t a = 0;
#pragma unroll
        for (int ww = 0; ww < W; ++ww) a += cnt_lds[j][ww][lane];
        return count_lane ? a : 0u;
    };
    auto flush_after_barrier = [&](int g) {
        if constexpr (COUNT && 2 * S <= K) {
            if (g >= 2 && w == ((g & 1) ? W - 1 : 0)) {
                uint32_t acc[1] = {cnt_sum(g - 2)};
                flush_counts<1>(acc, g - 2, lane, group, slots);
            }
        }
    };
    const bool full = o0 >= 0 && o0 + S <= nrows;
    const bool halo = o0 + S <= 0 || o0 >= nrows;
    // the sums (s, cy) and drifted centres (ctr) of the wave's S rows of the last generation whose
    // rows are complete; cnt: the popcount of the generation being assembled
    uint32_t s[S], cy[S], ctr[S];
    uint32_t cnt = 0;
    // row r (1..S) of generation gi (0-based): counts, flips, the output store of the last one
    auto emit = [&](auto last_c, auto full_c, auto cnt_c, int r, uint32_t nx, uint32_t centre, int gi) {
        constexpr bool LAST = decltype(last_c)::value, FULL = decltype(full_c)::value;
        constexpr bool CNT = COUNT && decltype(cnt_c)::value;
        const int o = o0 + r - 1;
        const bool mine = FULL || (o >= 0 && o < nrows);  // wave-uniform
        if (CNT) cnt = bcnt_acc(mine ? nx : 0u, cnt);
        if constexpr (LD == 2) {
            const __amdgpu_buffer_rsrc_t grsrc = __builtin_amdgcn_make_buffer_rsrc(
                p.diff + gi * p.diff_stride + (int64_t)ya * p.pitch, 0, nrows * rowbytes, kBufferRsrcWord3);
            Words<1> dv;
            dv.w[0] = realign_drift_rt(nx ^ centre, gi);
            golhip::store_row<1, false>(grsrc, ls, dv, mine ? o * rowbytes : kOutOfRange);
        }
        if constexpr (LAST) {
            const int rowoff = mine ? o * rowbytes : kOutOfRange;
            Words<1> v;
            v.w[0] = realign_drift<K>(nx);
            golhip::store_row<1, false>(orsrc, ls, v, rowoff);
            if constexpr (LD == 1) {
                Words<1> dv;
                dv.w[0] = realign_drift<K>(nx ^ centre);
                golhip::store_row<1, false>(drsrc, ls, dv, rowoff);
            }
        }
    };
    auto publish = [&](int g) {  // the edge rows' sums read by the neighbours after barrier g
        uint32_t *const b = ex_base0 + (g & 1) * kExPar;
        b[256] = s[0];
        b[320] = cy[0];
        b[384] = s[S - 1];
        b[448] = cy[S - 1];
    };
    // the interior rows 2..S-1 of generation gi (0-based) from the sums of all S rows
    auto interior = [&](auto last_c, auto full_c, auto cnt_c, int gi) {
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
            emit(last_c, full_c, cnt_c, i + 2, nx[i], mc[i], gi);
            c[i + 2] = nx[i];
        }
    };
    // iteration g (1-based, after barrier g): generation g's edge rows; with NEXT, generation
    // g + 1's interior rows (LASTI: that is the launch's last generation)
    auto iter = [&](auto laste_c, auto next_c, auto lasti_c, auto full_c, auto cnt_c, int g) {
        constexpr bool NEXT = decltype(next_c)::value;
        lds_barrier();
        const uint32_t *const b = ex_base0 + (g & 1) * kExPar;
        const uint32_t ts = b[128], tcy = b[192];    // the upper neighbour's last row
        const uint32_t bts = b[512], btcy = b[576];  // the lower neighbour's first row
        flush_after_barrier(g);
        // generation g - 1's sums of rows 1, 2, S - 1, S and centres of 1, S
        const uint32_t es0 = s[0], ecy0 = cy[0], ec0 = ctr[0], ns0 = s[1], ncy0 = cy[1];
        const uint32_t es1 = s[S - 1], ecy1 = cy[S - 1], ec1 = ctr[S - 1], ns1 = s[S - 2], ncy1 = cy[S - 2];
        if constexpr (NEXT) {  // generation g's interior rows (done before the barrier): their sums
            uint32_t x[S - 2], s2[S - 2], cy2[S - 2], c2[S - 2];
#pragma unroll
            for (int i = 0; i < S - 2; ++i) x[i] = c[i + 2];
            sums_om<S - 2>(x, s2, cy2, c2);
#pragma unroll
            for (int i = 0; i < S - 2; ++i) s[i + 1] = s2[i], cy[i + 1] = cy2[i], ctr[i + 1] = c2[i];
        }
        {  // generation g's edge rows, from the neighbours' sums
            uint32_t as[2] = {ts, ns1}, acy[2] = {tcy, ncy1};
            uint32_t ms[2] = {es0, es1}, mcy[2] = {ecy0, ecy1}, mc[2] = {ec0, ec1};
            uint32_t bs[2] = {ns0, bts}, bcy[2] = {ncy0, btcy}, nx[2];
            life_om<2>(as, acy, ms, mcy, mc, bs, bcy, nx, AllRows{});
            emit(laste_c, full_c, cnt_c, 1, nx[0], mc[0], g - 1);
            emit(laste_c, full_c, cnt_c, S, nx[1], mc[1], g - 1);
            c[1] = nx[0];
            c[S] = nx[1];
        }
        if constexpr (COUNT && decltype(cnt_c)::value) {
            cnt_my[(g - 1) * (W * 64)] = cnt;
            cnt = 0;
        }
        if constexpr (NEXT) {  // the edge rows' sums, published for barrier g + 1
            uint32_t x[2] = {c[1], c[S]}, s2[2], cy2[2], c2[2];
            sums_om<2>(x, s2, cy2, c2);
            s[0] = s2[0], cy[0] = cy2[0], ctr[0] = c2[0];
            s[S - 1] = s2[1], cy[S - 1] = cy2[1], ctr[S - 1] = c2[1];
            publish(g + 1);
            interior(lasti_c, full_c, cnt_c, g);  // generation g + 1 (0-based g)
        }
    };
    using No = std::false_type;
    using Yes = std::true_type;
    // prologue: the sums of the loaded rows, their edge sums for barrier 1, generation 1's interior
    {
        uint32_t x[S];
#pragma unroll
        for (int i = 0; i < S; ++i) x[i] = c[i + 1];
        sums_om<S>(x, s, cy, ctr);
        publish(1);
    }
    // the full loop of a wave with output rows: generations 1 .. K
    auto run_all = [&](auto full_c, auto cnt_c) {
        interior(No{}, full_c, cnt_c, 0);
#pragma clang loop unroll(disable)
        for (int g = 1; g < K - 1; ++g) iter(No{}, Yes{}, No{}, full_c, cnt_c, g);
        iter(No{}, Yes{}, Yes{}, full_c, cnt_c, K - 1);
        iter(Yes{}, No{}, No{}, full_c, cnt_c, K);
    };
    if constexpr (LD == 2 || !COUNT) {
        run_all(No{}, Yes{});
    } else if (halo) {
        // a pure-halo wave computes while its rows can still reach an output row, then only keeps
        // the barrier count (gol_slab2's g_end; its last publication -- generation g_end - 1's edge
        // sums, read after barrier g_end -- happens in iteration g_end - 1)
        const int g_end = std::min(std::min(w * S + S, W * S - w * S), K);
        interior(No{}, No{}, No{}, 0);
        int g = 1;
#pragma clang loop unroll(disable)
        for (; g < g_end && g < K - 1; ++g) iter(No{}, Yes{}, No{}, No{}, No{}, g);
        if (g < g_end && g == K - 1) {
            iter(No{}, Yes{}, Yes{}, No{}, No{}, g);
            ++g;
        }
        if (g < g_end && g == K) {
            iter(Yes{}, No{}, No{}, No{}, No{}, g);
            ++g;
        }
#pragma clang loop unroll(disable)
        for (; g <= K; ++g) {
            lds_barrier();
            flush_after_barrier(g);
        }
    } else if (full) {
        run_all(Yes{}, Yes{});
    } else {
        run_all(No{}, Yes{});
    }
    if constexpr (ST)
        if (p.stamp) st_t2 = __builtin_amdgcn_s_memrealtime();
    if constexpr (COUNT) {  // the generations not flushed yet
        lds_barrier();
        if constexpr (2 * S <= K) {
            if (w == ((K & 1) ? 0 : W - 1)) {
                uint32_t acc[1] = {cnt_sum(K - 1)};
                flush_counts<1>(acc, K - 1, lane, group, slots);
            }
        } else {
            for (int j = w; j < K; j += W) {
                uint32_t acc[1] = {cnt_sum(j)};
                flush_counts<1>(acc, j, lane, group, slots);
            }
        }
    }
    if constexpr (ST)
        if (p.stamp) {
            __builtin_amdgcn_s_waitcnt(0);
            const uint64_t t3 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
            const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
            const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
            if (lane == 0) {
                uint64_t *r = p.stamp + 8 * (group * W + w);
                r[0] = st_t0, r[1] = st_t1, r[2] = st_t2, r[3] = t3;
                r[4] = c1 - st_c0, r[5] = (uint64_t)hw | ((uint64_t)xcc << 32);
                r[6] = (uint64_t)group, r[7] = (uint64_t)w;
            }
        }
}

template <int K, int T>
hipError_t launch_tile_kt(const uint32_t *in, uint32_t *out, const StencilParams &p,
                          unsigned long long *slots, hipStream_t s) {
    const int64_t waves = p.nbands * (int64_t)p.nchunks;
    const unsigned blocks = (unsigned)std::max<int64_t>(1, (waves + 3) / 4);
    if (p.diff) {
        if (slots)
            hipLaunchKernelGGL((gol_tile<K, T, true, true>), dim3(blocks), dim3(256), 0, s, in, out, p, slots);
        else
            hipLaunchKernelGGL((gol_tile<K, T, false, true>), dim3(blocks), dim3(256), 0, s, in, out, p, slots);
    } else if (slots) {
        hipLaunchKernelGGL((gol_tile<K, T, true, false>), dim3(blocks), dim3(256), 0, s, in, out, p, slots);
    } else {
        hipLaunchKernelGGL((gol_tile<K, T, false, false>), dim3(blocks), dim3(256), 0, s, in, out, p, slots);
    }
    return hipGetLastError();
}

// The production slab shapes (pick_reg_kernel): only these instantiate the every-generation
// flips variant (LD = 2).  NC = kSlab2 selects gol_slab2 (the edge hand-off off the critical path).
constexpr int kSlab2 = 9;
constexpr int kSlab3 = 10;  // gol_slab3: gol_slab2 pipelined across generations
constexpr int kSlab2F = 11;  // gol_slab2, counts flushed in the launch whenever S <= K (FM = 1)
constexpr int kSlab2E = 12;  // gol_slab2, counts flushed at the end of the launch (FM = 2)
constexpr int kSlab2P = 13;  // gol_slab2 FM = 2 with the younger half of the waves at s_setprio 1
constexpr int kSlabP = 14;  // gol_slabp: P = 64 / (wd + 2) row segments packed per wave (wd <= 62)
constexpr int kSlab2Q = 15;  // gol_slab2 FM = 2 with neighbour flags instead of the barrier (PF)
constexpr bool slab_prod_ws(int K, int W, int S) {
    return (K == 16 && W == 8 && S == 12) || (K == 16 && W == 12 && S == 8) ||
           (K == 16 && W == 12 && S == 7) || (K == 16 && W == 16 && S == 6) || (K == 16 && W == 16 && S == 4) ||
           (K == 16 && W == 12 && S == 4) ||
           (K == 8 && W == 8 && S == 8) ||
           (K == 12 && W == 8 && S == 8) ||
           ((K == 16 || K == 12 || K == 8 || K == 4 || K == 2) && S == 3 && (W == 4 || W == 6 || W == 8));
}
constexpr bool slab_prod_shape(int K, int W, int S, int NC) {
    return slab_prod_ws(K, W, S) &&
           (NC == kSlab2 || NC == kSlab3 || NC == kSlab2F || NC == kSlab2E || NC == kSlab2P || NC == kSlabP ||
            (K == 16 ? NC == 2 : NC == 4));
}

template <int K, int W, int S, int NC, bool ST = false>
hipError_t launch_slab_kws(const uint32_t *in, uint32_t *out, const StencilParams &p,
                           unsigned long long *slots, hipStream_t s) {
    const int64_t ngroups = p.nbands * (int64_t)p.nchunks;
    const unsigned blocks = (unsigned)std::max<int64_t>(1, (ngroups + kXcds - 1) / kXcds * kXcds);
    const dim3 block(64 * W);
    if constexpr (NC == kSlab3) {
        if (p.diff && p.diff_stride > 0) {
            if constexpr (slab_prod_shape(K, W, S, NC)) {
                if (slots)
                    hipLaunchKernelGGL((gol_slab3<K, W, S, true, 2, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
                else
                    hipLaunchKernelGGL((gol_slab3<K, W, S, false, 2, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
                return hipGetLastError();
            } else {
                return hipErrorNotSupported;
            }
        }
        const int ld = p.diff ? 1 : 0;
        if (ld && slots)
            hipLaunchKernelGGL((gol_slab3<K, W, S, true, 1, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        else if (ld)
            hipLaunchKernelGGL((gol_slab3<K, W, S, false, 1, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        else if (slots)
            hipLaunchKernelGGL((gol_slab3<K, W, S, true, 0, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        else
            hipLaunchKernelGGL((gol_slab3<K, W, S, false, 0, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        return hipGetLastError();
    }
    if constexpr (NC == kSlabP) {
        if (p.wd > 62 || p.nchunks != 1) return hipErrorInvalidValue;
        if (p.diff && p.diff_stride > 0) {
            if constexpr (slab_prod_shape(K, W, S, NC)) {
                if (slots)
                    hipLaunchKernelGGL((gol_slabp<K, W, S, true, 2>), dim3(blocks), block, 0, s, in, out, p, slots);
                else
                    hipLaunchKernelGGL((gol_slabp<K, W, S, false, 2>), dim3(blocks), block, 0, s, in, out, p, slots);
                return hipGetLastError();
            } else {
                return hipErrorNotSupported;
            }
        }
        const int ld = p.diff ? 1 : 0;
        if (ld && slots)
            hipLaunchKernelGGL((gol_slabp<K, W, S, true, 1>), dim3(blocks), block, 0, s, in, out, p, slots);
        else if (ld)
            hipLaunchKernelGGL((gol_slabp<K, W, S, false, 1>), dim3(blocks), block, 0, s, in, out, p, slots);
        else if (slots)
            hipLaunchKernelGGL((gol_slabp<K, W, S, true, 0>), dim3(blocks), block, 0, s, in, out, p, slots);
        else
            hipLaunchKernelGGL((gol_slabp<K, W, S, false, 0>), dim3(blocks), block, 0, s, in, out, p, slots);
        return hipGetLastError();
    }
    if constexpr (NC == kSlab2Q) {  // tuning only: no flips every generation, no skipping
        if ((p.diff && p.diff_stride > 0) || p.act) return hipErrorNotSupported;
        const int ld = p.diff ? 1 : 0;
        if (ld && slots)
            hipLaunchKernelGGL((gol_slab2<K, W, S, true, 1, 2, false, ST, false, true>), dim3(blocks), block, 0, s, in, out, p, slots);
        else if (ld)
            hipLaunchKernelGGL((gol_slab2<K, W, S, false, 1, 2, false, ST, false, true>), dim3(blocks), block, 0, s, in, out, p, slots);
        else if (slots)
            hipLaunchKernelGGL((gol_slab2<K, W, S, true, 0, 2, false, ST, false, true>), dim3(blocks), block, 0, s, in, out, p, slots);
        else
            hipLaunchKernelGGL((gol_slab2<K, W, S, false, 0, 2, false, ST, false, true>), dim3(blocks), block, 0, s, in, out, p, slots);
        return hipGetLastError();
    }
    if constexpr (NC == kSlab2F || NC == kSlab2E || NC == kSlab2P) {
        constexpr int FM = NC == kSlab2P ? 2 : NC - 10;
        constexpr bool YP = NC == kSlab2P;
        if (p.diff && p.diff_stride > 0) {
            if constexpr (slab_prod_shape(K, W, S, NC)) {
                if (slots)
                    hipLaunchKernelGGL((gol_slab2<K, W, S, true, 2, FM, YP, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
                else
                    hipLaunchKernelGGL((gol_slab2<K, W, S, false, 2, FM, YP, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
                return hipGetLastError();
            } else {
                return hipErrorNotSupported;
            }
        }
        if (p.act) {  // stable-slab skipping (production shapes, no flips)
            if constexpr (slab_prod_shape(K, W, S, NC) && !ST && !YP) {
                if (p.diff) return hipErrorNotSupported;
                if (slots)
                    hipLaunchKernelGGL((gol_slab2<K, W, S, true, 0, FM, false, false, true>), dim3(blocks), block, 0, s, in, out, p, slots);
                else
                    hipLaunchKernelGGL((gol_slab2<K, W, S, false, 0, FM, false, false, true>), dim3(blocks), block, 0, s, in, out, p, slots);
                return hipGetLastError();
            } else {
                return hipErrorNotSupported;
            }
        }
        const int ld = p.diff ? 1 : 0;
        if (ld && slots)
            hipLaunchKernelGGL((gol_slab2<K, W, S, true, 1, FM, YP, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        else if (ld)
            hipLaunchKernelGGL((gol_slab2<K, W, S, false, 1, FM, YP, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        else if (slots)
            hipLaunchKernelGGL((gol_slab2<K, W, S, true, 0, FM, YP, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        else
            hipLaunchKernelGGL((gol_slab2<K, W, S, false, 0, FM, YP, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        return hipGetLastError();
    }
    if constexpr (NC == kSlab2) {
        if (p.diff && p.diff_stride > 0) {
            if constexpr (slab_prod_shape(K, W, S, NC)) {
                if (slots)
                    hipLaunchKernelGGL((gol_slab2<K, W, S, true, 2, 0, false, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
                else
                    hipLaunchKernelGGL((gol_slab2<K, W, S, false, 2, 0, false, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
                return hipGetLastError();
            } else {
                return hipErrorNotSupported;
            }
        }
        if (p.act) {  // stable-slab skipping (production shapes, no flips)
            if constexpr (slab_prod_shape(K, W, S, NC) && !ST) {
                if (p.diff) return hipErrorNotSupported;
                if (slots)
                    hipLaunchKernelGGL((gol_slab2<K, W, S, true, 0, 0, false, false, true>), dim3(blocks), block, 0, s, in, out, p, slots);
                else
                    hipLaunchKernelGGL((gol_slab2<K, W, S, false, 0, 0, false, false, true>), dim3(blocks), block, 0, s, in, out, p, slots);
                return hipGetLastError();
            } else {
                return hipErrorNotSupported;
            }
        }
        const int ld = p.diff ? 1 : 0;
        if (ld && slots)
            hipLaunchKernelGGL((gol_slab2<K, W, S, true, 1, 0, false, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        else if (ld)
            hipLaunchKernelGGL((gol_slab2<K, W, S, false, 1, 0, false, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        else if (slots)
            hipLaunchKernelGGL((gol_slab2<K, W, S, true, 0, 0, false, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        else
            hipLaunchKernelGGL((gol_slab2<K, W, S, false, 0, 0, false, ST>), dim3(blocks), block, 0, s, in, out, p, slots);
        return hipGetLastError();
    }
    if constexpr (NC != kSlabP) {
        if (p.diff && p.diff_stride > 0) {
            if constexpr (slab_prod_shape(K, W, S, NC)) {
                if (slots)
                    hipLaunchKernelGGL((gol_slab<K, W, S, true, 2, NC>), dim3(blocks), block, 0, s, in, out, p, slots);
                else
                    hipLaunchKernelGGL((gol_slab<K, W, S, false, 2, NC>), dim3(blocks), block, 0, s, in, out, p, slots);
                return hipGetLastError();
            } else {
                return hipErrorNotSupported;
            }
        }
        if (p.diff) {
            if (slots)
                hipLaunchKernelGGL((gol_slab<K, W, S, true, 1, NC>), dim3(blocks), block, 0, s, in, out, p, slots);
            else
                hipLaunchKernelGGL((gol_slab<K, W, S, false, 1, NC>), dim3(blocks), block, 0, s, in, out, p, slots);
        } else if (slots) {
            hipLaunchKernelGGL((gol_slab<K, W, S, true, 0, NC>), dim3(blocks), block, 0, s, in, out, p, slots);
        } else {
            hipLaunchKernelGGL((gol_slab<K, W, S, false, 0, NC>), dim3(blocks), block, 0, s, in, out, p, slots);
        }
    }
    return hipGetLastError();
}

}  // namespace
}  // namespace golhip
