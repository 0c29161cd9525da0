// stencil_board.hip -- gol_board: the WHOLE board in one workgroup, for the reference's own sizes
// (boards at most 16 packed words = 512 cells wide and 512 rows tall: images/16x16 ... 512x512,
// configs[0]).
//
// Every other kernel splits a board over many workgroups and pays for it per launch: a K-row
// trapezoid of redundant rows at each slab edge (temporal blocking), halo lanes at each column
// chunk, and a launch boundary (dispatch ramp, row loads, tail: ~3 us) every K <= 16 generations.
// On a 512^2 board those launches are latency-bound (~0.5 us per generation whatever the shape,
// profiles/r04/r04p4_narrow_sweep.log) and the boundaries add ~30 %.  Here one workgroup holds
// the whole torus in registers for ALL the generations of a call (K is a runtime count, up to
// kBoardMaxK): no trapezoid, no halo lanes, no launch boundary inside a call, per-generation counts
// summed in LDS.
//
// Layout: a wave's 64 lanes are four 16-lane DPP rows ("segments"); segment sg = 4 w + (lane / 16)
// holds board rows [sg R, sg R + R), one row per VGPR, lane l % 16 holding word (l % 16) % wd of
// the row -- a row of wd in {4, 8, 16} words is replicated to 16 lanes (the torus evolution keeps
// the horizontal period).  The west neighbour word is DPP row_ror:1 (the torus wrap inside the
// 16-lane row), so there is no horizontal halo and no stale bit: the drifting sums of gol_stencil
// (one DPP + two v_alignbit + nine v_bitop3 per word per generation) move the whole row one bit east
// per generation around the torus, and the stores rotate it back by K bits at the end.  Vertical
// neighbours are the next VGPR of the same lane; a segment's edge rows' SUMS go through LDS to the
// segments above and below (double-buffered by generation parity, one LDS-only barrier per
// generation), as in gol_slab2: the interior rows are computed before the barrier.
#include "stencil_tile.hpp"

namespace golhip {
namespace {

__device__ __forceinline__ uint32_t west16(uint32_t v) {  // lane l <- lane (l - 1) mod 16 of its row
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121 /* row_ror:1 */, 0xf, 0xf, false);
}

// Drifting 3-cell sums of N rows, op-major (sums_om with the 16-lane torus wrap).
template <int N>
__device__ __forceinline__ void sums16(const uint32_t (&x)[N], uint32_t (&s)[N], uint32_t (&cy)[N],
                                       uint32_t (&ctr)[N]) {
    uint32_t wl[N], w2[N];
#pragma unroll
    for (int i = 0; i < N; ++i) wl[i] = west16(x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) ctr[i] = __builtin_amdgcn_alignbit(x[i], wl[i], 31);  // cell x-1 onto x
#pragma unroll
    for (int i = 0; i < N; ++i) w2[i] = __builtin_amdgcn_alignbit(x[i], wl[i], 30);  // cell x-2 onto x
#pragma unroll
    for (int i = 0; i < N; ++i) s[i] = GOL_BOP3(w2[i], ctr[i], x[i], kXor3);
#pragma unroll
    for (int i = 0; i < N; ++i) cy[i] = GOL_BOP3(w2[i], ctr[i], x[i], kMaj);
}

// The word of a drifted row (K bits east around the replicated 512-bit torus) rotated back: bits
// [32 j + K, 32 j + K + 32) of the 16-lane row, for lane j of the row.
__device__ __forceinline__ uint32_t unrotate16(uint32_t v, int lane, int K) {
    const int base = lane & ~15, j = lane & 15, q = (K >> 5) & 15, r = K & 31;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((base + ((j + q) & 15)) << 2, (int)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((base + ((j + q + 1) & 15)) << 2, (int)v);
    return __builtin_amdgcn_alignbit(hi, lo, r);
}

// wave_sum_dpp of N values at once (the six DPP steps interleaved over the N independent sums)
template <int N>
__device__ __forceinline__ void wave_sum_dpp_n(uint32_t (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i], 0x111, 0xf, 0xf, false);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i], 0x112, 0xf, 0xf, false);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i], 0x114, 0xf, 0xf, false);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i], 0x118, 0xf, 0xf, false);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i], 0x142, 0xa, 0xf, false);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i], 0x143, 0xc, 0xf, false);
}

// W waves, R rows per segment: the board has exactly 4 W R rows.  COUNT: generation g's count of
// wave w into slots[g * kCountSlots + w] with a plain store from one lane (count_finalize sums the
// slots and re-zeroes them; W <= 16 < kCountSlots).  An LDS atomic per generation compiled to the
// atomic optimiser's lane loop plus a ds_add on the wave's critical path; the per-generation LDS
// array also capped K by the LDS size.  LD: the last generation's flips (gol/distributor.go:53-59)
// into p.diff.
template <int W, int R, bool COUNT, bool LD>
__global__ __launch_bounds__(64 * W) void gol_board(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                    StencilParams p, unsigned long long *__restrict__ slots,
                                                    int K) {
    constexpr int NSEG = 4 * W;
    __shared__ uint32_t ex[2][NSEG][4][16];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int c16 = lane & 15;
    const int sg = 4 * w + (lane >> 4);
    const int wd = p.wd;
    const bool own = c16 < wd;  // one copy of the replicated row stores and counts
    uint32_t c[R];
#pragma unroll
    for (int r = 0; r < R; ++r) c[r] = in[(int64_t)(sg * R + r) * p.pitch + c16 % wd];
    const int up = (sg + NSEG - 1) % NSEG, dn = (sg + 1) % NSEG;
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    uint32_t dlast[LD ? R : 1];  // LD: the last generation's flips (drifted frame)
    // generation g (exchange buffer par = g & 1): the rows advance in place; returns this lane's
    // alive cells of the new generation (COUNT)
    auto gen = [&](int g, int par) -> uint32_t {
        uint32_t s[R], cy[R], ctr[R], nx[R];
        sums16<R>(c, s, cy, ctr);
        ex[par][sg][0][c16] = s[0];
        ex[par][sg][1][c16] = cy[0];
        ex[par][sg][2][c16] = s[R - 1];
        ex[par][sg][3][c16] = cy[R - 1];
        if constexpr (R >= 3) {  // the interior rows from the segment's own sums
            constexpr int NI = R - 2;
            uint32_t as[NI], acy[NI], ms[NI], mcy[NI], mc[NI], bs[NI], bcy[NI], ni[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                as[i] = s[i], acy[i] = cy[i];
                ms[i] = s[i + 1], mcy[i] = cy[i + 1], mc[i] = ctr[i + 1];
                bs[i] = s[i + 2], bcy[i] = cy[i + 2];
            }
            life_om<NI>(as, acy, ms, mcy, mc, bs, bcy, ni, AllRows{});
#pragma unroll
            for (int i = 0; i < NI; ++i) nx[i + 1] = ni[i];
        }
        lds_barrier();
        const uint32_t ts = ex[par][up][2][c16], tcy = ex[par][up][3][c16];  // the row above row 0
        const uint32_t bts = ex[par][dn][0][c16], btcy = ex[par][dn][1][c16];  // below row R - 1
        if constexpr (R == 1) {
            uint32_t as[1] = {ts}, acy[1] = {tcy}, ms[1] = {s[0]}, mcy[1] = {cy[0]}, mc[1] = {ctr[0]};
            uint32_t bs[1] = {bts}, bcy[1] = {btcy}, n1[1];
            life_om<1>(as, acy, ms, mcy, mc, bs, bcy, n1, AllRows{});
            nx[0] = n1[0];
        } else {
            uint32_t as[2] = {ts, s[R - 2]}, acy[2] = {tcy, cy[R - 2]};
            uint32_t ms[2] = {s[0], s[R - 1]}, mcy[2] = {cy[0], cy[R - 1]}, mc[2] = {ctr[0], ctr[R - 1]};
            uint32_t bs[2] = {s[1], bts}, bcy[2] = {cy[1], btcy}, n2[2];
            life_om<2>(as, acy, ms, mcy, mc, bs, bcy, n2, AllRows{});
            nx[0] = n2[0];
            nx[R - 1] = n2[1];
        }
        uint32_t a = 0;
        if constexpr (COUNT)
#pragma unroll
            for (int r = 0; r < R; ++r) a += (uint32_t)__builtin_popcount(own ? nx[r] : 0u);
        if constexpr (LD)
            if (g == K - 1)
#pragma unroll
                for (int r = 0; r < R; ++r) dlast[r] = nx[r] ^ ctr[r];  // same (new) frame
#pragma unroll
        for (int r = 0; r < R; ++r) c[r] = nx[r];
        return a;
    };
    // Generations in groups of 4: their four per-wave count reductions (6 dependent DPP adds each)
    // run interleaved after the group instead of one chain inside every generation.
    int g = 0;
#pragma clang loop unroll(disable)
    for (; g + 4 <= K; g += 4) {
        uint32_t a[4];
        a[0] = gen(g, 0);
        a[1] = gen(g + 1, 1);
        a[2] = gen(g + 2, 0);
        a[3] = gen(g + 3, 1);
        if constexpr (COUNT) {
            wave_sum_dpp_n<4>(a);
            if (lane == 63)
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (a[u]) slots[(int64_t)(g + u) * kCountSlots + w] = a[u];  // vector stores (lane 63)
        }
    }
#pragma clang loop unroll(disable)
    for (; g < K; ++g) {
        uint32_t a = gen(g, g & 1);
        if constexpr (COUNT) {
            a = wave_sum_dpp(a);
            if (lane == 63 && a) slots[(int64_t)g * kCountSlots + w] = a;
        }
    }
    // the rows back in the board frame (K bits west around the torus), one copy stored
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t v = unrotate16(c[r], lane, K);
        if (own) out[(int64_t)(sg * R + r) * p.pitch + c16] = v;
        if constexpr (LD) {
            const uint32_t d = unrotate16(dlast[r], lane, K);
            if (own) p.diff[(int64_t)(sg * R + r) * p.pitch + c16] = d;
        }
    }
}

template <int W, int R>
hipError_t launch_board_wr(int K, const uint32_t *in, uint32_t *out, const StencilParams &p,
                           unsigned long long *slots, hipStream_t s) {
    if (p.diff && slots)
        hipLaunchKernelGGL((gol_board<W, R, true, true>), dim3(1), dim3(64 * W), 0, s, in, out, p, slots, K);
    else if (p.diff)
        hipLaunchKernelGGL((gol_board<W, R, false, true>), dim3(1), dim3(64 * W), 0, s, in, out, p, slots, K);
    else if (slots)
        hipLaunchKernelGGL((gol_board<W, R, true, false>), dim3(1), dim3(64 * W), 0, s, in, out, p, slots, K);
    else
        hipLaunchKernelGGL((gol_board<W, R, false, false>), dim3(1), dim3(64 * W), 0, s, in, out, p, slots, K);
    return hipGetLastError();
}

// (W, R) by board height, first match: 4 W R == height.  16 waves while the rows allow (4 per SIMD
// hide the VALU latency of each wave's R independent rows), then fewer.
#define GOLHIP_BOARD_SHAPES(X) X(16, 8) X(16, 4) X(8, 4) X(4, 4) X(2, 4) X(1, 4) X(1, 2) X(1, 1)

}  // namespace

bool stencil_board_shape(int64_t height, int32_t wd, int *W, int *R) {
    if (wd != 4 && wd != 8 && wd != 16) return false;  // 16 % wd == 0: the row replicates to 16 lanes
#define GOLHIP_X(WW, RR)                       \
    if (height == 4 * WW * RR) {               \
        if (W) *W = WW;                        \
        if (R) *R = RR;                        \
        return true;                           \
    }
    GOLHIP_BOARD_SHAPES(GOLHIP_X)
#undef GOLHIP_X
    return false;
}

hipError_t launch_stencil_board(int K, int W, int R, const uint32_t *in_row0, uint32_t *out_row0,
                                const StencilParams &p, unsigned long long *slots, hipStream_t s) {
    if (K < 1 || K > kBoardMaxK || p.wrap_rows != (int64_t)4 * W * R) return hipErrorInvalidValue;
#define GOLHIP_X(WW, RR) \
    if (W == WW && R == RR) return launch_board_wr<WW, RR>(K, in_row0, out_row0, p, slots, s);
    GOLHIP_BOARD_SHAPES(GOLHIP_X)
#undef GOLHIP_X
    return hipErrorInvalidValue;
}

}  // namespace golhip
