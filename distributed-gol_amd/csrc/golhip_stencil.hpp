// golhip_stencil.hpp -- device code of the hot path (gol_stencil, gol_step1, gol_stencil_split)
// and its launch templates, shared by the per-depth translation units stencil_k*.hip and
// stencil_split.hip (one TU per launch depth K so the kernels build in parallel).
#pragma once
// golhip_kernels.hip -- hand-written gfx950 (CDNA4, wave64) kernels of libgolhip.
//
// Hot path: gol_stencil<K>, a temporally blocked, bit-sliced B3/S23 stencil on a 1-bit-per-cell
// torus.  It replaces the reference's per-cell worker loop
//   calculateNextState / updateCell / countAliveCellsAdjacent   server/server.go:21-75
// and the per-turn alive scan calculateAliveCells (gol/distributor.go:153-166,186) is fused into
// it as a per-generation popcount.
//
// Mapping (see DESIGN.md for the roofline):
//   * one lane = one 32-bit word (32 cells) of a row; a wave = 64 consecutive words of a row.
//     The outer bits of lanes 0 and 63 go stale one bit per generation (their outer neighbour
//     is outside the wave): for K <= 16 lane 0 still owns its upper and lane 63 its lower half
//     word (63 words per wave), for K <= 32 lanes 0 and 63 are pure halo (62 words per wave);
//   * horizontal neighbours cross lanes with DPP and are merged with v_alignbit; the production
//     variant (DR) uses drifting row sums, which need only the west neighbour: one DPP + 2
//     v_alignbit per row, the sums and the rule are v_bitop3 (gfx950): 12 VALU per word per
//     generation (13 with the two-sided sums);
//   * each wave streams down a band of rows keeping, per generation level, the last two rows'
//     (sum, carry, cell) in registers: one input row in -> one row out per level per step, so a
//     launch advances K generations while reading the board once and writing it once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "golhip_internal.hpp"

namespace golhip {
namespace {

#ifdef GOLHIP_WEST_BPERM
// Experiment (not the production build): the west word through the LDS crossbar (ds_bpermute)
// instead of a DPP move, taking the cross-lane move off the VALU issue port.
__device__ __forceinline__ uint32_t lane_from_west(uint32_t v) {  // lane i <- lane i-1
    const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    return (uint32_t)__builtin_amdgcn_ds_bpermute(((lane - 1) & 63) << 2, (int)v);
}
#else
__device__ __forceinline__ uint32_t lane_from_west(uint32_t v) {  // lane i <- lane i-1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138 /* wave_shr:1 */, 0xf, 0xf, false);
}
#endif
__device__ __forceinline__ uint32_t lane_from_east(uint32_t v) {  // lane i <- lane i+1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130 /* wave_shl:1 */, 0xf, 0xf, false);
}
// A drifted row (K bits east of the board frame) moved back K bits west: the lane's word takes
// its upper 32 - K bits and the east lane's low K bits (K = 32: the east lane's word).
template <int K>
__device__ __forceinline__ uint32_t realign_drift(uint32_t v) {
    if constexpr (K >= 32)
        return lane_from_east(v);
    else
        return __builtin_amdgcn_alignbit(lane_from_east(v), v, K);
}

// v_bitop3_b32 (gfx950): any 3-input boolean function in one VALU op.  The immediate is the
// truth table indexed by (s0 << 2) | (s1 << 1) | s2, i.e. f(0xF0, 0xCC, 0xAA).
#define GOL_TT(EXPR) ((uint8_t)([](uint32_t a, uint32_t b, uint32_t c) { return (EXPR); }(0xF0u, 0xCCu, 0xAAu)))
#define GOL_BOP3(A, B, C, TT) __builtin_amdgcn_bitop3_b32((A), (B), (C), (TT))
constexpr uint8_t kXor3 = GOL_TT(a ^ b ^ c);                          // 0x96
constexpr uint8_t kMaj = GOL_TT((a & b) | (c & (a | b)));             // 0xE8
constexpr uint8_t kTwosEven = GOL_TT(~(a | b | c) | (~a & ~b & c) | (a & b & ~c));  // k,p,q
constexpr uint8_t kOddSelect = GOL_TT((a & ~b) | (~a & c));                    // o ? !q : mc
static_assert(kTwosEven == 0x43 && kOddSelect == 0x3a, "bitop3 truth tables");

// D consecutive 32-bit words of one row held by one lane (D = 1 or 2).
template <int D>
struct Words {
    uint32_t w[D];
};

// Neighbour words of a lane's row: by DPP from lanes -1 / +1 (NoNb), or given (Nb: level 0 reads
// them next to its own word from the LDS-DMA ring, saving the two cross-lane moves).
struct NoNb {};
struct Nb {
    uint32_t wl, el;  // the word west of the lane's first word, east of its last word
};

// Horizontal 3-cell sums (west + self + east) of a lane's D words as sum bits s and carries cy.
// The lane's outer neighbour words come from lanes -1 / +1 (one per side per row, so D = 2
// halves the cross-lane ops per word); the 1-bit shifts are v_alignbit funnel shifts.
template <int D, class N = NoNb>
__device__ __forceinline__ void row_sum3(const Words<D> &c, Words<D> &s, Words<D> &cy,
                                         const N &nb = N{}) {
    uint32_t wl, el;
    if constexpr (std::is_same_v<N, Nb>) {
        wl = nb.wl;
        el = nb.el;
    } else {
        wl = lane_from_west(c.w[D - 1]);
        el = lane_from_east(c.w[0]);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const uint32_t left = d == 0 ? wl : c.w[d - 1];
        const uint32_t right = d == D - 1 ? el : c.w[d + 1];
        const uint32_t w = __builtin_amdgcn_alignbit(c.w[d], left, 31);  // cell x-1 onto x
        const uint32_t e = __builtin_amdgcn_alignbit(right, c.w[d], 1);  // cell x+1 onto x
        s.w[d] = GOL_BOP3(w, c.w[d], e, kXor3);
        cy.w[d] = GOL_BOP3(w, c.w[d], e, kMaj);
    }
}

// Drifting 3-cell sums (DR variants, D = 1): only the WEST neighbour word is needed.  Position P
// of the result holds the sum of cells P-2, P-1, P of the input, i.e. the sum centred on cell
// P-1, and the centre cell P-1 itself (ctr): each generation moves the row one bit east in the
// lane's frame, so a level costs one cross-lane move instead of two.  Nothing is lost at the east
// edge (position 63*32+31 needs nothing beyond its own lane); the west edge goes stale two bits
// per generation instead of one bit at each edge, the same cells in total.
template <class N = NoNb>
__device__ __forceinline__ void row_sum3_drift(uint32_t c, uint32_t &s, uint32_t &cy,
                                               uint32_t &ctr, const N &nb = N{}) {
    uint32_t wl;
    if constexpr (std::is_same_v<N, Nb>)
        wl = nb.wl;
    else
        wl = lane_from_west(c);
    const uint32_t w1 = __builtin_amdgcn_alignbit(c, wl, 31);  // cell x-1 onto x
    const uint32_t w2 = __builtin_amdgcn_alignbit(c, wl, 30);  // cell x-2 onto x
    s = GOL_BOP3(w2, w1, c, kXor3);
    cy = GOL_BOP3(w2, w1, c, kMaj);
    ctr = w1;
}

// B3/S23 from three rows' 3-cell sums: S9 = 9-cell sum including the centre cell mc;
// alive next iff S9 == 3, or S9 == 4 and the cell is alive (server/server.go:35-52).
// S9 = o + 2T with T = k + p + 2q (o,k: full adder of the sum bits, p,q: of the carries).
//   o = 1: next iff T == 1, i.e. q = 0 and T != 0, 2;     o = 0: next iff mc and T in {0, 2}
//   (T == 0 with mc alive cannot happen: mc is part of S9).
// With u = [T in {0,2}] and v = o ? !q : mc this is next = v & (o ^ u): 7 v_bitop3 per word,
// u and v independent (found by exhaustive search over 3-gate circuits on o,k,p,q,mc).
__device__ __forceinline__ uint32_t life_next(uint32_t as, uint32_t acy, uint32_t ms,
                                              uint32_t mcy, uint32_t mc, uint32_t bs,
                                              uint32_t bcy) {
    const uint32_t o = GOL_BOP3(as, ms, bs, kXor3);    // S9 bit 0
    const uint32_t k = GOL_BOP3(as, ms, bs, kMaj);     // carry into the twos
    const uint32_t p = GOL_BOP3(acy, mcy, bcy, kXor3);
    const uint32_t q = GOL_BOP3(acy, mcy, bcy, kMaj);
    const uint32_t u = GOL_BOP3(k, p, q, kTwosEven);
    const uint32_t v = GOL_BOP3(o, q, mc, kOddSelect);
    return GOL_BOP3(v, o, u, GOL_TT(a & (b ^ c)));
}

// A row's per-level state: 3-cell sum, carry and the cells themselves.
template <int D>
struct RowState {
    Words<D> s, cy, c;
};

// One level update: `in` is the new row (below), `above`/`mid` the two previous rows of the level.
// Writes the next generation of `mid` to nx and stores `in`'s state into `above` (now free).
// DR: drifting sums (row_sum3_drift); the state keeps the drifted centre cells.
template <int D, bool DR = false, class N = NoNb>
__device__ __forceinline__ void level_update(RowState<D> &above, const RowState<D> &mid,
                                             const Words<D> &in, Words<D> &nx, const N &nb = N{}) {
    Words<D> ns, ncy, nc = in;
    if constexpr (DR) {
        static_assert(D == 1, "drift needs one word per lane");
        row_sum3_drift<N>(in.w[0], ns.w[0], ncy.w[0], nc.w[0], nb);
    } else {
        row_sum3<D>(in, ns, ncy, nb);
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
        nx.w[d] = life_next(above.s.w[d], above.cy.w[d], mid.s.w[d], mid.cy.w[d], mid.c.w[d],
                            ns.w[d], ncy.w[d]);
    above.s = ns;
    above.cy = ncy;
    above.c = nc;
}

template <int D>
__device__ __forceinline__ Words<D> load_words(const uint32_t *p) {
    Words<D> v;
    if constexpr (D == 2) {
        const uint2 t = *reinterpret_cast<const uint2 *>(p);
        v.w[0] = t.x;
        v.w[1] = t.y;
    } else {
        v.w[0] = *p;
    }
    return v;
}

// Raw buffer store of a lane's D words: an offset past the descriptor's range is dropped by the
// hardware, which is how halo lanes and pipeline-fill steps skip their store WITHOUT a branch
// (a branch around the store would make the waitcnt pass count conservatively and shorten the
// load prefetch distance).
constexpr uint32_t kBufferRsrcWord3 = 0x00020000;  // gfx9-family raw buffer, 32-bit dwords
constexpr int kOutOfRange = 0x40000000;
template <int D>
__device__ __forceinline__ void buffer_store_words(__amdgpu_buffer_rsrc_t r, int off,
                                                   const Words<D> &v) {
    if constexpr (D == 2) {
        typedef int v2i __attribute__((ext_vector_type(2)));
        v2i x = {(int)v.w[0], (int)v.w[1]};
        __builtin_amdgcn_raw_buffer_store_b64(x, r, off, 0, 0);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32((int)v.w[0], r, off, 0, 0);
    }
}

template <int... I, class F>
__device__ __forceinline__ void static_for(std::integer_sequence<int, I...>, F &&f) {
    (f(std::integral_constant<int, I>{}), ...);
}

// Level update without the rule: only ingests the new row's 3-cell sums into the ring (pipeline
// fill: the level's output would be garbage, but the rows it holds are needed two steps later).
template <int D, bool DR = false, class N = NoNb>
__device__ __forceinline__ void level_ingest(RowState<D> &above, const Words<D> &in,
                                             const N &nb = N{}) {
    if constexpr (DR) {
        row_sum3_drift<N>(in.w[0], above.s.w[0], above.cy.w[0], above.c.w[0], nb);
    } else {
        row_sum3<D>(in, above.s, above.cy, nb);
        above.c = in;
    }
}

// Output rows [ya, yb) of band `bandi` of a launch (range 0 bands first, then range 1).
// Row indices fit in 32 bits; keeping every loop-carried counter 32-bit keeps the compares on the
// SALU (gfx9 has no 64-bit signed s_cmp, a 64-bit compare would drag them into VGPRs).
__device__ __forceinline__ void band_rows(const StencilParams &p, int64_t bandi, int &ya, int &yb) {
    if (bandi < p.nbands0) {
        if (p.band2 > 0 && bandi >= p.nbig0) {  // graded: the short tail bands
            ya = (int)(p.r0b + p.nbig0 * p.band + (bandi - p.nbig0) * p.band2);
            yb = (int)min((int64_t)ya + p.band2, p.r0e);
        } else {
            ya = (int)(p.r0b + bandi * p.band);
            yb = (int)min((int64_t)ya + p.band, p.r0e);
        }
    } else {
        ya = (int)(p.r1b + (bandi - p.nbands0) * p.band);
        yb = (int)min((int64_t)ya + p.band, p.r1e);
    }
}

// Input row stream of a band: rows ya-K, ya-K+1, ... wrapped mod H (single strip holding the
// torus) or clamped to the halo'd strip [lo, hi).  Branch-free (scalar selects), so the waitcnt
// pass sees one straight line of loads and stores and keeps the full prefetch distance.
struct RowStream {
    int ly, wrap, hi;
    __device__ __forceinline__ RowStream(const StencilParams &p, int first) {
        wrap = (int)p.wrap_rows;
        hi = (int)p.hi;
        const int lo = (int)p.lo;
        ly = first;
        if (wrap > 0) {
            ly %= wrap;
            if (ly < 0) ly += wrap;
        } else {
            ly = ly < lo ? lo : (ly >= hi ? hi - 1 : ly);
        }
    }
    __device__ __forceinline__ void advance() {
        const int nx = ly + 1;
        ly = wrap > 0 ? (nx == wrap ? 0 : nx) : (nx < hi ? nx : hi - 1);
    }
};

// Where a lane stores its (first) word: through at most one of a full store (off_full), the low
// half (off_lo) or the high half (off_hi, HH only); the others point past the buffer descriptor
// and are dropped.  own_mask: the owned cells of the word, for the counts.
struct LaneStore {
    int off_full = kOutOfRange, off_lo = kOutOfRange, off_hi = kOutOfRange;
    uint32_t own_mask = 0;
};
template <bool HH>
__device__ __forceinline__ LaneStore lane_store(int lane, int colraw, int col, int wd) {
    LaneStore o;
    if (HH) {
        // owned unwrapped cells: [-16, 32wd - 16); lane 0 -> upper half, lane 63 -> lower half
        const int last = wd - 1;
        if (lane == 0) {
            if (colraw <= last - 1) { o.off_hi = col * 4 + 2; o.own_mask = 0xffff0000u; }
        } else if (lane == 63) {
            if (colraw <= last) { o.off_lo = col * 4; o.own_mask = 0x0000ffffu; }
        } else if (colraw < last) {
            o.off_full = col * 4; o.own_mask = ~0u;
        } else if (colraw == last) {
            o.off_lo = col * 4; o.own_mask = 0x0000ffffu;
        }
    } else if (lane >= 1 && lane <= 62 && colraw < wd) {
        o.off_full = col * 4;
        o.own_mask = ~0u;
    }
    return o;
}

// PRE geometry (gol_stencil PRE): lanes 1..63 own whole words (63 per wave), lane 0 is halo.
__device__ __forceinline__ LaneStore lane_store_pre(int lane, int colraw, int col, int wd) {
    LaneStore o;
    if (lane >= 1 && colraw < wd) {
        o.off_full = col * 4;
        o.own_mask = ~0u;
    }
    return o;
}

template <int D, bool HH>
__device__ __forceinline__ void store_row(__amdgpu_buffer_rsrc_t r, const LaneStore &ls,
                                          const Words<D> &v, int rowoff) {
    buffer_store_words<D>(r, ls.off_full + rowoff, v);
    if (HH) {
        __builtin_amdgcn_raw_buffer_store_b16((short)v.w[0], r, ls.off_lo + rowoff, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b16((short)(v.w[0] >> 16), r, ls.off_hi + rowoff, 0, 0);
    }
}

// Sum of v over the wave's 64 lanes, returned in lane 63: the DPP prefix-sum ladder (row_shr 1, 2,
// 4, 8 within each 16-lane row, then row_bcast 15 / 31 across rows) -- 6 dependent VALU ops
// instead of 6 dependent ds_bpermute round trips through the LDS pipe.
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111 /* row_shr:1 */, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112 /* row_shr:2 */, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114 /* row_shr:4 */, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118 /* row_shr:8 */, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142 /* row_bcast:15 */, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143 /* row_bcast:31 */, 0xc, 0xf, false);
    return v;
}

// Per-level alive counts of a wave -> its spread slot of each generation (agent-scope atomics,
// issued by lane 63, which holds the wave's sum).
template <int NL>
__device__ __forceinline__ void flush_counts(const uint32_t (&acc)[NL], int j0, int lane,
                                             int64_t wave, unsigned long long *slots) {
    uint32_t v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) v[j] = wave_sum_dpp(acc[j]);
#pragma unroll
    for (int j = 0; j < NL; ++j)
        if (lane == 63 && v[j])
            __hip_atomic_fetch_add(&slots[(j0 + j) * kCountSlots + (int)(wave & (kCountSlots - 1))],
                                   (unsigned long long)v[j], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
}

// The end-of-launch count flush of a register slab: wave w reduces generations w, w + W, ... (G of
// them) -- all G DPP ladders issued together, then the atomics -- instead of one generation after
// another (W = 4 waves of a packed slab own 4 of K = 16 generations each).  part(g) is the lane's
// partial count of generation g (the W waves' LDS slots summed, masked to the counting lanes).
template <int G, class Part>
__device__ __forceinline__ void flush_counts_strided(int w, int W, int K, int lane, int64_t group,
                                                     unsigned long long *slots, Part part) {
    uint32_t v[G];
#pragma unroll
    for (int i = 0; i < G; ++i) v[i] = w + i * W < K ? part(w + i * W) : 0u;
#pragma unroll
    for (int i = 0; i < G; ++i) v[i] = wave_sum_dpp(v[i]);
#pragma unroll
    for (int i = 0; i < G; ++i)
        if (lane == 63 && v[i])
            __hip_atomic_fetch_add(&slots[(w + i * W) * kCountSlots + (int)(group & (kCountSlots - 1))],
                                   (unsigned long long)v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Column geometry of a wave's 64 lanes (shared with the host via chunk_words()):
//   default : lanes 1..62 own D words each, lanes 0 and 63 are the horizontal halo (K <= 32);
//   HH      : (D = 1, K <= 16) a halo needs only K <= 16 bits, so lane 0 owns the upper and lane 63
//             the lower half of its word: 63 words per wave, chunk c owns cells
//             [2016c - 16, 2016(c+1) - 16) (unwrapped), stored as full words plus two halves.
// The hot kernel.  K = generations per launch, D = words per lane.
// SKEW = false: the K levels of one step form one dependent chain (level j+1 consumes the row
//               level j produced in the same step).
// SKEW = true : level j consumes the row level j-1 produced in the PREVIOUS step, so the K level
//               updates of a step are independent (K-way ILP); the pipeline is K-1 steps deeper.
// DR = true: drifting row sums (row_sum3_drift, one cross-lane move per level update instead of
//             two); level j's rows sit j+1 bits east in the lane frame, the stored level-K row is
//             shifted back by one DPP + v_alignbit per stored word, and the per-level count masks
//             follow the drift.  Needs the half-word halo geometry (D = 1, K <= 16, chained).
// ZIP = 2 (chained, LDS-DMA): two consecutive steps run together, level by level -- step st's
//             level j, then step st+1's level j.  The two level chains are independent except
//             that step st+1's level j reads the row sums step st's level j has just ingested, so
//             a wave carries two dependency chains instead of one (the chained kernel is
//             latency-bound: each level's 12 ops form a chain of ~7 and the next level waits for
//             it, with an s_nop before every DPP), at the cost of a second chain's temporaries.
// FILLU = false: the pipeline-fill steps run through the steady loop (garbage levels computed and
//             dropped) instead of being unrolled at compile time -- a smaller code footprint.
// LD = true: also store the last generation's flips (output XOR the generation before it) to
//             p.diff: at the last level the mid row's centre cells are generation K-1 in the same
//             (drifted) frame as the output, so the diff costs one XOR, its realignment and the
//             store(s) per step.
// WPE > 0: minimum resident waves per SIMD forced on the register allocator (the vmcnt guard's
//             self-test instantiates a spilling configuration this way; production: 0).
// PRE = true (drift, LDS-DMA, K <= 16): the input row is shifted K bits WEST as it leaves the
//             ring, so the K generations of eastward drift bring the level-K row back to the board
//             frame: no realignment before the store.  The ring row holds 65 words (the 65th, the
//             first word of the next chunk, comes from a second DMA of the row one word east), so lane 63's
//             shifted word is complete, and after K <= 16 generations only lane 0 has gone stale
//             (2K <= 32 bits from the west edge): 63 whole words per wave with one full-word store
//             per lane -- the half-word halo's width without its two 16-bit stores.  The shift of
//             the row and of its west word (2 v_alignbit, the neighbours read from the ring)
//             replaces the store's realignment (1 DPP + 1 v_alignbit): the same VALU per step.
// MASK = true: lanes no output or count depends on (past the row end in the last column chunk:
//             at 65536 wide its 62-word chunk holds 2 words) run the launch exec-masked off, so
//             they issue nothing into the datapath; the wave's instruction stream is unchanged.
// STAMP = true (tuning build, kVariantStamp): lane 0 of every wave writes its start and end
//             (s_memrealtime, 100 MHz), its shader-clock cycles (s_memtime delta) and its
//             HW_ID / XCC_ID to ((uint64_t *)p.diff)[4 wave ..]: the launch's dispatch skew,
//             wave durations, per-SIMD tails and in-kernel clock (scripts/stamp_launch.py).
template <int K, bool COUNT, bool SKEW, int D, int PF, bool HH, bool DR = false, int ZIP = 1,
          bool FILLU = true, bool LD = false, int WPE = 0, bool PRE = false, bool MASK = false,
          bool STAMP = false>
// (PRE with counts at K = 16 (production): left alone, the allocator spends 224 VGPRs, i.e. 2 waves
// per SIMD; held to the half-word-halo kernel's 3 it needs 142 and no scratch.  At K = 12, 4 waves
// would spill: no hint there.)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    WPE > 0 ? WPE : (ZIP == 2 && !COUNT && K >= 12 && K <= 16 ? 4 : (PRE && COUNT && K >= 14 ? 3 : 1)))))
void gol_stencil(const uint32_t *__restrict__ in,
                                                   uint32_t *__restrict__ out, StencilParams p,
                                                   unsigned long long *__restrict__ slots) {
    static_assert(!HH || (D == 1 && K <= 16), "half-word halo needs D = 1, K <= 16");
    static_assert(!DR || (D == 1 && !SKEW && K <= 32), "drift: one word per lane, chained levels");
    static_assert(ZIP == 1 || (ZIP == 2 && PF == 1 && !SKEW && D == 1), "zip: chained LDS-DMA, D = 1");
    static_assert(!PRE || (D == 1 && DR && !HH && PF == 1 && ZIP == 1 && K <= 16),
                  "pre-shifted rows: drift, one word per lane, LDS-DMA ring, K <= 16");
    const int lane = threadIdx.x & 63;
    // wave index made provably uniform so every band/row quantity lives in SGPRs
    const int64_t wave =
        (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t chunk = wave % p.nchunks;
    const int64_t bandi = wave / p.nchunks;
    if (bandi >= p.nbands) return;  // wave-uniform
    // the split step's boundary bands (p.prio, uniform): issue ahead of the interior's waves on
    // the same SIMD, so the chain bands -> halo exchange -> next bands is not starved
    if (p.prio) __builtin_amdgcn_s_setprio(3);
    uint64_t stamp_t0 = 0, stamp_c0 = 0;
    if constexpr (STAMP) {
        stamp_t0 = __builtin_amdgcn_s_memrealtime();
        stamp_c0 = __builtin_amdgcn_s_memtime();
    }
    int ya, yb;
    band_rows(p, bandi, ya, yb);
    // First word (unwrapped) of this lane and its wrapped column.
    const int stride = (HH || PRE) ? 63 : 62 * D;
    const int colraw = (int)chunk * stride + (lane - 1) * D;
    const int col = (colraw + p.wd) % p.wd;
    RowStream rows(p, ya - K);
    auto load_next = [&]() -> Words<D> {
        const Words<D> v = load_words<D>(in + (int64_t)rows.ly * p.pitch + col);
        rows.advance();
        return v;
    };
    // Output: one raw-buffer descriptor over the band's rows.  Offsets are 32-bit: the host caps
    // band * rowbytes below kOutOfRange = 2^30 (max_band_rows in golhip_engine.hip), so a dropped
    // store's offset kOutOfRange + r * rowbytes neither wraps nor lands inside the band.
    const int rowbytes = (int)(p.pitch * 4);
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)ya * p.pitch, 0, (yb - ya) * rowbytes, kBufferRsrcWord3);
    const LaneStore ls = PRE ? lane_store_pre(lane, colraw, col, p.wd) : lane_store<HH>(lane, colraw, col, p.wd);
    const uint32_t own_mask = ls.own_mask;
    // DR counts need no per-level mask: level j's row sits d = j+1 bits east, so positions
    // [32, 2048) (lanes 1..63 in full) hold cells [2016c - d, 2016(c+1) - d) of chunk c -- windows
    // that tile the row at every level (valid: the drift leaves [2d, 2048) valid, 2d <= 32) -- and
    // the last chunk's window ends at the row end (colraw < wd) for every d.  So every lane counts
    // its whole word and the lanes outside the window drop their sums once, at the flush.
    // Drift with the 62-word geometry (!HH, lanes 1..62 store whole words, K <= 32): positions
    // [64, 2048) (lanes 2..63) hold cells [1984c + 32 - d, 1984(c+1) + 32 - d), valid for 2d <= 64;
    // the last chunk's window ends at cell 32 wd + 32 - d, i.e. at the lane with colraw == wd (the
    // wrapped word 0, whose cells [0, 32 - d) no chunk's first window covers).
    // PRE: level j's row sits d = j + 1 - K <= 0 bits east of the board frame, so lanes 1..63 hold
    // cells [2016c - d, 2016(c+1) - d) (valid: the drift leaves [2(j+1), 2048) valid, 2(j+1) <= 32)
    // and the lanes with colraw < wd end the last chunk's window at the row end plus -d cells: the
    // wrapped cells [0, -d) that chunk 0's window leaves out.
    const bool count_lane = (HH || PRE) ? (lane >= 1 && colraw < p.wd) : (lane >= 2 && colraw <= p.wd);
    // vector-memory stores per step: the output row (3 with the half-word halo), twice with LD
    constexpr int NSTORE = (HH ? 3 : 1) * (LD ? 2 : 1);
    __amdgpu_buffer_rsrc_t drsrc = orsrc;
    if constexpr (LD)
        drsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + (int64_t)ya * p.pitch, 0,
                                                  (yb - ya) * rowbytes, kBufferRsrcWord3);
    // the output row (and, LD, its diff): rowoff kOutOfRange (+ small offsets) drops the stores
    auto store_row = [&](const Words<D> &v, int rowoff, const Words<D> *dv = nullptr) {
        golhip::store_row<D, HH>(orsrc, ls, v, rowoff);
        if constexpr (LD) golhip::store_row<D, HH>(drsrc, ls, dv ? *dv : v, rowoff);
    };
    // the diff of the last level's output nx against its mid row's centre cells (same frame)
    auto last_diff = [&](const Words<D> &nx, const RowState<D> &mid) {
        Words<D> dv;
#pragma unroll
        for (int d = 0; d < D; ++d) dv.w[d] = nx.w[d] ^ mid.c.w[d];
        return dv;
    };

    // Per level: a two-slot ring (X/Y swap roles every step) and, skewed, the pending input row.
    RowState<D> X[K], Y[K];
    Words<D> pend[K];
    uint32_t acc[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            X[j].s.w[d] = X[j].cy.w[d] = X[j].c.w[d] = 0;
            Y[j].s.w[d] = Y[j].cy.w[d] = Y[j].c.w[d] = 0;
            pend[j].w[d] = 0;
        }
        acc[j] = 0;
    }
    const int nrows = yb - ya;
    const int lag = SKEW ? 3 * K - 1 : 2 * K;  // steps before the first stored row
    const int nsteps = nrows + lag;

    // One step: a new level-0 row enters, every level emits one row, the level-K row is stored.
    // PAR 0: above = X, mid = Y, new -> X.  PAR 1: above = Y, mid = X, new -> Y.
    // Chained: level j+1 takes level j's output of this step; level j's output row is
    //   ya - K + st - (j+1), valid from step 2j+2 on (its above/mid rows arrive at steps 2j and
    //   2j+1).  FILL = true (pipeline-fill steps only): level j is skipped before step 2j and only
    //   ingests its input at steps 2j, 2j+1 -- the garbage rows of the fill are never computed.
    // Skewed: levels in descending order, level j takes pend[j] (level j-1's output of the
    //   previous step) and its output overwrites pend[j+1] after level j+1 has read it; level j's
    //   output row is ya - K + st - 1 - 2j.
    auto step = [&](auto par, auto fill, const Words<D> &vin, int st, const auto &nb0) {
        constexpr int PAR = decltype(par)::value;
        constexpr int FST = decltype(fill)::value;  // fill step index (compile time) or -1
        constexpr bool FILL = FST >= 0 && !SKEW;
        Words<D> nc = vin;
#pragma unroll
        for (int jj = 0; jj < K; ++jj) {
            const int j = SKEW ? K - 1 - jj : jj;
            const Words<D> lin = SKEW ? (j == 0 ? vin : pend[j]) : nc;
            if (FILL && FST < 2 * j + 2) {  // folds away: FST and (unrolled) j are constants
                if (FST >= 2 * j) {
                    if (j == 0)
                        level_ingest<D, DR>(PAR == 0 ? X[j] : Y[j], lin, nb0);
                    else
                        level_ingest<D, DR>(PAR == 0 ? X[j] : Y[j], lin);
                }
                if (j == K - 1) store_row(lin, kOutOfRange);  // keep the per-step store count
                continue;
            }
            Words<D> nx;
            if (j == 0)  // level 0 takes the new row with its given neighbours (if any)
                level_update<D, DR>(PAR == 0 ? X[j] : Y[j], PAR == 0 ? Y[j] : X[j], lin, nx, nb0);
            else
                level_update<D, DR>(PAR == 0 ? X[j] : Y[j], PAR == 0 ? Y[j] : X[j], lin, nx);
            Words<D> dv{};
            if (LD && j == K - 1) dv = last_diff(nx, PAR == 0 ? Y[j] : X[j]);
            if (COUNT) {
                const int r = SKEW ? st - K - 1 - 2 * j : st - K - (j + 1);
                const uint32_t m = DR ? ~0u : own_mask;  // DR: whole words, see count_lane
                if (r >= 0 && r < nrows) acc[j] += __builtin_popcount(nx.w[0] & m) +
                                                   (D == 2 ? __builtin_popcount(nx.w[D - 1] & own_mask) : 0);
            }
            if (j == K - 1) {
                const int r = st - lag;  // stored row - ya
                if constexpr (DR && !PRE) {  // back to the board frame: K bits west
                    nx.w[0] = realign_drift<K>(nx.w[0]);
                    if constexpr (LD) dv.w[0] = realign_drift<K>(dv.w[0]);
                }
                store_row(nx, (r >= 0 && r < nrows) ? r * rowbytes : kOutOfRange, &dv);
                if (PF) asm volatile("" ::: "memory");
            } else if (SKEW) {
                pend[j + 1] = nx;
            } else {
                nc = nx;
            }
        }
    };
    using Par0 = std::integral_constant<int, 0>;
    using Par1 = std::integral_constant<int, 1>;
    using Steady = std::integral_constant<int, -1>;
    // One level of one step of the chained kernel (ZIP path): nc = the level's input row, replaced
    // by its output; the same fill rules as `step` (levels before step 2j skipped, steps 2j and
    // 2j+1 ingest only), all decided at compile time.
    auto lvl = [&](auto par, auto fill, auto jc, Words<D> &nc, int st, const auto &nb0) {
        constexpr int PAR = decltype(par)::value;
        constexpr int FST = decltype(fill)::value;
        constexpr int j = decltype(jc)::value;
        RowState<D> &above = PAR == 0 ? X[j] : Y[j];
        const RowState<D> &mid = PAR == 0 ? Y[j] : X[j];
        if constexpr (FST >= 0 && FST < 2 * j + 2) {
            if constexpr (FST >= 2 * j) {
                if constexpr (j == 0)
                    level_ingest<D, DR>(above, nc, nb0);
                else
                    level_ingest<D, DR>(above, nc);
            }
            if constexpr (j == K - 1) {
                store_row(nc, kOutOfRange);  // keep the per-step store count
                asm volatile("" ::: "memory");
            }
        } else {
            Words<D> nx;
            if constexpr (j == 0)
                level_update<D, DR>(above, mid, nc, nx, nb0);
            else
                level_update<D, DR>(above, mid, nc, nx);
            Words<D> dv{};
            if constexpr (LD && j == K - 1) dv = last_diff(nx, mid);
            if (COUNT) {
                const int r = st - K - (j + 1);
                const uint32_t m = DR ? ~0u : own_mask;  // DR: whole words, see count_lane
                if (r >= 0 && r < nrows) acc[j] += __builtin_popcount(nx.w[0] & m);
            }
            if constexpr (j == K - 1) {
                const int r = st - lag;
                if constexpr (DR) {
                    nx.w[0] = realign_drift<K>(nx.w[0]);
                    if constexpr (LD) dv.w[0] = realign_drift<K>(dv.w[0]);
                }
                store_row(nx, (r >= 0 && r < nrows) ? r * rowbytes : kOutOfRange, &dv);
                asm volatile("" ::: "memory");
            }
            nc = nx;
        }
    };
    // Steps st (even: PAR 0) and st+1 (PAR 1) level by level.
    auto step2 = [&](auto fill0, auto fill1, Words<D> nc0, Words<D> nc1, int st, const auto &nb0a,
                     const auto &nb0b) {
        static_for(std::make_integer_sequence<int, K>{}, [&](auto jc) {
            lvl(Par0{}, fill0, jc, nc0, st, nb0a);
            lvl(Par1{}, fill1, jc, nc1, st + 1, nb0b);
        });
    };

    // MASK: the lanes any stored or counted word depends on -- the west halo lane, the owned and
    // counted lanes, and (62-word drift) the lane with colraw == wd, whose word is the east
    // neighbour of the last owned one and holds the wrapped count window
    const bool live = !MASK || lane == 0 || (PRE ? colraw < p.wd : colraw <= p.wd);
    if (live) {
    if constexpr (PF == 0) {
        // Register prefetch ring: loads run P steps ahead of their use (deeper for small K,
        // whose steps are short and would otherwise expose HBM latency).
        constexpr int P = K >= 4 ? 4 : (K == 2 ? 8 : 16);
        Words<D> buf[P];
#pragma unroll
        for (int u = 0; u < P; ++u) buf[u] = load_next();
        for (int s = 0; s < nsteps; s += P) {
#pragma unroll
            for (int u = 0; u < P; ++u) {
                const Words<D> vin = buf[u];
                buf[u] = load_next();
                if (u & 1)
                    step(Par1{}, Steady{}, vin, s + u, NoNb{});
                else
                    step(Par0{}, Steady{}, vin, s + u, NoNb{});
            }
        }
    } else {
        // LDS ring filled by LDS-DMA (global_load_lds): no VGPR destination, so the prefetch
        // distance costs no registers and no register moves.  A row chunk is D DMAs of 64
        // consecutive words (lane L of DMA i fetches word base + 64i + L), read back as the
        // lane's D consecutive words.  PL slots, PL-1 rows in flight: step st reads slot
        // st % PL and refills the slot step st-1 read, AFTER an lgkmcnt(0) wait -- a DMA's LDS
        // write is not ordered with this wave's earlier ds_reads, so a slot is only refilled once
        // its reads have returned.  Each step waits (by hand: the compiler does not track LDS-DMA
        // completion) until its row's DMAs have landed: a step issues D DMAs and NSTORE stores,
        // so after the last DMA for step st-(PL-1) this wave issued NSTORE stores of that step and
        // (D + NSTORE) ops for each of the PL-2 steps after it; the wait leaves a margin of 2.
        // Deeper ring for K <= 2: steps are short, the launch is HBM-bound and needs more bytes
        // in flight per CU.
        // PRE: NDMA = 2 DMAs per row (the row's 64 words and the 65th word)
        constexpr int NDMA = D + (PRE ? 1 : 0);
        constexpr int PL = (K <= 2 && NSTORE + (NDMA + NSTORE) * 14 - 2 <= 63) ? 16 : 8;
        constexpr int kWait = NSTORE + (NDMA + NSTORE) * (PL - 2) - 2;
        static_assert(kWait <= 63, "vmcnt field");
        __shared__ __attribute__((aligned(16))) uint32_t ring[4][PL][64 * D + (PRE ? 4 : 0)];
        const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
        const int nb_w = max(lane * D - 1, 0), nb_e = min(lane * D + D, 64 * D - 1);
        int dcol4[D];  // byte offset of lane L's word of DMA i in the row
        int dcol65 = 0;  // PRE: lane L's word of the second DMA (word L + 1 of the ring row)
        {
            const int base = (int)chunk * stride - D;
#pragma unroll
            for (int i = 0; i < D; ++i) dcol4[i] = ((base + 64 * i + lane + p.wd) % p.wd) * 4;
            if constexpr (PRE) dcol65 = ((base + 1 + lane + p.wd) % p.wd) * 4;
        }
        // Compiler-level fences (empty asm with a memory clobber) keep every DMA and store in
        // program order, so the per-step vmcnt accounting holds whatever the scheduler does.
        // The DMA is a raw-buffer load to LDS over ONE row (descriptor built on the SALU per
        // row): the per-lane operand is a 32-bit byte offset instead of a 64-bit address, one
        // VGPR and one 64-bit VALU add per row fewer than global_load_lds.
        auto dma_next = [&](int slot) {
            const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint32_t *>(in + (int64_t)rows.ly * p.pitch), 0, rowbytes,
                kBufferRsrcWord3);
#pragma unroll
            for (int i = 0; i < D; ++i) {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, &ring[w][slot][64 * i], 4, dcol4[i], 0, 0, 0);
                asm volatile("" ::: "memory");
            }
            if constexpr (PRE) {
                // the 65th word: the same row once more, one word east, into ring[1..64] -- lanes
                // 0..62 rewrite the words the first DMA puts there (same values: the order of the
                // two LDS writes does not matter), lane 63 adds word 64.  A whole-wave DMA: a
                // lane-0-only one made the compiler wrap it in exec-mask branches every step
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, &ring[w][slot][1], 4, dcol65, 0, 0, 0);
                asm volatile("" ::: "memory");
            }
            rows.advance();
        };
        Words<D> zero;
#pragma unroll
        for (int d = 0; d < D; ++d) zero.w[d] = 0;
        if constexpr (ZIP == 2) {
            // Steps in pairs.  A pair waits for its two rows, refills the two slots the previous
            // pair read (their ds_reads returned: lgkmcnt(0)) with the rows PL-2 and PL-1 steps
            // ahead, reads its rows and runs step2.  VMEM ops per pair: 2 DMAs + 2 NSTORE stores;
            // row st+1's DMA was the second DMA of the pair PL/2 - 1 pairs back, after which that
            // pair's 2 NSTORE stores and (2 + 2 NSTORE) ops of each of the PL/2 - 2 pairs between
            // were issued; the wait leaves a margin of 2.
            constexpr int kWait2 = 2 * NSTORE + (2 + 2 * NSTORE) * (PL / 2 - 2) - 2;
            static_assert(kWait2 <= 63 && PL % 2 == 0, "vmcnt field, whole pairs per ring");
#pragma unroll
            for (int q = 0; q < PL / 2 - 1; ++q) {  // rows 0 .. PL-3 in (DMA, DMA, stores) pairs
                dma_next(2 * q);
                dma_next(2 * q + 1);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    store_row(zero, kOutOfRange + 16 * q + 8 * i);
                    asm volatile("" ::: "memory");
                }
            }
            auto pair = [&](int u, auto fill0, auto fill1, int st) {
                asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(kWait2) : "memory");
                dma_next((u + PL - 2) % PL);
                dma_next((u + PL - 1) % PL);
                Words<D> v0, v1;
                v0.w[0] = ring[w][u][lane];
                v1.w[0] = ring[w][u + 1][lane];
                const Nb nba{ring[w][u][nb_w], ring[w][u][nb_e]};
                const Nb nbb{ring[w][u + 1][nb_w], ring[w][u + 1][nb_e]};
                step2(fill0, fill1, v0, v1, st, nba, nbb);
            };
            // pipeline fill (2K steps, rounded up to whole rings), unrolled: every level's
            // skip / ingest-only / full decision is a compile-time constant
            constexpr int FILL = (2 * K + PL - 1) / PL * PL;
            static_for(std::make_integer_sequence<int, FILL / 2>{}, [&](auto qc) {
                constexpr int ST = 2 * decltype(qc)::value;
                pair(ST % PL, std::integral_constant<int, ST>{}, std::integral_constant<int, ST + 1>{}, ST);
            });
            for (int s = FILL; s < nsteps; s += PL) {
#pragma unroll
                for (int u = 0; u < PL; u += 2) pair(u, Steady{}, Steady{}, s + u);
            }
        } else {
#pragma unroll
            for (int u = 0; u < PL - 1; ++u) {
                dma_next(u);
                // dummy (dropped) stores keep the (DMA, stores) cadence; distinct offsets so no
                // dead-store elimination merges them
                store_row(zero, kOutOfRange + 8 * u);
                asm volatile("" ::: "memory");
            }
            auto one_step = [&](int u, auto fill, int st) {
                asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(kWait) : "memory");
                dma_next((u + PL - 1) % PL);
                Words<D> vin;
#pragma unroll
                for (int d = 0; d < D; ++d) vin.w[d] = ring[w][u][lane * D + d];
                // level 0's neighbour words straight from the ring (the row's lanes -1 / +1; the
                // edge lanes read a clamped, garbage word: they are halo, as with DPP)
                Nb nb0{ring[w][u][nb_w], ring[w][u][nb_e]};
                if constexpr (PRE) {  // the row and its west word, K bits west (lane 63: word 65)
                    const uint32_t xe = ring[w][u][lane + 1];
                    nb0.wl = __builtin_amdgcn_alignbit(vin.w[0], nb0.wl, K);
                    vin.w[0] = __builtin_amdgcn_alignbit(xe, vin.w[0], K);
                }
                if (st & 1)
                    step(Par1{}, fill, vin, st, nb0);
                else
                    step(Par0{}, fill, vin, st, nb0);
            };
            int s = 0;
            // Pipeline fill of the chained levels (2K steps, rounded up to whole rings so the main
            // loop stays slot-aligned), fully unrolled so every level's skip / ingest-only / full
            // decision is a compile-time constant: no branches, no extra registers.
            if constexpr (!SKEW && FILLU) {
                constexpr int FILL = (2 * K + PL - 1) / PL * PL;
                static_for(std::make_integer_sequence<int, FILL>{}, [&](auto stc) {
                    constexpr int ST = decltype(stc)::value;
                    one_step(ST % PL, stc, ST);
                });
                s = FILL;
            }
            for (; s < nsteps; s += PL) {
#pragma unroll
                for (int u = 0; u < PL; ++u) one_step(u, Steady{}, s + u);
            }
        }
        // Drain the ring's in-flight DMAs before the wave can retire: a DMA landing after the
        // workgroup released its LDS would write into the next workgroup's ring.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    }  // live

    if (COUNT) {
        if (DR && !count_lane) {
#pragma unroll
            for (int j = 0; j < K; ++j) acc[j] = 0;
        }
        flush_counts<K>(acc, 0, lane, wave, slots);
    }
    if constexpr (STAMP) {
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
        const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
        const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
        if (lane == 0 && p.diff != nullptr) {  // no buffer (split boards, graphs): no stamps
            uint64_t *st = reinterpret_cast<uint64_t *>(p.diff) + 4 * wave;
            st[0] = stamp_t0;
            st[1] = t1;
            st[2] = c1 - stamp_c0;
            st[3] = (uint64_t)hw | ((uint64_t)xcc << 32);
        }
    }
}

// ---------------------------------------------------------------- one generation (K = 1)
// K = 1 is HBM-bound (0.25 B per cell update against ~13 VALU per 32 cells), so it gets its own
// memory-shaped kernel: a lane holds 4 consecutive words (one 16-byte load / store per row, 1 KiB
// per wave instruction), a wave covers 256 words with NO halo lanes (one generation needs only
// the single bit beyond each edge: lanes 0 and 63 load the word outside the wave as a 4-byte side
// load, which DPP with bound_ctrl off leaves in place at the wave edge), so 65536-wide rows tile
// into exactly 8 waves.  Rows stream through a register ring P rows deep; the row sums of the
// row above and of the middle row stay in registers.  Lanes past the torus width hold the
// wrapped words (the torus continuation), so partial last chunks need no special case; they
// just do not store.
// P = rows in flight per wave; NT bit 0 / bit 1 = non-temporal loads / stores (streamed once).
template <bool COUNT, int P = 8, int NT = 0, bool LD = false>
__global__ __launch_bounds__(256) void gol_step1(const uint32_t *__restrict__ in,
                                                 uint32_t *__restrict__ out, StencilParams p,
                                                 unsigned long long *__restrict__ slots) {
    const int lane = threadIdx.x & 63;
    const int64_t wave =
        (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t chunk = wave % p.nchunks, bandi = wave / p.nchunks;
    if (bandi >= p.nbands) return;
    int ya, yb;
    band_rows(p, bandi, ya, yb);
    const int base = (int)chunk * 256;
    const int colraw = base + lane * 4;  // unwrapped index of the lane's first word
    const int col = colraw % p.wd;       // wd % 4 == 0: the 4 words never straddle the wrap
    // side word: west of the wave (lane 0), east of it (lane 63); other lanes reload their own
    // first word (same cache line, no extra traffic) so the load needs no branch
    const int xcol = lane == 0 ? (base - 1 + p.wd) % p.wd : lane == 63 ? (base + 256) % p.wd : col;
    const int nrows = yb - ya, nsteps = nrows + 2;
    const int rowbytes = (int)(p.pitch * 4);
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)ya * p.pitch, 0, (yb - ya) * rowbytes, kBufferRsrcWord3);
    const bool owned = colraw < p.wd;
    const int off = owned ? col * 4 : kOutOfRange;
    __amdgpu_buffer_rsrc_t drsrc = orsrc;  // LD: the generation's flips beside the output
    if constexpr (LD)
        drsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + (int64_t)ya * p.pitch, 0,
                                                  (yb - ya) * rowbytes, kBufferRsrcWord3);

    RowStream rows(p, ya - 1);
    uint4 buf[P];
    uint32_t xbuf[P];
    auto load_next = [&](int u) {
        const uint32_t *r = in + (int64_t)rows.ly * p.pitch;
        if constexpr (NT & 1) {
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(r + col));
            buf[u] = make_uint4(t.x, t.y, t.z, t.w);
            xbuf[u] = __builtin_nontemporal_load(r + xcol);
        } else {
            buf[u] = *reinterpret_cast<const uint4 *>(r + col);
            xbuf[u] = r[xcol];
        }
        rows.advance();
    };
#pragma unroll
    for (int u = 0; u < P; ++u) load_next(u);

    Words<4> as, acy, ms, mcy, mc;  // row sums of the row above and of the middle row + its cells
#pragma unroll
    for (int d = 0; d < 4; ++d) as.w[d] = acy.w[d] = ms.w[d] = mcy.w[d] = mc.w[d] = 0;
    uint32_t acc = 0;
    for (int s = 0; s < nsteps; s += P) {
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int st = s + u;
            Words<4> c;
            c.w[0] = buf[u].x;
            c.w[1] = buf[u].y;
            c.w[2] = buf[u].z;
            c.w[3] = buf[u].w;
            const uint32_t x = xbuf[u];
            load_next(u);
            // neighbour words: lane L-1's last word / lane L+1's first word; at the wave edges the
            // source lane does not exist and the side word x stays (bound_ctrl off keeps `old`)
            const Nb nb{(uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)c.w[3], 0x138, 0xf, 0xf, false),
                        (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)c.w[0], 0x130, 0xf, 0xf, false)};
            Words<4> bs, bcy;
            row_sum3<4>(c, bs, bcy, nb);
            Words<4> nx;
#pragma unroll
            for (int d = 0; d < 4; ++d)
                nx.w[d] = life_next(as.w[d], acy.w[d], ms.w[d], mcy.w[d], mc.w[d], bs.w[d], bcy.w[d]);
            const int r = st - 2;  // the middle row, relative to ya
            const bool live = r >= 0 && r < nrows;
            typedef int v4i __attribute__((ext_vector_type(4)));
            const v4i v = {(int)nx.w[0], (int)nx.w[1], (int)nx.w[2], (int)nx.w[3]};
            __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, off + (live ? r * rowbytes : kOutOfRange), 0,
                                                   (NT & 2) ? 2 /* nt */ : 0);
            if constexpr (LD) {
                const v4i dv = {(int)(nx.w[0] ^ mc.w[0]), (int)(nx.w[1] ^ mc.w[1]),
                                (int)(nx.w[2] ^ mc.w[2]), (int)(nx.w[3] ^ mc.w[3])};
                __builtin_amdgcn_raw_buffer_store_b128(dv, drsrc, off + (live ? r * rowbytes : kOutOfRange),
                                                       0, (NT & 2) ? 2 : 0);
            }
            if (COUNT && live && owned)
                acc += __builtin_popcount(nx.w[0]) + __builtin_popcount(nx.w[1]) +
                       __builtin_popcount(nx.w[2]) + __builtin_popcount(nx.w[3]);
            as = ms;
            acy = mcy;
            ms = bs;
            mcy = bcy;
            mc = c;
        }
    }
    if (COUNT) {
        const uint32_t a[1] = {acc};
        flush_counts<1>(a, 0, lane, wave, slots);
    }
}

// ---------------------------------------------------------------- level-split stencil
// Small boards are latency-bound: a round of minimal bands gives fewer waves than SIMDs, and a
// lone wave's time is its dependent chain -- band*K level updates (+ the fill), K levels deep
// per step.  gol_stencil_split spreads the K levels of one (band, chunk) over a workgroup of S
// waves: wave R computes levels [R*K/S, (R+1)*K/S) and hands its last level's output row to wave
// R+1 through LDS; the group steps in lockstep (one s_barrier per step), so every wave's chain is
// K/S levels and the board runs S times as many waves, with no extra (halo) work.
// Wave R's level j outputs row ya - K + st - (j+1) - R at step st (one step of delay per hand-off),
// valid from step 2j + 2 + R; the final row (j = K-1, R = S-1) lags by 2K + S - 1 steps.
template <int K, bool COUNT, int S, int R, bool LD = false>
__device__ __forceinline__ void split_role(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                           const StencilParams &p,
                                           unsigned long long *__restrict__ slots, int64_t group,
                                           int lane, uint32_t (*xring)[2][64],
                                           uint32_t (*ring)[64]) {
    constexpr bool HH = K <= 16;
    constexpr bool DR = HH;                 // drifting row sums (see gol_stencil)
    constexpr int NL = K / S, J0 = R * NL;  // this wave's levels: [J0, J0 + NL)
    constexpr int PL = 8;                   // LDS-DMA ring depth (wave 0)
    constexpr int LAG = 2 * K + S - 1;
    constexpr int FILL = (LAG + PL - 1) / PL * PL;  // unrolled fill steps (ring-aligned)
    const int64_t chunk = group % p.nchunks, bandi = group / p.nchunks;
    int ya, yb;
    band_rows(p, bandi, ya, yb);
    const int colraw = (int)chunk * split_chunk_words(K) + lane - 1;  // HH: 63 words per chunk
    const int col = (colraw + p.wd) % p.wd;
    const int nrows = yb - ya, nsteps = nrows + LAG;
    const int rowbytes = (int)(p.pitch * 4);
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)ya * p.pitch, 0, (yb - ya) * rowbytes, kBufferRsrcWord3);
    const LaneStore ls = lane_store<HH>(lane, colraw, col, p.wd);
    __amdgpu_buffer_rsrc_t drsrc = orsrc;  // LD: the last generation's flips beside the output
    if constexpr (LD)
        drsrc = __builtin_amdgcn_make_buffer_rsrc(p.diff + (int64_t)ya * p.pitch, 0,
                                                  (yb - ya) * rowbytes, kBufferRsrcWord3);
    uint32_t midc = 0;  // LD: the step's last-level output XOR its mid row's centre cells
    const bool count_lane = lane >= 1 && colraw < p.wd;  // DR count window (see gol_stencil)
    RowStream rows(p, ya - K);

    RowState<1> X[NL], Y[NL];
    uint32_t acc[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        X[j].s.w[0] = X[j].cy.w[0] = X[j].c.w[0] = 0;
        Y[j].s.w[0] = Y[j].cy.w[0] = Y[j].c.w[0] = 0;
        acc[j] = 0;
    }
    auto dma_next = [&](int slot) {
        __builtin_amdgcn_global_load_lds(in + (int64_t)rows.ly * p.pitch + col, &ring[slot][0], 4, 0, 0);
        asm volatile("" ::: "memory");
        rows.advance();
    };
    if (R == 0) {
#pragma unroll
        for (int u = 0; u < PL - 1; ++u) dma_next(u);
    }
    // One lockstep step: take the input row (DMA ring or the previous wave's hand-off), run this
    // wave's levels (compile-time fill guards when FST >= 0), hand off or store, barrier.
    auto step = [&](auto par, auto fill, int u, int st) {
        constexpr int PAR = decltype(par)::value;
        constexpr int FST = decltype(fill)::value;
        Words<1> nc;
        if (R == 0) {
            // PL-1 rows in flight: this slot's DMA has PL-2 younger ones (margin of 2); refill
            // the slot the previous step read (its read returned before that step's barrier)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PL - 2 - 2) : "memory");
            dma_next((u + PL - 1) % PL);
            nc.w[0] = ring[u][lane];
        } else {
            nc.w[0] = xring[R - 1][(st - 1) & 1][lane];
        }
#pragma unroll
        for (int jl = 0; jl < NL; ++jl) {
            const int j = J0 + jl;
            if (FST >= 0 && FST < 2 * j + 2 + R) {  // folds away: FST and (unrolled) j constant
                if (FST >= 2 * j + R) level_ingest<1, DR>(PAR == 0 ? X[jl] : Y[jl], nc);
                nc.w[0] = 0;
                continue;
            }
            Words<1> nx;
            if (PAR == 0)
                level_update<1, DR>(X[jl], Y[jl], nc, nx);
            else
                level_update<1, DR>(Y[jl], X[jl], nc, nx);
            if (LD && R == S - 1 && jl == NL - 1)  // last level: the generation before, same frame
                midc = nx.w[0] ^ (PAR == 0 ? Y[jl] : X[jl]).c.w[0];
            if (COUNT) {
                const int rr = st - K - (j + 1) - R;
                const uint32_t m = DR ? ~0u : ls.own_mask;
                if (rr >= 0 && rr < nrows) acc[jl] += __builtin_popcount(nx.w[0] & m);
            }
            nc = nx;
        }
        if (R < S - 1) {
            xring[R][st & 1][lane] = nc.w[0];
        } else {
            const int rr = st - LAG;
            if constexpr (DR) {  // back to the board frame: K bits west
                nc.w[0] = realign_drift<K>(nc.w[0]);
                if constexpr (LD) midc = realign_drift<K>(midc);
            }
            store_row<1, HH>(orsrc, ls, nc, (rr >= 0 && rr < nrows) ? rr * rowbytes : kOutOfRange);
            if constexpr (LD) {
                Words<1> dv;
                dv.w[0] = midc;
                store_row<1, HH>(drsrc, ls, dv, (rr >= 0 && rr < nrows) ? rr * rowbytes : kOutOfRange);
            }
        }
        // hand-off visible to the next wave, and this step's reads done before slots are reused
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    using Par0 = std::integral_constant<int, 0>;
    using Par1 = std::integral_constant<int, 1>;
    static_for(std::make_integer_sequence<int, FILL>{}, [&](auto stc) {
        constexpr int ST = decltype(stc)::value;
        if (ST & 1)
            step(Par1{}, stc, ST % PL, ST);
        else
            step(Par0{}, stc, ST % PL, ST);
    });
    for (int s = FILL; s < nsteps; s += PL) {
#pragma unroll
        for (int u = 0; u < PL; ++u) {
            if (u & 1)
                step(Par1{}, std::integral_constant<int, -1>{}, u, s + u);
            else
                step(Par0{}, std::integral_constant<int, -1>{}, u, s + u);
        }
    }
    if (R == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the ring
    if (COUNT) {
        if (DR && !count_lane) {
#pragma unroll
            for (int j = 0; j < NL; ++j) acc[j] = 0;
        }
        flush_counts<NL>(acc, J0, lane, group, slots);
    }
}

template <int K, bool COUNT, int S, bool LD = false>
__global__ __launch_bounds__(64 * S) void gol_stencil_split(const uint32_t *__restrict__ in,
                                                            uint32_t *__restrict__ out,
                                                            StencilParams p,
                                                            unsigned long long *__restrict__ slots) {
    static_assert(S >= 2 && K % S == 0, "levels split evenly over S >= 2 waves");
    __shared__ __attribute__((aligned(16))) uint32_t xring[S - 1][2][64];
    __shared__ __attribute__((aligned(16))) uint32_t ring[8][64];
    const int64_t group = blockIdx.x;
    if (group / p.nchunks >= p.nbands) return;  // whole workgroup
    const int lane = threadIdx.x & 63;
    const int r = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    static_for(std::make_integer_sequence<int, S>{}, [&](auto rc) {
        constexpr int RR = decltype(rc)::value;
        if (r == RR) split_role<K, COUNT, S, RR, LD>(in, out, p, slots, group, lane, xring, ring);
    });
}
template <int K, int D>
constexpr bool kHalfHalo = D == 1 && K <= 16;  // keep in sync with chunk_words()

template <int P, int NT>
hipError_t launch_step1_cfg(const uint32_t *in, uint32_t *out, const StencilParams &p,
                            unsigned long long *slots, hipStream_t s) {
    const unsigned blocks = (unsigned)std::max<int64_t>(1, (p.nbands * (int64_t)p.nchunks + 3) / 4);
    if (p.diff && slots)
        hipLaunchKernelGGL((gol_step1<true, P, NT, true>), dim3(blocks), dim3(256), 0, s, in, out, p, slots);
    else if (p.diff)
        hipLaunchKernelGGL((gol_step1<false, P, NT, true>), dim3(blocks), dim3(256), 0, s, in, out, p, slots);
    else if (slots)
        hipLaunchKernelGGL((gol_step1<true, P, NT>), dim3(blocks), dim3(256), 0, s, in, out, p, slots);
    else
        hipLaunchKernelGGL((gol_step1<false, P, NT>), dim3(blocks), dim3(256), 0, s, in, out, p, slots);
    return hipGetLastError();
}
// Production gol_step1: 4 rows in flight, non-temporal stores (profiles/r01_tune_step1.txt).  The
// tuning library can register other prefetch depths / cache policies (GOLHIP_STEP1).
inline hipError_t launch_step1(const uint32_t *in, uint32_t *out, const StencilParams &p,
                               unsigned long long *slots, hipStream_t s) {
    if (const auto f = kernel_extras().step1) return f(in, out, p, slots, s);
    return launch_step1_cfg<4, 2>(in, out, p, slots, s);
}
inline const void *step1_fn() {
    if (const auto f = kernel_extras().step1_fn) return f();
    return (const void *)gol_step1<false, 4, 2>;
}

template <int K, bool SKEW, int D, int PF = 0, bool DR = false, int ZIP = 1, bool HH = kHalfHalo<K, D>,
          bool FILLU = true, bool ALLOW_LD = false, bool PRE = false, bool MASK = false, bool STAMP = false>
hipError_t launch_stencil_k(const uint32_t *in, uint32_t *out, const StencilParams &p,
                            unsigned long long *slots, hipStream_t s) {
    const int64_t waves = p.nbands * (int64_t)p.nchunks;
    // at least one block: an empty launch (nbands = 0, every wave returns at once) is how
    // warm_stencil_k loads this depth's code object before anything is timed
    const unsigned blocks = (unsigned)std::max<int64_t>(1, (waves + 3) / 4);
    if constexpr (STAMP) {  // p.diff is the stamp buffer (no flips in this variant)
        if (slots)
            hipLaunchKernelGGL((gol_stencil<K, true, SKEW, D, PF, HH, DR, ZIP, FILLU, false, 0, PRE, MASK, true>),
                               dim3(blocks), dim3(256), lds_pad_bytes(), s, in, out, p, slots);
        else
            hipLaunchKernelGGL((gol_stencil<K, false, SKEW, D, PF, HH, DR, ZIP, FILLU, false, 0, PRE, MASK, true>),
                               dim3(blocks), dim3(256), lds_pad_bytes(), s, in, out, p, slots);
        return hipGetLastError();
    }
    if (p.diff) {  // last-generation flips beside the output (production variants only)
        if constexpr (ALLOW_LD) {
            if (slots)
                hipLaunchKernelGGL((gol_stencil<K, true, SKEW, D, PF, HH, DR, ZIP, FILLU, true, 0, PRE, MASK>),
                                   dim3(blocks), dim3(256), lds_pad_bytes(), s, in, out, p, slots);
            else
                hipLaunchKernelGGL((gol_stencil<K, false, SKEW, D, PF, HH, DR, ZIP, FILLU, true, 0, PRE, MASK>),
                                   dim3(blocks), dim3(256), lds_pad_bytes(), s, in, out, p, slots);
            return hipGetLastError();
        } else {
            return hipErrorNotSupported;
        }
    }
    if (slots)
        hipLaunchKernelGGL((gol_stencil<K, true, SKEW, D, PF, HH, DR, ZIP, FILLU, false, 0, PRE, MASK>), dim3(blocks), dim3(256),
                           lds_pad_bytes(), s, in, out, p, slots);
    else
        hipLaunchKernelGGL((gol_stencil<K, false, SKEW, D, PF, HH, DR, ZIP, FILLU, false, 0, PRE, MASK>), dim3(blocks), dim3(256),
                           lds_pad_bytes(), s, in, out, p, slots);
    return hipGetLastError();
}

// The production kernel of depth K (kVariantProd): gol_step1 at K = 1; the drifting-sum stencil
// with the column geometry measured fastest per depth and counting mode (prod_pre, internal.hpp).
template <int K>
hipError_t launch_prod(const uint32_t *in, uint32_t *out, const StencilParams &p,
                       unsigned long long *slots, hipStream_t s) {
    if constexpr (K == 1) return launch_step1(in, out, p, slots, s);
    else if constexpr (K <= 16) {
        if (prod_pre(K, slots != nullptr))
            return launch_stencil_k<K, false, 1, 1, true, 1, false, true, true, true>(in, out, p, slots, s);
        return launch_stencil_k<K, false, 1, 1, true, 1, false, true, true>(in, out, p, slots, s);
    } else return launch_stencil_k<K, false, 1, 1, true, 1, false, true, true>(in, out, p, slots, s);
}
template <int K>
const void *prod_fn() {
    if constexpr (K == 1) return step1_fn();
    else if constexpr (prod_pre(K)) return (const void *)gol_stencil<K, false, false, 1, 1, false, true, 1, true, false, 0, true>;
    else return (const void *)gol_stencil<K, false, false, 1, 1, false, true, 1>;
}


template <int K, int S>
hipError_t launch_split_ks(const uint32_t *in, uint32_t *out, const StencilParams &p,
                           unsigned long long *slots, hipStream_t s) {
    const unsigned blocks = (unsigned)(p.nbands * (int64_t)p.nchunks);
    if (blocks == 0) return hipSuccess;
    if (p.diff && slots)
        hipLaunchKernelGGL((gol_stencil_split<K, true, S, true>), dim3(blocks), dim3(64 * S), 0, s,
                           in, out, p, slots);
    else if (p.diff)
        hipLaunchKernelGGL((gol_stencil_split<K, false, S, true>), dim3(blocks), dim3(64 * S), 0, s,
                           in, out, p, slots);
    else if (slots)
        hipLaunchKernelGGL((gol_stencil_split<K, true, S>), dim3(blocks), dim3(64 * S), 0, s, in,
                           out, p, slots);
    else
        hipLaunchKernelGGL((gol_stencil_split<K, false, S>), dim3(blocks), dim3(64 * S), 0, s, in,
                           out, p, slots);
    return hipGetLastError();
}

}  // namespace

// Defines the production launcher of depth K (launch_stencil_k<K> / stencil_fn_k<K> /
// warm_stencil_k<K>, declared in golhip_internal.hpp) in the TU that includes this header for one
// depth.
#define GOLHIP_DEFINE_STENCIL_K(K)                                                            \
    hipError_t launch_stencil_k##K(const uint32_t *in, uint32_t *out, const StencilParams &p, \
                                   unsigned long long *slots, hipStream_t s) {                \
        return launch_prod<K>(in, out, p, slots, s);                                          \
    }                                                                                          \
    const void *stencil_fn_k##K() { return prod_fn<K>(); }                                     \
    hipError_t warm_stencil_k##K(hipStream_t s) {                                              \
        StencilParams p{};                                                                      \
        p.nchunks = 1; /* nbands = 0: every wave returns at once */                            \
        return launch_prod<K>(nullptr, nullptr, p, nullptr, s);                                 \
    }

}  // namespace golhip
