// engine_plan.hip -- the launch planner: launch depths, wave bands, and which kernel a board runs.
//
// Reference role: server/server.go:77-107 (GolOP.Work splits a strip's rows over req.Threads
// goroutines, one turn per RPC).  Here a call of n turns becomes a sequence of K-generation launches
// (temporal blocking) whose grid is sized to the chip's wave slots, or captured graph replays on
// boards too small to fill the chip.
#include <algorithm>
#include <cmath>

#include "golhip_engine.hpp"

namespace golhip {

int64_t strip_plan_rows(int64_t height, int strips) { return (height + strips - 1) / strips; }

// Largest supported launch depth <= n.
int pick_k(int n) {
    int kk = 1;
    for (int c : {32, 24, 20, 16, 14, 12, 10, 8, 6, 4, 2, 1})  // 24 / 20: tuning library only
        if (c <= n && stencil_k_supported(c)) {
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
double launch_rate_tcups(int K, double cells) {
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
        if (stencil_k_supported(K) && launch_rate_tcups(K, cells) > launch_rate_tcups(best, cells))
            best = K;
    return best;
}

// Register-slab boards: a slab launch is latency-bound (a chain of barrier-bound generations plus a
// ~3 us launch boundary, about the same at any depth), so the tail takes the fewest launches: the
// largest depth of the slab kernels' {16, 12, 8, 4, 2, 1} that fits.
int slab_first_k(int64_t n, int kmax) {
    for (int K : {16, 12, 8, 4, 2})
        if (K <= n && K <= kmax && stencil_k_supported(K)) return K;
    return 1;
}

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
            if (K > m || K > kmax || !stencil_k_supported(K)) continue;
            const double c = best[m - K] + cells * K / (launch_rate_tcups(K, cells) * 1e6) + kLaunchOverheadUs;
            if (c < best[m]) {
                best[m] = c;
                first[m] = K;
            }
        }
    return first[N];
}

static int device_cus(golhip_t h) {
    if (h->cus == 0) {
        hipDeviceProp_t prop;
        h->cus = hipGetDeviceProperties(&prop, h->shards[0].device) == hipSuccess ? prop.multiProcessorCount
                                                                                   : 256;
    }
    return h->cus;
}

// Rows per wave band of a stencil launch over rows_total rows.  reserve_waves: resident wave
// slots to leave free for a concurrent launch (the boundary bands of a split board).
int64_t auto_band(golhip_t h, int64_t rows_total, int K, int64_t reserve_waves, bool counting) {
    if (h->band_rows > 0) return h->band_rows;
    const int64_t per = chunk_words(K, h->variant, counting);
    const int64_t nchunks = (h->wd + per - 1) / per;
    // Fill the chip in whole rounds of resident waves (CUs x resident waves per CU), so every
    // SIMD gets the same number of equal bands.
    const int cus = device_cus(h);
    int &wpc = h->waves_per_cu[K][h->variant];
    if (wpc == 0) wpc = stencil_waves_per_cu(K, h->variant);
    // The one-generation kernel (K = 1, production variant) is HBM-bound: it runs best with 2
    // long-streaming waves per SIMD in one round (measured: 2/SIMD 21.9, 4/SIMD 21.1, 1/SIMD
    // 19.6 TCUPS at 65536^2; uneven rounds lose 10-20 %, profiles/r01_tune_step1.txt).
    const bool step1 = K == 1 && variant_is_production_family(h->variant);
    const int64_t capacity = (int64_t)cus * (step1 ? kStep1WavesPerCu : wpc);
    constexpr int64_t kMaxBand = 4096;
    const bool skew = h->variant == kVariantSkew || h->variant == kVariantSkewD2 ||
                      h->variant == kVariantSkewLdsPf || h->variant == kVariantSkewLdsD2;
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
        const int64_t simds = 4 * (int64_t)cus;  // gfx9: 4 SIMDs per CU
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
// GOLHIP_SPLIT=1/2/4/8 (tuning library) forces it.  The production library has no level-split
// kernel (stencil_split_supported is false there), so this is 1 in production.
int pick_split(golhip_t h, int64_t rows_total, int K) {
    if (!variant_is_production_family(h->variant)) return 1;
    if (h->force_split > 0)
        return h->force_split > 1 && stencil_split_supported(K, h->force_split) ? h->force_split : 1;
    // measured (profiles/r01_tune_small.txt): a gain at K = 16 (-10 % per turn at 5120^2), none
    // at K = 12 and a loss at K = 8, where the lockstep barriers cost more than the shorter chain
    if (K < 16) return 1;
    const int64_t per = chunk_words(K, h->variant);
    const int64_t nchunks = (h->wd + per - 1) / per;
    const int64_t minband = std::max(K, 8);
    const int64_t waves1 = (rows_total + minband - 1) / minband * nchunks;
    int &wpc = h->waves_per_cu[K][h->variant];
    if (wpc == 0) wpc = stencil_waves_per_cu(K, h->variant);
    const int64_t capacity = (int64_t)h->cus * wpc;  // 0 until a planner call has read the device
    // S = 8 (two levels per wave at K = 16) on the boards that fit S = 4 in one round: its waves
    // are light (few VGPRs), so up to two rounds' worth: 5120^2 with counts 1.70 -> 1.58 us per
    // turn, 4096^2 1.49 -> 1.35 (profiles/r01_tune_small_split8.txt)
    if (stencil_split_supported(K, 8) && waves1 * 8 <= 2 * capacity) return 8;
    for (int S : {4, 2})
        if (stencil_split_supported(K, S) && waves1 * S <= capacity) return S;
    return 1;
}

// The register kernels for boards too small for the streaming kernel (stencil_tile.hpp): gol_tile
// (one wave per T + 2K row tile) and gol_slab (a workgroup of W waves x S rows, edge rows through
// LDS).  They replace the streaming band's pipeline fill (2K rows per band, one dependency chain
// per wave) by a K-row trapezoid per tile/slab with every row of a generation independent; they
// win where the streaming kernel cannot get both tall bands and enough waves (small boards;
// profiles/r02/small_boards.txt).
RegKernel pick_reg_kernel(golhip_t h, int64_t rows_total, int K, bool counting) {
    RegKernel rk;
    if (!variant_is_production_family(h->variant) || h->split) return rk;
    // an explicit level split or band height (tests, tuning) asks for the streaming kernels
    const bool forced = h->force_tile > 0 || h->force_slab > 0;
    if (!forced && (h->force_split > 0 || h->band_rows > 0)) return rk;
    // the input descriptor spans the board's rows; offsets are 32-bit signed
    if ((int64_t)h->height * h->pitch * 4 >= ((int64_t)1 << 31)) return rk;
    if (h->force_tile > 0) {
        if (stencil_tile_supported(K, h->force_tile)) rk.kind = 2, rk.T = h->force_tile;
        return rk;
    }
    if (h->force_slab > 0) {  // [NC x 10000 +] W x 100 + S
        const int NC = h->force_slab >= 10000 ? h->force_slab / 10000 : 4;
        const int W = h->force_slab / 100 % 100, S = h->force_slab % 100;
        // NC = 14 (gol_slabp): P = 64 / (wd + 2) segments of S rows per wave, boards of <= 62 words
        const int P = NC == 14 ? (h->wd <= 62 ? (int)(64 / (h->wd + 2)) : 0) : 1;
        if (P > 0 && W * P * S - 2 * K >= 1 && stencil_slab_supported(K, W, S, NC))
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
    const int cus = device_cus(h);
    const int64_t per = chunk_words(K, h->variant, counting);
    const int64_t nchunks = (h->wd + per - 1) / per;
    const int64_t minband = std::max(K, 8);
    const int64_t waves1 = (rows_total + minband - 1) / minband * nchunks;
    if (waves1 > kSlabMaxWaves1PerCu * (int64_t)cus) return rk;
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
    if ((K == 16 || K == 12 || K == 8 || K == 4 || K == 2) && h->wd <= 30) {  // round 5: also the tail depths
        const int P = (int)(64 / (h->wd + 2));
        for (const int W : {4, 6, 8}) {
            const int T = W * P * 3 - 2 * K;
            if (T < 1 || !stencil_slab_supported(K, W, 3, 14)) continue;
            rk.kind = 3, rk.W = W, rk.S = 3, rk.NC = 14, rk.T = T;
            if ((rows_total + T - 1) / T <= cus) break;
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
    // Round 5: 16 x 4 (T = 32, 16 rows per SIMD) for boards whose 16 x 4 slabs fit one round over
    // the CUs, e.g. two-chunk widths at 4096 rows: 3968 x 4096 with every count 0.706 (12 x 7,
    // 158 slabs) -> 0.583 us/turn (256 slabs), without counts 0.659 -> 0.543; 12 x 6 0.652, 16 x 5
    // 0.654 (profiles/r05/r05y_rows_per_cu_ab.log).  The rows-per-SIMD model orders all four; 16 x 4
    // is a candidate only in one round (larger boards keep the taller slabs' lower halo share).
    // Round 6: 12 x 4 (T = 16, 12 rows per SIMD) under the same one-round rule: 2048^2 with every
    // count 0.503 against 16 x 4's 0.556 us/turn (profiles/r05/r05zc_t16_slabs_ab.log; without
    // counts: profiles/r06/).
    static constexpr Cand kCount16[] = {{16, 6, 12}, {8, 12, 9}, {12, 8, 12}, {12, 7, 12}, {16, 4, 12}, {12, 4, 12}};
    static constexpr Cand kPlain16[] = {{16, 6, 9}, {12, 8, 9}, {8, 12, 9}, {12, 7, 9}, {16, 4, 9}, {12, 4, 9}};
    static constexpr Cand kOther[] = {{8, 8, 4}};
    const Cand *cands = K == 16 ? (counting ? kCount16 : kPlain16) : kOther;
    const int ncand = K == 16 ? 6 : 1;
    double best = 1e300;
    for (int i = 0; i < ncand; ++i) {
        const Cand c = cands[i];
        if (!stencil_slab_supported(K, c.W, c.S, c.NC)) continue;
        const int64_t T = (int64_t)c.W * c.S - 2 * K;
        if (T < 1) continue;
        const int64_t slabs = (rows_total + T - 1) / T * ((h->wd + kTileChunkWords - 1) / kTileChunkWords);
        const int64_t rounds = (slabs + cus - 1) / cus;
        if (c.S == 4 && rounds > 1) continue;  // 16 x 4, 12 x 4: measured in one round only
        const double cost = (double)rounds * (double)((c.W + 3) / 4) * c.S;
        if (cost < best) {  // ties keep the earlier (measured-preferred) shape
            best = cost;
            rk.kind = 3, rk.W = c.W, rk.S = c.S, rk.NC = c.NC, rk.T = (int)T;
        }
    }
    return rk;
}

bool board_applies(golhip_t h, int *W, int *R) {
    // the production kernel family only, and no forced kernel or band (tests, tuning)
    if (!h->board_kernel || h->split || h->shards.size() != 1 || h->variant != kVariantProd) return false;
    if (h->force_split > 0 || h->force_tile >= 0 || h->force_slab >= 0 || h->band_rows > 0) return false;
    // golhip_set_fixed_k: every launch exactly k deep (depth sweeps measure the stencil kernels at
    // that depth; the whole-board kernel is not a k-deep launch)
    if (h->fixed_k) return false;
    if (h->board_kernel < 0 && h->height > kBoardAutoRows) return false;
    return stencil_board_shape(h->height, h->wd, W, R);
}

// Largest band the kernels' 32-bit store offsets can address: a band's output descriptor spans
// band * rowbytes bytes, and dropped stores use offset kOutOfRange (2^30) + row * rowbytes, so
// band * rowbytes must stay below 2^30 (golhip_kernels.hip, buffer_store_words).  At 262144 wide
// that is 32767 rows; only --band-rows / very wide boards can reach it.
static int64_t max_band_rows(golhip_t h) {
    const int64_t rowbytes = h->pitch * 4;
    return std::max<int64_t>(1, ((int64_t)1 << 30) / rowbytes - 1);
}

// Launch the K-generation stencil described by p (the register kernels or the level-split kernel
// when the board asks for them).
// Stable-slab skipping applies to a slab launch when: enabled, a production gol_slab2 shape, no flips,
// the whole torus in one strip (bands wrap), and full bands at least K rows tall (the kernel checks
// the slabs within K rows: the adjacent bands, and one more beyond the short last band).
static bool activity_applies(golhip_t h, const RegKernel &rk, const StencilParams &q, int K) {
    if (!h->activity || h->split || q.diff || q.diff_stride > 0 || q.r1e > q.r1b || q.wrap_rows <= 0) return false;
    if (rk.kind != 3 || !stencil_slab_activity(K, rk.W, rk.S, rk.NC)) return false;
    // automatic: only boards with more slabs than CUs.  With one slab per CU a launch lasts as long
    // as its slowest computed slab, so skipped slabs save nothing and the flags cost ~8 %
    // (profiles/r05/r05l_act_probe.log)
    if (h->activity < 0 && q.nbands * (int64_t)q.nchunks <= std::max(h->cus, 1)) return false;
    const int64_t rows = q.r0e - q.r0b;
    return q.r0b == 0 && rows == q.wrap_rows && q.band >= K && K <= 16;
}

// the slab launch's params (band = T rows, one slab per band and 62-word chunk)
static StencilParams slab_params(golhip_t h, const StencilParams &p, int T) {
    StencilParams q = p;
    q.band = T;
    q.band2 = q.nbig0 = 0;
    q.nbands0 = (p.r0e - p.r0b + T - 1) / T;
    q.nbands = q.nbands0 + (p.r1e - p.r1b + T - 1) / T;
    q.nchunks = (int32_t)((h->wd + kTileChunkWords - 1) / kTileChunkWords);
    return q;
}

int ensure_activity(golhip_t h, Shard &s, int K, bool counting) {
    const RegKernel rk = pick_reg_kernel(h, s.rows, K, counting);
    if (!rk.kind || !h->activity) return GOLHIP_OK;
    const StencilParams q = slab_params(h, make_params(h, s, K, 0, s.rows, 0, 0, 0, counting), rk.out_rows());
    const int64_t need = q.nbands * (int64_t)q.nchunks;
    if (!activity_applies(h, rk, q, K) || need <= s.act_cap) return GOLHIP_OK;
    HIPCHK(h, hipSetDevice(s.device));
    SYNCCHK(h, s.compute);
    if (s.act) HIPCHK(h, hipFree(s.act));
    s.act = nullptr;
    s.act_cap = 0;
    HIPCHK(h, hipMalloc(&s.act, sizeof(uint32_t) * kActWords * (size_t)need));
    HIPCHK(h, hipMemsetAsync(s.act, 0, sizeof(uint32_t) * kActWords * (size_t)need, s.compute));
    if (!s.act_stats) {
        HIPCHK(h, hipMalloc(&s.act_stats, sizeof(unsigned long long) * 2 * kActStatSlots));
        HIPCHK(h, hipMemsetAsync(s.act_stats, 0, sizeof(unsigned long long) * 2 * kActStatSlots, s.compute));
    }
    s.act_cap = need;
    h->act_valid = false;
    return GOLHIP_OK;
}

hipError_t launch_auto(golhip_t h, int K, const uint32_t *in, uint32_t *out, const StencilParams &p,
                       unsigned long long *slots, hipStream_t s, Shard *sh, int par, bool act_reset_first) {
    const int64_t rows_total = (p.r0e - p.r0b) + (p.r1e - p.r1b);
    if (const RegKernel rk = pick_reg_kernel(h, rows_total, K, slots != nullptr); rk.kind) {
        StencilParams q = slab_params(h, p, rk.out_rows());
        // the flags' geometry: band rows, bands, chunks, and waves per slab (pop is per wave)
        const int64_t key[3] = {rk.out_rows() * 64 + rk.W, q.nbands, q.nchunks};
        if (sh && sh->act && activity_applies(h, rk, q, K) && q.nbands * (int64_t)q.nchunks <= sh->act_cap) {
            q.act = sh->act;
            q.act_stats = sh->act_stats;
            q.act_par = par;
            q.act_reset = act_reset_first || !h->act_valid || !std::equal(key, key + 3, h->act_key);
            h->act_valid = true;
            std::copy(key, key + 3, h->act_key);
        } else {
            h->act_valid = false;
        }
        return rk.kind == 2 ? launch_stencil_tile(K, q.band, in, out, q, slots, s)
                            : launch_stencil_slab(K, rk.W, rk.S, rk.NC, in, out, q, slots, s);
    }
    h->act_valid = false;
    const int S = pick_split(h, rows_total, K);
    if (S > 1) {
        // the level-split kernel has its own column geometry (half-word halo for K <= 16)
        StencilParams q = p;
        if (q.band2 > 0) {  // uniform bands for the level-split kernel
            q.band2 = q.nbig0 = 0;
            q.nbands0 = (p.r0e - p.r0b + p.band - 1) / p.band;
            q.nbands = q.nbands0 + (p.r1e - p.r1b + p.band - 1) / p.band;
        }
        const int per = split_chunk_words(K);
        q.nchunks = (int32_t)((h->wd + per - 1) / per);
        return launch_stencil_split(K, S, in, out, q, slots, s);
    }
    return launch_stencil(K, h->variant, in, out, p, slots, s);
}

// counting: the launch writes per-generation counts (its kernel, hence its column geometry,
// can differ: chunk_words / prod_pre)
StencilParams make_params(golhip_t h, const Shard &s, int K, int64_t r0b, int64_t r0e, int64_t r1b,
                          int64_t r1e, int64_t reserve_waves, bool counting) {
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
    const int per = chunk_words(K, h->variant, counting);
    p.nchunks = (h->wd + per - 1) / per;
    return p;
}

// Graphs pay off when a launch is short (launch-bound): < ~100 us of stencil work.
bool small_board(double cells, int K) { return cells * K <= 8e9; }

// k: the maximum depth; Kfull: the deepest depth used (graph replays), pick_k(k) unless the
// streaming kernel's bulk depth is capped; Kbulk: the bulk depth of long runs without graphs.
// stream: the board runs the streaming kernel (no register slab/tile, no level split): its graph
// replays use the best-rate depth too (16384^2: 64.5 vs 55.3 TCUPS at K = 12 vs 16,
// profiles/r02/r02ae_depth_by_size.txt); the register kernels are tuned at the full depth.
LaunchPlanner::LaunchPlanner(double cells_, int k, int64_t turns, bool small, bool fixed, bool keep_last_,
                             int window, bool stream, bool reg_)
    : cells(cells_),
      Kfull(small && stream && !fixed ? best_rate_k(pick_k(k), cells_) : pick_k(k)),
      left(turns),
      keep_last(keep_last_) {
    reg = reg_;
    M = std::max(2, (kGraphGens / Kfull) & ~1);
    Mbig = std::max(M, (std::min(kGraphGensBig, window) / Kfull) & ~1);
    graphs = small && turns >= (int64_t)M * Kfull + (keep_last ? 1 : 0);
    Kbulk = small || fixed ? Kfull : best_rate_k(Kfull, cells);
}

int LaunchPlanner::next() {
    for (int m : {Mbig, M})
        if (graphs && left >= (int64_t)m * Kfull + (keep_last ? 1 : 0)) {
            left -= (int64_t)m * Kfull;
            last_M = m;
            return 0;
        }
    const int K = left >= 2 * (int64_t)Kbulk ? Kbulk : reg ? slab_first_k(left, Kfull) : plan_first_k(left, Kfull, cells);
    left -= K;
    return K;
}

}  // namespace golhip

using namespace golhip;

// ================================================================================ C ABI ====
extern "C" {

int golhip_launch_kind(golhip_t h, int k, int *kind, int *param) {
    return golhip_launch_kind_counts(h, k, 0, kind, param);
}

int golhip_launch_kind_counts(golhip_t h, int k, int counting, int *kind, int *param) {
    if (!h || !kind || !param || k < 1 || k > kMaxK) return GOLHIP_ERR_ARG;
    *kind = 0;
    *param = 0;
    if (h->split) return GOLHIP_OK;  // strips: the streaming kernel around the halo exchange
    if (int W = 0, R = 0; board_applies(h, &W, &R)) {  // the whole board in one workgroup
        *kind = 4;
        *param = W * 100 + R;
        return GOLHIP_OK;
    }
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
    if (width <= 0 || height <= 0 || strips <= 0 || k < 1 || k > kMaxK || turns < 0 || !n)
        return GOLHIP_ERR_ARG;
    const double cells = (double)lcm64(width, 128) * (double)height;
    const double strip_cells = (double)lcm64(width, 128) * (double)strip_plan_rows(height, strips);
    const int Kfull = pick_k(k);
    // the engine's automatic choice for one strip: the register slab where the streaming kernel
    // would have at most kSlabMaxWaves1PerCu minimal-band waves per CU (256 CUs), else streaming
    // (pick_reg_kernel)
    const int64_t wd = lcm64(width, 128) / 32;
    const int64_t per = chunk_words(Kfull, kVariantProd);
    const int64_t waves1 = (height + std::max(Kfull, 8) - 1) / std::max(Kfull, 8) * ((wd + per - 1) / per);
    const bool stream = strips > 1 ||
                        !stencil_slab_supported(Kfull, 8, Kfull == 16 ? 12 : 8, Kfull == 16 ? 9 : 4) ||
                        waves1 > kSlabMaxWaves1PerCu * 256;
    size_t cnt = 0;
    if (strips == 1 && height <= kBoardAutoRows && stencil_board_shape(height, (int32_t)wd, nullptr, nullptr)) {
        // the whole-board kernel: one launch per kBoardMaxK generations (of the count window)
        for (int64_t left = turns; left > 0; left -= kBoardMaxK) {
            if (depths && cnt < cap) depths[cnt] = (int32_t)std::min<int64_t>(left, kBoardMaxK);
            ++cnt;
        }
        *n = cnt;
        return cnt > cap && depths ? GOLHIP_ERR_CAP : GOLHIP_OK;
    }
    LaunchPlanner plan(strip_cells, k, turns, strips == 1 && small_board(cells, Kfull), !stream, false,
                       4096, stream, !stream);  // a register-slab board: full depth, fewest launches (run_steps)
    while (plan.left > 0) {
        const int K = plan.next();
        if (depths && cnt < cap) depths[cnt] = K == 0 ? -(plan.last_M * plan.Kfull) : K;
        ++cnt;
    }
    *n = cnt;
    return cnt > cap && depths ? GOLHIP_ERR_CAP : GOLHIP_OK;
}

}  // extern "C"
