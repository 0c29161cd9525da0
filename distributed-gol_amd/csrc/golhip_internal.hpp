// golhip_internal.hpp -- launch-side interface between the engine (golhip_engine.hip) and the
// gfx950 kernels (golhip_kernels.hip).  Not part of the public ABI (include/golhip.h is).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstddef>

namespace golhip {

// Two libraries from the same production sources (Makefile):
//   lib/libgolhip.so         production: only the kernels the automatic planner runs (the
//                            production drift stencil at every depth, gol_step1, the production
//                            register-slab shapes); no tuning environment variable is read;
//   lib_tuning/libgolhip.so  the same objects PLUS the tuning-only translation units under
//                            csrc/tuning/: the measured-and-rejected stencil variants, the
//                            level-split and register-tile kernels, the other slab shapes, the
//                            timestamping kernels, the fault-injection hooks and the environment
//                            selectors of the A/B scripts.  Those TUs register themselves in
//                            kernel_extras() (below) / engine_hooks() (golhip_engine.hpp) when the
//                            library loads; the production sources never name the tuning build.

// Device layout of one row strip (see DESIGN.md "Data layout in HBM"):
//   torus width L = lcm(width, 128) bits, wd = L/32 uint32 words per row, LSB-first
//   (bit b of word j is x = 32j+b; identical bytes to LSB-first uint64 words), rows
//   contiguous at `pitch` words; `halo` extra rows above row 0 and below the last row.

// Stencil launch: output rows [r0b, r0e) and [r1b, r1e) (second range may be empty) of the
// strip after K generations, computed from the input strip.
// StencilParams::act layout (uint32 offsets for G slabs): changed[par] at 4 G par (16 bytes per
// slab), same at 8 G, pop at 9 G (16 per slab); kActWords * G in all.
constexpr int kActWords = 25;
__host__ __device__ inline int64_t act_chg_off(int par, int64_t G) { return 4 * G * par; }
__host__ __device__ inline int64_t act_same_off(int64_t G) { return 8 * G; }
__host__ __device__ inline int64_t act_pop_off(int64_t G) { return 9 * G; }
constexpr int kActStatSlots = 64;  // StencilParams::act_stats: [computed x 64][skipped x 64]

struct StencilParams {
    int64_t pitch;       // words between consecutive rows
    int64_t r0b, r0e;    // output range 0
    int64_t r1b, r1e;    // output range 1 (r1b == r1e: none)
    int64_t band;        // output rows per wave band
    // > 0: range 0 is nbig0 bands of `band` rows, then bands of band2 rows (shorter: the last
    // dispatched waves are short, so the launch's tail is short -- graded bands)
    int64_t band2, nbig0;
    int64_t nbands0;     // bands in range 0
    int64_t nbands;      // bands in total
    int64_t wrap_rows;   // > 0: single strip holding the whole torus height (row index mod H)
    int64_t lo, hi;      // halo mode: readable input rows [lo, hi) relative to row 0
    int32_t wd;          // words per row of the torus
    int32_t nchunks;     // column chunks per row (chunk_words() words each)
    // 1: the waves raise their issue priority (s_setprio 3) -- the split step's boundary bands,
    // a few dozen waves on the critical path that share SIMDs with the interior's (gol_stencil)
    int32_t prio;
    // nullable: row 0 of a board (same pitch and rows) that receives the XOR of the output
    // generation with the one before it -- the cells the launch's last generation flipped
    // (gol/distributor.go:53-59), written beside the output rows (no extra pass)
    uint32_t *diff;
    // > 0 (gol_slab only; golhip_step_flips): EVERY generation g (0-based) of the launch writes its
    // flips to diff + g * diff_stride words (consecutive slots of the per-turn flips ring)
    int64_t diff_stride;
    // null in production; the tuning library's stamp handles: gol_slab2's per-wave phase stamps,
    // 8 uint64 per wave (golhip_tuning_stamps_ex, scripts/slab_stamps.py)
    uint64_t *stamp;
    // Stable-slab skipping (gol_slab2 ACT, single-strip torus boards; null: off).  act holds, per slab
    // (workgroup) g of G = nbands * nchunks (offsets: act_*_off below, kActWords * G uint32 in all):
    // changed[2] -- 16 bytes per slab, byte w: did wave w's output rows change in the last generation
    // of the launch that wrote them (this launch reads changed[act_par], writes changed[act_par ^ 1]);
    // same -- both ping-pong buffers hold the slab's output region identically; pop -- 16 uint32
    // per slab, wave w's alive cells at that last generation.  Per-wave entries written with plain
    // stores: one shared flag per slab took an OR / add atomic from every wave (+11 % kernel time on
    // dense boards, profiles/r05/r05n_act_ablation.log).  act_reset: the flags are stale (a new
    // board, another kernel or slab shape ran): every slab computes and rewrites them.
    // act_stats (nullable): slabs computed / skipped, spread over kActStatSlots uint64 each (slot
    // group % kActStatSlots: one shared counter serialised ~10 ns per workgroup at L2).
    uint32_t *act;
    unsigned long long *act_stats;
    int32_t act_par, act_reset;
};

constexpr int kMaxK = 32;         // generations per launch limit (halo lane = 32 bits)
constexpr int kCountSlots = 64;   // per-generation count slots (spread the atomics)

// Stencil variants: levels of a step as one dependent chain or skewed across steps (K-way ILP),
// with 1 or 2 words (32 / 64 cells) per lane.
constexpr int kVariantSkew = 0;
constexpr int kVariantChain = 1;
constexpr int kVariantSkewD2 = 2;
constexpr int kVariantChainD2 = 3;
constexpr int kVariantSkewLdsPf = 4;   // input rows prefetched by LDS-DMA instead of VGPRs
constexpr int kVariantChainLdsPf = 5;
constexpr int kVariantSkewLdsD2 = 6;   // LDS-DMA ring, 2 words (64 cells) per lane
constexpr int kVariantChainLdsD2 = 7;
constexpr int kVariantDriftLds = 8;    // chained LDS-DMA levels with drifting row sums (K <= 16)
constexpr int kVariantDriftZip = 9;    // drift, 62-word chunks, two steps interleaved (ZIP = 2)
constexpr int kVariantDrift62 = 10;    // drift, 62-word chunks (one whole-word store per step)
constexpr int kVariantDriftNoFill = 11;  // driftlds without the compile-time unrolled fill
// Production: drifting sums at every depth, with the chunk geometry measured fastest per depth:
// at K = 16 the pre-shifted 63-word rows (PRE, below; round 3: +2.9 % at 65536^2 and +3.0 % at
// 262144^2 over the half-word halo, pre-heated lockstep A/B, profiles/r03/r03p_ab_*.log), 62-word
// chunks (one store per step) at every other K >= 2 (PRE measured equal at K = 12, +0.6 % at 8;
// profiles/r02/tune_depth_geometry.txt for the earlier geometries); gol_step1 at K = 1.
constexpr int kVariantProd = 12;
// drift with the input rows pre-shifted K bits west (gol_stencil PRE): 63-word chunks, one whole-word
// store per step, no store realignment (K <= 16; drift62 above)
constexpr int kVariantPre63 = 13;
// production with the lanes of the last column chunk that nothing depends on exec-masked off
constexpr int kVariantProdMask = 14;
// production with per-wave timestamps (tuning build: dispatch skew, wave durations, per-SIMD
// tails and the in-kernel clock of a launch; golhip_tuning_stamps)
constexpr int kVariantStamp = 15;
constexpr int kNumVariants = 16;
// The pre-shifted geometry in production: every non-counting launch of depth 2..16 (the driver's
// dense 20-turn region, pre-heated: +1.2 % over the 62-word chunks, profiles/r03/r03aa_ab_split.log;
// K = 16 +2.9 %), and counting launches at K = 16 only (with counts at K < 16 its allocator holds
// 168 VGPRs, 3 waves per SIMD, against the 62-word kernel's 110 and 4).
constexpr bool prod_pre(int K, bool counting = false) { return K == 16 || (!counting && K >= 2 && K < 16); }
// Variants of the production family: gol_step1 at K = 1, the level-split kernel for small boards.
inline bool variant_is_production_family(int v) {
    return v == kVariantChainLdsPf || v == kVariantDriftLds || v == kVariantDriftZip ||
           v == kVariantDrift62 || v == kVariantDriftNoFill || v == kVariantProd || v == kVariantPre63 ||
           v == kVariantProdMask || v == kVariantStamp;
}
inline int variant_words(int v) {
    return (v == kVariantSkewD2 || v == kVariantChainD2 || v == kVariantSkewLdsD2 ||
            v == kVariantChainLdsD2)
               ? 2
               : 1;
}
// Words of a row owned by one wave of the stencil (its column chunk): 62 lanes x D words, or 63
// words with the half-word halo (D = 1, K <= 16: lanes 0 and 63 own half a word each).
constexpr int kStep1WavesPerCu = 8;  // gol_step1 grid: resident waves per CU it is sized for
inline int chunk_words(int K, int variant, bool counting = false) {
    if (K == 1 && variant_is_production_family(variant))
        return 256;  // gol_step1: 4 words x 64 lanes
    const int d = variant_words(variant);
    if (variant == kVariantDriftZip || variant == kVariantDrift62) return 62;
    if (variant == kVariantProd || variant == kVariantProdMask || variant == kVariantStamp)
        return prod_pre(K, counting) ? 63 : 62;
    if (variant == kVariantPre63) return K <= 16 ? 63 : 62;
    return (d == 1 && K <= 16) ? 63 : 62 * d;
}

// Production launch depths, one translation unit each (stencil_k<K>.hip).  The tuning library adds
// K = 20 / 24 through kernel_extras().
#define GOLHIP_STENCIL_DEPTHS(X) X(1) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(32)
#define GOLHIP_X(K)                                                                           \
    hipError_t launch_stencil_k##K(const uint32_t *in, uint32_t *out, const StencilParams &p, \
                                   unsigned long long *slots, hipStream_t s);                \
    const void *stencil_fn_k##K();                                                            \
    hipError_t warm_stencil_k##K(hipStream_t s);
GOLHIP_STENCIL_DEPTHS(GOLHIP_X)
#undef GOLHIP_X

// Kernels beyond the production set.  Empty in the production library; the tuning library's
// TUs (csrc/tuning/) fill it from static initialisers when the library loads.  Every dispatcher
// asks the production kernels first and falls back to an entry here (a null entry: the kernel is
// not in this library).
using StencilLaunchFn = hipError_t (*)(int variant, const uint32_t *in, uint32_t *out,
                                       const StencilParams &p, unsigned long long *slots,
                                       hipStream_t s);
struct KernelExtras {
    // per depth: every kernel variant of that depth (the tuning variants, and the depths
    // production lacks: K = 20 / 24); fn / warm as stencil_fn_k / warm_stencil_k
    StencilLaunchFn stencil[kMaxK + 1] = {};
    const void *(*stencil_fn[kMaxK + 1])(int variant) = {};
    hipError_t (*stencil_warm[kMaxK + 1])(int variant, hipStream_t s) = {};
    // gol_step1 configurations other than the production one (GOLHIP_STEP1); null: production
    hipError_t (*step1)(const uint32_t *in, uint32_t *out, const StencilParams &p,
                        unsigned long long *slots, hipStream_t s) = nullptr;
    const void *(*step1_fn)() = nullptr;
    // the level-split kernel, the register tiles, the slab shapes and slab variants production
    // lacks
    bool (*split_supported)(int K, int S) = nullptr;
    hipError_t (*split)(int K, int S, const uint32_t *in, uint32_t *out, const StencilParams &p,
                        unsigned long long *slots, hipStream_t s) = nullptr;
    hipError_t (*split_warm)(hipStream_t s) = nullptr;
    bool (*tile_supported)(int K, int T) = nullptr;
    hipError_t (*tile)(int K, int T, const uint32_t *in, uint32_t *out, const StencilParams &p,
                       unsigned long long *slots, hipStream_t s) = nullptr;
    bool (*slab_supported)(int K, int W, int S, int NC) = nullptr;
    // also every slab launch with p.stamp set (the timestamping slab kernels)
    hipError_t (*slab)(int K, int W, int S, int NC, const uint32_t *in, uint32_t *out,
                       const StencilParams &p, unsigned long long *slots, hipStream_t s) = nullptr;
    // bytes of unused dynamic LDS per stencil block (GOLHIP_LDS_PAD: caps resident blocks per CU)
    size_t lds_pad = 0;
};
KernelExtras &kernel_extras();

// Unused dynamic LDS per stencil block: 0 in production.
inline size_t lds_pad_bytes() { return kernel_extras().lds_pad; }

// Launch the K-generation stencil (a production depth, or one kernel_extras() adds). count_slots (nullable) receives
// per-generation alive counts in kCountSlots slots per generation.
hipError_t launch_stencil(int K, int variant, const uint32_t *in_row0, uint32_t *out_row0,
                          const StencilParams &p, unsigned long long *count_slots,
                          hipStream_t s);
bool stencil_k_supported(int K);
// Load every stencil code object (one per depth TU + the level-split TU) with empty launches, so
// no code-object load lands inside a timed or latency-sensitive step.
hipError_t warm_stencils(int variant, hipStream_t s);
hipError_t warm_stencil_split(hipStream_t s);
// Level-split stencil (small boards): the K levels of a (band, chunk) over a workgroup of S waves
// (S = 2 or 4, D = 1, LDS-DMA input, chained levels; same geometry as kVariantChainLdsPf).
hipError_t launch_stencil_split(int K, int S, const uint32_t *in_row0, uint32_t *out_row0,
                                const StencilParams &p, unsigned long long *count_slots,
                                hipStream_t s);
bool stencil_split_supported(int K, int S);
// Register-tile stencil (small boards, stencil_tile.hip): each wave holds T + 2K rows of a 62-word
// column chunk in VGPRs and runs the K generations over them in place; T output rows per wave.
hipError_t launch_stencil_tile(int K, int T, const uint32_t *in_row0, uint32_t *out_row0,
                               const StencilParams &p, unsigned long long *count_slots,
                               hipStream_t s);
bool stencil_tile_supported(int K, int T);
// Register slab (stencil_tile.hip): a workgroup of W waves, S rows each, edge rows swapped through
// LDS every generation; T = W*S - 2K output rows per workgroup.
// NC: independent row chains per wave (segments advanced op-major).
hipError_t launch_stencil_slab(int K, int W, int S, int NC, const uint32_t *in_row0, uint32_t *out_row0,
                               const StencilParams &p, unsigned long long *count_slots,
                               hipStream_t s);
bool stencil_slab_supported(int K, int W, int S, int NC = 4);
// the slab shapes that can write EVERY generation's flips (StencilParams::diff_stride > 0): the
// production shapes pick_reg_kernel chooses
bool stencil_slab_flips_every_gen(int K, int W, int S, int NC = 4);
// the slab shapes whose launches can skip stable slabs (StencilParams::act): the production gol_slab2
// shapes, without flips
bool stencil_slab_activity(int K, int W, int S, int NC);
hipError_t warm_stencil_tile(hipStream_t s);
// The whole-board kernel (stencil_board.hip): one workgroup holds a board of wd in {4, 8, 16} words
// and `height` = 4 W R rows in registers and runs K (runtime, <= kBoardMaxK) generations in one
// launch.  stencil_board_shape: whether the board fits, and its (W waves, R rows per segment).
constexpr int kBoardMaxK = 4096;
// Automatic use (golhip_set_board_kernel -1): boards of at most this many rows.  One CU issues the
// whole board's VALU work per generation, so the kernel gains while the board is short and loses
// beyond: us per turn, board / slab kernels, calls of 1000 turns with counts
// (profiles/r05/r05k_board_ab.log): 16^2 0.31 / 0.52, 64^2 0.37 / 0.53, 128^2 0.42 / 0.53,
// 256^2 0.57 / 0.54, 512^2 0.88 / 0.55.
constexpr int64_t kBoardAutoRows = 256;
bool stencil_board_shape(int64_t height, int32_t wd, int *W, int *R);
hipError_t launch_stencil_board(int K, int W, int R, const uint32_t *in_row0, uint32_t *out_row0,
                                const StencilParams &p, unsigned long long *slots, hipStream_t s);
constexpr int kTileChunkWords = 62;
// Words per column chunk of the level-split kernel (half-word halo for K <= 16).
__host__ __device__ constexpr int split_chunk_words(int K) { return K <= 16 ? 63 : 62; }
// Resident waves per CU of the stencil launch (occupancy query), for sizing the grid.
int stencil_waves_per_cu(int K, int variant);
// Sum the slots of K generations into counts[0..K) and zero the slots.
hipError_t launch_count_finalize(int K, unsigned long long *slots, unsigned long long *counts,
                                 hipStream_t s);

// 0/nonzero bytes (rows x width, compact, stride == width) -> packed torus rows.
hipError_t launch_pack(const uint8_t *bytes, int64_t rows, int64_t width, int32_t wd,
                       uint32_t *row0, int64_t pitch, hipStream_t s);
// First `width` columns of packed rows -> 0/255 bytes (compact, stride == width).
hipError_t launch_unpack(const uint32_t *row0, int64_t pitch, int64_t rows, int64_t width,
                         uint8_t *bytes, hipStream_t s);
// Counter-based random rows; gy0 = global index of local row 0.
hipError_t launch_init_random(uint32_t *row0, int64_t pitch, int64_t rows, int64_t gy0,
                              int64_t width, int32_t wd, uint64_t seed, uint32_t density_q32,
                              hipStream_t s);
// Popcount of rows x wd words, added into *out.
hipError_t launch_popcount(const uint32_t *row0, int64_t pitch, int64_t rows, int32_t wd,
                           unsigned long long *out, hipStream_t s);
// Alive-cell / flip extraction (row-major): cells are bits of (a ^ b) (b nullable) in the first
// `width` columns.  row_counts[rows], offsets[rows+1], block_sums[kScanBlocks] are scratch;
// offsets = the exclusive scan of the row counts, offsets[rows] = total.  Multi-block: every
// block counts a contiguous range of rows, one block scans the block sums, every block then scans
// its range (three launches, no serial walk over the rows).
constexpr int kScanBlocks = 1024;
hipError_t launch_extract_count(const uint32_t *a, const uint32_t *b, int64_t pitch,
                                int64_t rows, int64_t width, uint32_t *row_counts,
                                unsigned long long *offsets, unsigned long long *block_sums,
                                hipStream_t s);
// slot_rows: rows per slot of a tall board of slots (y is reported within its slot).
hipError_t launch_extract_emit(const uint32_t *a, const uint32_t *b, int64_t pitch,
                               int64_t rows, int64_t width, const unsigned long long *offsets,
                               int64_t gy0, int64_t slot_rows, int32_t *xy, uint64_t cap,
                               hipStream_t s);
// x coordinates only, as uint16 (width <= 65536), in the same order (golhip_step_flips_rows).
hipError_t launch_extract_emit_x16(const uint32_t *a, const uint32_t *b, int64_t pitch,
                                   int64_t rows, int64_t width, const unsigned long long *offsets,
                                   uint16_t *x, uint64_t cap, hipStream_t s);
// counts[t] = cells of slot t (rows [t * slot_rows, (t+1) * slot_rows)) from the extract scan.
hipError_t launch_extract_slot_counts(const unsigned long long *offsets, int64_t slot_rows,
                                      int64_t slots, unsigned long long *counts, hipStream_t s);
// Packed torus rows <-> logical uint64 words (width % 64 == 0; first width bits of each row).
hipError_t launch_words_out(const uint32_t *row0, int64_t pitch, int64_t rows, int64_t width,
                            uint64_t *words, hipStream_t s);
hipError_t launch_words_in(const uint64_t *words, int64_t rows, int64_t width, int32_t wd,
                           uint32_t *row0, int64_t pitch, hipStream_t s);

}  // namespace golhip
