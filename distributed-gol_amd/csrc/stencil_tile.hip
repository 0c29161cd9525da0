// stencil_tile.hip -- the production register-slab shapes for small boards and their dispatch.
// The kernels and launch templates are in stencil_tile.hpp (shared with the tuning library's
// tuning/stencil_tile_tuning.hip, which registers the other shapes, the register tiles and the
// timestamping slab kernels in kernel_extras()).
#include "stencil_tile.hpp"

namespace golhip {

// (K, waves, rows per wave, interleaved row chains): the production shapes (pick_reg_kernel:
// slab_prod_shape in stencil_tile.hpp).
// Round 4: K = 16 runs gol_slab2 (NC = 9) in production (configs[1] 5120^2 with every count 0.908
// -> 0.843 us/turn, configs[4]-sized 4096^2 0.829 -> 0.781; profiles/r04/r04c_tune_slab.log), and
// with counts gol_slab2 flushing every generation's count at the end of the launch (NC = 12: 0.772
// at 5120^2 with 16 x 6, 0.730 at 4096^2 with 12 x 7; profiles/r04/r04u_tune.log).  Narrow boards
// (wd <= 30) run the packed gol_slabp (NC = 14) at 4 / 6 / 8 waves x 3 rows (512^2 with every
// count 0.811 -> 0.570 us/turn, without 0.708 -> 0.373: profiles/r04/r04p4_narrow_sweep.log).
// Round 5: the packed slab at depths 2 / 4 / 8 / 12 too, for the tails of narrow-board calls
// (configs[0]'s 100 turns ended in gol_slab 12 + 8 launches at 11.8 + 8.0 us against ~7 us per
// packed launch: profiles/r05/r05p_cfg0_timeline.log).
// Round 6: 12 x 4 (T = 16: 12 rows per SIMD against 16 x 4's 16) with and without counts, for boards
// whose 12 x 4 slabs fit one round over the CUs (2048^2 with every count 0.556 -> 0.503 us/turn in
// the tuning build, profiles/r05/r05zc_t16_slabs_ab.log; round 6 A/B: profiles/r06/).
#define GOLHIP_SLAB_PROD_CONFIGS(X) \
    X(8, 8, 8, 4) X(12, 8, 8, 4) X(16, 8, 12, 9) X(16, 16, 6, 9) X(16, 12, 8, 9) X(16, 12, 7, 9) \
    X(16, 16, 6, 12) X(16, 12, 7, 12) X(16, 12, 8, 12) X(16, 16, 4, 9) X(16, 16, 4, 12) X(16, 12, 4, 9) X(16, 12, 4, 12) \
    X(16, 4, 3, 14) X(16, 6, 3, 14) X(16, 8, 3, 14) \
    X(12, 4, 3, 14) X(12, 6, 3, 14) X(12, 8, 3, 14) X(8, 4, 3, 14) X(8, 6, 3, 14) X(8, 8, 3, 14) \
    X(4, 4, 3, 14) X(4, 6, 3, 14) X(4, 8, 3, 14) X(2, 4, 3, 14) X(2, 6, 3, 14) X(2, 8, 3, 14)

static bool slab_prod_supported(int K, int W, int S, int NC) {
#define GOLHIP_X(KK, WW, SS, NN) \
    if (K == KK && W == WW && S == SS && NC == NN) return true;
    GOLHIP_SLAB_PROD_CONFIGS(GOLHIP_X)
#undef GOLHIP_X
    return false;
}

bool stencil_slab_flips_every_gen(int K, int W, int S, int NC) {
    return stencil_slab_supported(K, W, S, NC) && slab_prod_shape(K, W, S, NC);
}

bool stencil_slab_activity(int K, int W, int S, int NC) {
    return slab_prod_supported(K, W, S, NC) && (NC == kSlab2 || NC == kSlab2E);
}

bool stencil_slab_supported(int K, int W, int S, int NC) {
    if (slab_prod_supported(K, W, S, NC)) return true;
    const auto f = kernel_extras().slab_supported;
    return f && f(K, W, S, NC);
}

hipError_t launch_stencil_slab(int K, int W, int S, int NC, const uint32_t *in_row0, uint32_t *out_row0,
                               const StencilParams &p, unsigned long long *slots, hipStream_t s) {
    if (!p.stamp) {
#define GOLHIP_X(KK, WW, SS, NN) \
    if (K == KK && W == WW && S == SS && NC == NN) \
        return launch_slab_kws<KK, WW, SS, NN>(in_row0, out_row0, p, slots, s);
        GOLHIP_SLAB_PROD_CONFIGS(GOLHIP_X)
#undef GOLHIP_X
    }
    if (const auto f = kernel_extras().slab) return f(K, W, S, NC, in_row0, out_row0, p, slots, s);
    return hipErrorInvalidValue;
}

// The register tiles are tuning-library kernels (kernel_extras().tile).
bool stencil_tile_supported(int K, int T) {
    const auto f = kernel_extras().tile_supported;
    return f && f(K, T);
}

hipError_t launch_stencil_tile(int K, int T, const uint32_t *in_row0, uint32_t *out_row0,
                               const StencilParams &p, unsigned long long *slots, hipStream_t s) {
    if (const auto f = kernel_extras().tile) return f(K, T, in_row0, out_row0, p, slots, s);
    return hipErrorInvalidValue;
}

// The level-split kernel is a tuning-library kernel (kernel_extras().split): since the register
// slab took the small boards, the automatic planner never picks it.
bool stencil_split_supported(int K, int S) {
    const auto f = kernel_extras().split_supported;
    return f && f(K, S);
}

hipError_t launch_stencil_split(int K, int S, const uint32_t *in_row0, uint32_t *out_row0,
                                const StencilParams &p, unsigned long long *slots, hipStream_t s) {
    if (const auto f = kernel_extras().split) return f(K, S, in_row0, out_row0, p, slots, s);
    return hipErrorInvalidValue;
}

hipError_t warm_stencil_split(hipStream_t s) {
    if (const auto f = kernel_extras().split_warm) return f(s);
    return hipSuccess;
}

// Load the register kernels' code object before anything is timed (an empty launch: nbands = 0).
hipError_t warm_stencil_tile(hipStream_t s) {
    StencilParams p{};
    p.nchunks = 1;  // nbands = 0: every wave returns at once
    hipLaunchKernelGGL((gol_slab2<16, 8, 12, false, 0>), dim3(1), dim3(512), 0, s, nullptr, nullptr, p,
                       nullptr);
    return hipGetLastError();
}

}  // namespace golhip
