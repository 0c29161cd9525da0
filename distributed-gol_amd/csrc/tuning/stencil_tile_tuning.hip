// tuning/stencil_tile_tuning.hip -- tuning library only: the register-slab shapes and slab kernels
// production does not ship (the measured neighbours of the production shapes, gol_slab3, the
// gol_slab2 flush / priority variants, other packed-slab shapes), the register tiles gol_tile, and
// the timestamping slab kernels (StencilParams::stamp; scripts/slab_stamps.py).  Registered in
// kernel_extras() when the library loads (profiles/r02/small_boards.txt, profiles/r03/r03e_tune_slab.log,
// profiles/r04/r04c_tune_slab.log, r04o_tune.log, r04w_tune_prio.log).
#include "../stencil_tile.hpp"

namespace golhip {
namespace {

#define GOLHIP_SLAB_TUNING_CONFIGS(X) \
    X(16, 8, 12, 2) X(16, 12, 8, 2) X(16, 12, 7, 2) \
    X(8, 8, 4, 4) X(16, 8, 8, 4) X(16, 8, 12, 4) X(16, 16, 8, 4) \
    X(16, 12, 8, 4) X(16, 10, 8, 2) X(16, 14, 6, 2) X(16, 16, 6, 2) X(16, 16, 5, 2) \
    X(8, 8, 8, 9) X(12, 8, 8, 9) X(16, 16, 5, 9) X(16, 10, 8, 9) X(16, 8, 8, 9) X(16, 12, 6, 9) \
    X(16, 8, 12, 10) X(16, 16, 6, 10) X(16, 12, 8, 10) X(16, 12, 7, 10) X(16, 10, 8, 10) X(16, 8, 10, 10) \
    X(16, 8, 12, 11) X(16, 8, 10, 11) X(16, 10, 8, 11) X(16, 12, 8, 11) \
    X(16, 16, 5, 12) X(16, 16, 6, 13) X(16, 12, 7, 13) X(16, 8, 12, 13) \
    X(16, 8, 11, 12) X(16, 8, 10, 12) X(16, 8, 11, 9) X(16, 10, 9, 12) X(16, 12, 6, 12) X(16, 16, 4, 12) X(16, 8, 6, 12) X(16, 12, 4, 12) \
    X(16, 4, 4, 14) X(16, 8, 4, 14) X(16, 8, 6, 14) X(16, 16, 3, 14) \
    X(16, 4, 5, 14) X(16, 4, 6, 14) X(16, 12, 3, 14) X(16, 2, 6, 14) X(16, 2, 8, 14) \
    X(12, 8, 3, 14) X(12, 4, 3, 14) X(8, 8, 3, 14) X(8, 4, 3, 14) X(8, 4, 4, 14) \
    X(16, 12, 7, 15) X(16, 16, 6, 15) X(16, 12, 4, 15) X(16, 16, 4, 15) X(16, 12, 8, 15) X(16, 8, 12, 15)
// the production shapes of the slab2 / slab3 families, timestamped (p.stamp)
#define GOLHIP_SLAB_STAMP_CONFIGS(X) \
    X(16, 8, 12, 9) X(16, 16, 6, 9) X(16, 12, 8, 9) X(16, 12, 7, 9) \
    X(16, 16, 6, 12) X(16, 12, 7, 12) X(16, 12, 8, 12) \
    X(16, 8, 12, 10) X(16, 16, 6, 10) X(16, 12, 8, 10) X(16, 12, 7, 10) X(16, 10, 8, 10) X(16, 8, 10, 10) \
    X(16, 8, 12, 11) X(16, 8, 10, 11) X(16, 10, 8, 11) X(16, 12, 8, 11) \
    X(16, 16, 5, 12) X(16, 16, 6, 13) X(16, 12, 7, 13) X(16, 8, 12, 13)
#define GOLHIP_TILE_CONFIGS(X) \
    X(2, 16) X(4, 8) X(4, 16) X(4, 32) X(6, 16) X(8, 8) X(8, 16) X(8, 32) X(10, 16) X(12, 8) \
    X(12, 16) X(12, 32) X(14, 16) X(16, 8) X(16, 16) X(16, 32)

bool slab_supported(int K, int W, int S, int NC) {
#define GOLHIP_X(KK, WW, SS, NN) \
    if (K == KK && W == WW && S == SS && NC == NN) return true;
    GOLHIP_SLAB_TUNING_CONFIGS(GOLHIP_X)
#undef GOLHIP_X
    return false;
}

hipError_t slab(int K, int W, int S, int NC, const uint32_t *in, uint32_t *out, const StencilParams &p,
                unsigned long long *slots, hipStream_t s) {
    if (p.stamp) {
#define GOLHIP_X(KK, WW, SS, NN) \
    if (K == KK && W == WW && S == SS && NC == NN) \
        return launch_slab_kws<KK, WW, SS, NN, true>(in, out, p, slots, s);
        GOLHIP_SLAB_STAMP_CONFIGS(GOLHIP_X)
#undef GOLHIP_X
        return hipErrorInvalidValue;
    }
#define GOLHIP_X(KK, WW, SS, NN) \
    if (K == KK && W == WW && S == SS && NC == NN) return launch_slab_kws<KK, WW, SS, NN>(in, out, p, slots, s);
    GOLHIP_SLAB_TUNING_CONFIGS(GOLHIP_X)
#undef GOLHIP_X
    return hipErrorInvalidValue;
}

bool tile_supported(int K, int T) {
#define GOLHIP_X(KK, TT) \
    if (K == KK && T == TT) return true;
    GOLHIP_TILE_CONFIGS(GOLHIP_X)
#undef GOLHIP_X
    return false;
}

hipError_t tile(int K, int T, const uint32_t *in, uint32_t *out, const StencilParams &p,
                unsigned long long *slots, hipStream_t s) {
#define GOLHIP_X(KK, TT) \
    if (K == KK && T == TT) return launch_tile_kt<KK, TT>(in, out, p, slots, s);
    GOLHIP_TILE_CONFIGS(GOLHIP_X)
#undef GOLHIP_X
    return hipErrorInvalidValue;
}

const bool registered = [] {
    KernelExtras &x = kernel_extras();
    x.slab_supported = slab_supported;
    x.slab = slab;
    x.tile_supported = tile_supported;
    x.tile = tile;
    return true;
}();

}  // namespace
}  // namespace golhip
