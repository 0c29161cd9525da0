// tuning/stencil_split_tuning.hip -- tuning library only: the level-split stencil
// (gol_stencil_split) launchers, registered in kernel_extras().  Since the register slab
// (stencil_tile.hip) took the small boards, the automatic planner never picks the level split
// (pick_split needs fewer minimal-band waves than the slab leaves it), so the production library
// ships no instantiation and reports every (K, S) unsupported.
#include "../golhip_stencil.hpp"

namespace golhip {
namespace {

bool split_supported(int K, int S) {
    if (S == 2) return K == 4 || K == 6 || K == 8 || K == 12 || K == 16 || K == 32;
    if (S == 4) return K == 4 || K == 8 || K == 12 || K == 16 || K == 32;
    if (S == 8) return K == 8 || K == 16 || K == 32;
    return false;
}

hipError_t split(int K, int S, const uint32_t *in_row0, uint32_t *out_row0, const StencilParams &p,
                 unsigned long long *slots, hipStream_t s) {
#define GOL_SPLIT_CASE(KK, SS) \
    if (K == KK && S == SS) return launch_split_ks<KK, SS>(in_row0, out_row0, p, slots, s);
    GOL_SPLIT_CASE(4, 2) GOL_SPLIT_CASE(6, 2) GOL_SPLIT_CASE(8, 2) GOL_SPLIT_CASE(12, 2)
    GOL_SPLIT_CASE(16, 2) GOL_SPLIT_CASE(32, 2)
    GOL_SPLIT_CASE(4, 4) GOL_SPLIT_CASE(8, 4) GOL_SPLIT_CASE(12, 4) GOL_SPLIT_CASE(16, 4)
    GOL_SPLIT_CASE(32, 4)
    GOL_SPLIT_CASE(8, 8) GOL_SPLIT_CASE(16, 8) GOL_SPLIT_CASE(32, 8)
#undef GOL_SPLIT_CASE
    return hipErrorInvalidValue;
}

hipError_t split_warm(hipStream_t s) {
    StencilParams p{};
    p.nchunks = 1;  // nbands = 0: the workgroup returns at once
    hipLaunchKernelGGL((gol_stencil_split<16, false, 8>), dim3(1), dim3(64 * 8), 0, s, nullptr,
                       nullptr, p, nullptr);
    return hipGetLastError();
}

const bool registered = [] {
    KernelExtras &x = kernel_extras();
    x.split_supported = split_supported;
    x.split = split;
    x.split_warm = split_warm;
    return true;
}();

}  // namespace
}  // namespace golhip
