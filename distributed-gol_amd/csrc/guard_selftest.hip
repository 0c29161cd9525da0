// guard_selftest.hip -- NOT part of libgolhip.  A deliberately spilling instantiation of the hot
// stencil (K = 16 forced to 8 waves per SIMD: 64 VGPRs for ~110 of live state) that
// scripts/check_vmcnt.py must REJECT: spilled registers go through scratch loads/stores, which are
// vector-memory operations the hand-counted LDS-DMA vmcnt waits do not account for.  The Makefile's
// guard target builds this object and requires the check to fail on it.
#include "golhip_stencil.hpp"

namespace golhip {

hipError_t guard_selftest_launch(const uint32_t *in, uint32_t *out, const StencilParams &p,
                                 hipStream_t s) {
    hipLaunchKernelGGL((gol_stencil<16, false, false, 1, 1, false, true, 1, true, false, 8, true>),
                       dim3(1), dim3(256), 0, s, in, out, p, nullptr);
    return hipGetLastError();
}

}  // namespace golhip
