// tuning/stencil_step1_tuning.hip -- tuning library only: gol_step1's prefetch depth and cache
// policy by GOLHIP_STEP1 = P*10 + NT (read when the library loads; unset or 42 = the production
// configuration, 4 rows in flight with non-temporal stores: profiles/r01_tune_step1.txt).
#include <cstdlib>

#include "../golhip_stencil.hpp"

namespace golhip {
namespace {

#define GOLHIP_STEP1_CONFIGS(X) \
    X(20, 2, 0) X(22, 2, 2) X(30, 3, 0) X(32, 3, 2) X(40, 4, 0) X(41, 4, 1) X(42, 4, 2) \
    X(43, 4, 3) X(60, 6, 0) X(62, 6, 2) X(80, 8, 0) X(82, 8, 2)

int g_cfg = 42;

hipError_t step1(const uint32_t *in, uint32_t *out, const StencilParams &p, unsigned long long *slots,
                 hipStream_t s) {
    switch (g_cfg) {
#define GOLHIP_X(C, P, NT) \
    case C: return launch_step1_cfg<P, NT>(in, out, p, slots, s);
        GOLHIP_STEP1_CONFIGS(GOLHIP_X)
#undef GOLHIP_X
        default: return launch_step1_cfg<4, 2>(in, out, p, slots, s);
    }
}

const void *step1_fn_cfg() {
    switch (g_cfg) {
#define GOLHIP_X(C, P, NT) \
    case C: return (const void *)gol_step1<false, P, NT>;
        GOLHIP_STEP1_CONFIGS(GOLHIP_X)
#undef GOLHIP_X
        default: return (const void *)gol_step1<false, 4, 2>;
    }
}

const bool registered = [] {
    const char *e = std::getenv("GOLHIP_STEP1");
    g_cfg = e ? std::atoi(e) : 42;
    if (g_cfg != 42) {
        kernel_extras().step1 = step1;
        kernel_extras().step1_fn = step1_fn_cfg;
    }
    return true;
}();

}  // namespace
}  // namespace golhip
