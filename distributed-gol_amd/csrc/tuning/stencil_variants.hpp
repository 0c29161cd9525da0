// tuning/stencil_variants.hpp -- tuning library only: every measured gol_stencil variant of a launch
// depth (GOLHIP_VARIANT; tests/test_gpu_tuning.py, scripts/ab_*.py), registered per depth in
// kernel_extras() by tuning/stencil_variants_k<K>.hip.  Variants and their measurements: DESIGN.md
// section 3 and golhip_internal.hpp (kVariant*).
#pragma once
#include "../golhip_stencil.hpp"

namespace golhip {
namespace {

// Every measured variant (GOLHIP_VARIANT, tests/test_gpu_tuning.py, scripts/ab_*.py).
template <int K>
hipError_t launch_variant(int variant, const uint32_t *in, uint32_t *out, const StencilParams &p,
                          unsigned long long *slots, hipStream_t s) {
    switch (variant) {
        case kVariantChain: return launch_stencil_k<K, false, 1>(in, out, p, slots, s);
        case kVariantSkewD2: return launch_stencil_k<K, true, 2>(in, out, p, slots, s);
        case kVariantChainD2: return launch_stencil_k<K, false, 2>(in, out, p, slots, s);
        case kVariantSkewLdsPf: return launch_stencil_k<K, true, 1, 1>(in, out, p, slots, s);
        case kVariantChainLdsPf:
            if constexpr (K == 1) return launch_step1(in, out, p, slots, s);  // production K = 1
            return launch_stencil_k<K, false, 1, 1>(in, out, p, slots, s);
        case kVariantSkewLdsD2: return launch_stencil_k<K, true, 2, 1>(in, out, p, slots, s);
        case kVariantChainLdsD2: return launch_stencil_k<K, false, 2, 1>(in, out, p, slots, s);
        case kVariantDriftLds:
            if constexpr (K == 1) return launch_step1(in, out, p, slots, s);
            else if constexpr (K > 16) return launch_stencil_k<K, false, 1, 1, false, 1, kHalfHalo<K, 1>, true, true>(in, out, p, slots, s);
            else return launch_stencil_k<K, false, 1, 1, true, 1, true, true, true>(in, out, p, slots, s);
        case kVariantDrift62:
            if constexpr (K == 1) return launch_step1(in, out, p, slots, s);
            else return launch_stencil_k<K, false, 1, 1, true, 1, false, true, true>(in, out, p, slots, s);
        case kVariantProd:  // per depth and counting: the fastest measured (golhip_internal.hpp)
            return launch_prod<K>(in, out, p, slots, s);
        case kVariantStamp:  // the production kernel with per-wave timestamps (p.diff: stamps)
            if constexpr (K == 1) return launch_step1(in, out, p, slots, s);
            else if constexpr (K <= 16) {
                if (prod_pre(K, slots != nullptr))
                    return launch_stencil_k<K, false, 1, 1, true, 1, false, true, false, true, false, true>(in, out, p, slots, s);
                return launch_stencil_k<K, false, 1, 1, true, 1, false, true, false, false, false, true>(in, out, p, slots, s);
            } else return launch_stencil_k<K, false, 1, 1, true, 1, false, true, false, false, false, true>(in, out, p, slots, s);
        case kVariantDriftNoFill:
            if constexpr (K == 1) return launch_step1(in, out, p, slots, s);
            else return launch_stencil_k<K, false, 1, 1, (K <= 16), 1, kHalfHalo<K, 1>, false>(in, out, p, slots, s);
        case kVariantProdMask:  // production with the idle lanes of the last chunk masked off
            if constexpr (K == 1) return launch_step1(in, out, p, slots, s);
            else if constexpr (K <= 16) {
                if (prod_pre(K, slots != nullptr))
                    return launch_stencil_k<K, false, 1, 1, true, 1, false, true, true, true, true>(in, out, p, slots, s);
                return launch_stencil_k<K, false, 1, 1, true, 1, false, true, true, false, true>(in, out, p, slots, s);
            } else return launch_stencil_k<K, false, 1, 1, true, 1, false, true, true, false, true>(in, out, p, slots, s);
        case kVariantPre63:  // pre-shifted rows, 63-word chunks (K <= 16; drift62 above)
            if constexpr (K == 1) return launch_step1(in, out, p, slots, s);
            else if constexpr (K > 16) return launch_stencil_k<K, false, 1, 1, true, 1, false, true, true>(in, out, p, slots, s);
            else return launch_stencil_k<K, false, 1, 1, true, 1, false, true, true, true>(in, out, p, slots, s);
        case kVariantDriftZip:
            if constexpr (K == 1) return launch_step1(in, out, p, slots, s);
            else return launch_stencil_k<K, false, 1, 1, true, 2, false>(in, out, p, slots, s);
        default: return launch_stencil_k<K, true, 1>(in, out, p, slots, s);
    }
}

template <int K>
const void *variant_fn(int variant) {
    switch (variant) {
        case kVariantChain: return (const void *)gol_stencil<K, false, false, 1, 0, kHalfHalo<K, 1>>;
        case kVariantSkewD2: return (const void *)gol_stencil<K, false, true, 2, 0, kHalfHalo<K, 2>>;
        case kVariantChainD2: return (const void *)gol_stencil<K, false, false, 2, 0, kHalfHalo<K, 2>>;
        case kVariantSkewLdsPf: return (const void *)gol_stencil<K, false, true, 1, 1, kHalfHalo<K, 1>>;
        case kVariantChainLdsPf:
            if constexpr (K == 1) return step1_fn();
            return (const void *)gol_stencil<K, false, false, 1, 1, kHalfHalo<K, 1>>;
        case kVariantSkewLdsD2: return (const void *)gol_stencil<K, false, true, 2, 1, kHalfHalo<K, 2>>;
        case kVariantChainLdsD2: return (const void *)gol_stencil<K, false, false, 2, 1, kHalfHalo<K, 2>>;
        case kVariantDriftLds:
            if constexpr (K == 1) return step1_fn();
            else return (const void *)gol_stencil<K, false, false, 1, 1, kHalfHalo<K, 1>, (K <= 16)>;
        case kVariantDrift62:
            if constexpr (K == 1) return step1_fn();
            else return (const void *)gol_stencil<K, false, false, 1, 1, false, true, 1>;
        case kVariantProd: return prod_fn<K>();
        case kVariantStamp:
            if constexpr (K == 1) return step1_fn();
            else if constexpr (prod_pre(K)) return (const void *)gol_stencil<K, false, false, 1, 1, false, true, 1, true, false, 0, true, false, true>;
            else return (const void *)gol_stencil<K, false, false, 1, 1, false, true, 1, true, false, 0, false, false, true>;
        case kVariantDriftNoFill:
            if constexpr (K == 1) return step1_fn();
            else return (const void *)gol_stencil<K, false, false, 1, 1, kHalfHalo<K, 1>, (K <= 16), 1, false>;
        case kVariantProdMask:
            if constexpr (K == 1) return step1_fn();
            else if constexpr (prod_pre(K)) return (const void *)gol_stencil<K, false, false, 1, 1, false, true, 1, true, false, 0, true, true>;
            else return (const void *)gol_stencil<K, false, false, 1, 1, false, true, 1, true, false, 0, false, true>;
        case kVariantPre63:
            if constexpr (K == 1) return step1_fn();
            else if constexpr (K > 16) return (const void *)gol_stencil<K, false, false, 1, 1, false, true, 1>;
            else return (const void *)gol_stencil<K, false, false, 1, 1, false, true, 1, true, false, 0, true>;
        case kVariantDriftZip:
            if constexpr (K == 1) return step1_fn();
            else return (const void *)gol_stencil<K, false, false, 1, 1, false, true, 2>;
        default: return (const void *)gol_stencil<K, false, true, 1, 0, kHalfHalo<K, 1>>;
    }
}
}  // namespace
}  // namespace golhip

// The variant launchers of depth K, registered in kernel_extras() when the library loads.
#define GOLHIP_REGISTER_VARIANTS_K(K)                                                              \
    namespace golhip {                                                                             \
    namespace {                                                                                    \
    hipError_t tv_launch(int v, const uint32_t *in, uint32_t *out, const StencilParams &p,         \
                         unsigned long long *slots, hipStream_t s) {                               \
        return launch_variant<K>(v, in, out, p, slots, s);                                         \
    }                                                                                              \
    const void *tv_fn(int v) { return variant_fn<K>(v); }                                          \
    hipError_t tv_warm(int v, hipStream_t s) {                                                     \
        StencilParams p{};                                                                         \
        p.nchunks = 1; /* nbands = 0: every wave returns at once */                               \
        return launch_variant<K>(v, nullptr, nullptr, p, nullptr, s);                              \
    }                                                                                              \
    const bool tv_registered = [] {                                                                \
        KernelExtras &x = kernel_extras();                                                         \
        x.stencil[K] = tv_launch;                                                                  \
        x.stencil_fn[K] = tv_fn;                                                                   \
        x.stencil_warm[K] = tv_warm;                                                               \
        return true;                                                                               \
    }();                                                                                           \
    }                                                                                              \
    }
