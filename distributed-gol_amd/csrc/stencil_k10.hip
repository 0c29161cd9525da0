// stencil_k10.hip -- the production 10-generation stencil launcher, one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(10)
}  // namespace golhip
