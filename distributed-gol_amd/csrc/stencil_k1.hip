// stencil_k1.hip -- the production 1-generation stencil launcher, one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(1)
}  // namespace golhip
