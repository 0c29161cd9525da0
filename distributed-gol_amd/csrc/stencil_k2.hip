// stencil_k2.hip -- the production 2-generation stencil launcher, one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(2)
}  // namespace golhip
