// stencil_k6.hip -- the production 6-generation stencil launcher, one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(6)
}  // namespace golhip
