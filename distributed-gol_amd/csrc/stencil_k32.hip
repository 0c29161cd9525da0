// stencil_k32.hip -- the production 32-generation stencil launcher, one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(32)
}  // namespace golhip
