// stencil_k16.hip -- the production 16-generation stencil launcher, one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(16)
}  // namespace golhip
