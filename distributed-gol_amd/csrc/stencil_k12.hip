// stencil_k12.hip -- the production 12-generation stencil launcher, one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(12)
}  // namespace golhip
