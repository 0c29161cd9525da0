// stencil_k4.hip -- the production 4-generation stencil launcher, one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(4)
}  // namespace golhip
