// stencil_k14.hip -- the production 14-generation stencil launcher, one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(14)
}  // namespace golhip
