// stencil_k8.hip -- the production 8-generation stencil launcher, one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(8)
}  // namespace golhip
