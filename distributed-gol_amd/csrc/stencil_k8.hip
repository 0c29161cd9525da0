// stencil_k8.hip -- the 8-generation stencil launchers (every variant), one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(8)
}  // namespace golhip
