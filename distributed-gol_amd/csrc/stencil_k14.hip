// stencil_k14.hip -- the 14-generation stencil launchers (every variant), one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(14)
}  // namespace golhip
