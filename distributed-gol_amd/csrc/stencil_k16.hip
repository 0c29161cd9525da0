// stencil_k16.hip -- the 16-generation stencil launchers (every variant), one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(16)
}  // namespace golhip
