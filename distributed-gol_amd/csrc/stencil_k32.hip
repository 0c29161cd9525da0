// stencil_k32.hip -- the 32-generation stencil launchers (every variant), one TU per launch depth.
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(32)
}  // namespace golhip
