// stencil_k24.hip -- the 24-generation stencil launchers (tuning build only: Makefile TDEPTHS).
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(24)
}  // namespace golhip
