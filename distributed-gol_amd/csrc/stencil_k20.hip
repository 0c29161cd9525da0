// stencil_k20.hip -- the 20-generation stencil launchers (tuning build only: Makefile TDEPTHS).
#include "golhip_stencil.hpp"

namespace golhip {
GOLHIP_DEFINE_STENCIL_K(20)
}  // namespace golhip
