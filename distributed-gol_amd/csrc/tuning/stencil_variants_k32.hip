// tuning/stencil_variants_k32.hip -- tuning library only: every gol_stencil variant at depth K = 32.
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(32)
