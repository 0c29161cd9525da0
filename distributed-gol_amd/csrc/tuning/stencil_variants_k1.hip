// tuning/stencil_variants_k1.hip -- tuning library only: every gol_stencil variant at depth K = 1.
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(1)
