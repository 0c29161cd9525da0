// tuning/stencil_variants_k2.hip -- tuning library only: every gol_stencil variant at depth K = 2.
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(2)
