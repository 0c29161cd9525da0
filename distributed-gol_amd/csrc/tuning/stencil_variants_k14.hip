// tuning/stencil_variants_k14.hip -- tuning library only: every gol_stencil variant at depth K = 14.
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(14)
