// tuning/stencil_variants_k6.hip -- tuning library only: every gol_stencil variant at depth K = 6.
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(6)
