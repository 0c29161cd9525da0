// tuning/stencil_variants_k16.hip -- tuning library only: every gol_stencil variant at depth K = 16.
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(16)
