// tuning/stencil_variants_k4.hip -- tuning library only: every gol_stencil variant at depth K = 4.
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(4)
