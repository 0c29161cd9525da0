// tuning/stencil_variants_k12.hip -- tuning library only: every gol_stencil variant at depth K = 12.
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(12)
