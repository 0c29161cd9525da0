// tuning/stencil_variants_k10.hip -- tuning library only: every gol_stencil variant at depth K = 10.
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(10)
