// tuning/stencil_variants_k8.hip -- tuning library only: every gol_stencil variant at depth K = 8.
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(8)
