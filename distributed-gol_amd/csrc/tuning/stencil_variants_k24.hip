// tuning/stencil_variants_k24.hip -- tuning library only: every gol_stencil variant at depth K = 24 (K = 20 / 24: depths only the tuning library has, the 62-word drift geometry measured for
// the driver's 20-turn region).
#include "stencil_variants.hpp"

GOLHIP_REGISTER_VARIANTS_K(24)
