// variant_backlash.hip — kernels for the 'backlash' model (generated/duck_model_backlash.h).
#include "duck_env_kernels.h"
#include "generated/duck_model_backlash.h"

DUCK_DEFINE_VARIANT(backlash, DuckModel_backlash)
