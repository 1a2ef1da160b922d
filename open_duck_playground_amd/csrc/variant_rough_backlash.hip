// variant_rough_backlash.hip — kernels for the 'rough_backlash' model (generated/duck_model_rough_backlash.h).
#include "duck_env_kernels.h"
#include "generated/duck_model_rough_backlash.h"

DUCK_DEFINE_VARIANT(rough_backlash, DuckModel_rough_backlash)
