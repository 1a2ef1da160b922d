// variant_rough.hip — kernels for the 'rough' model (generated/duck_model_rough.h).
#include "duck_env_kernels.h"
#include "generated/duck_model_rough.h"

DUCK_DEFINE_VARIANT(rough, DuckModel_rough)
