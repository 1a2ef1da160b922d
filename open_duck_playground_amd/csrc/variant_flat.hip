// variant_flat.hip — kernels for the 'flat' model (generated/duck_model_flat.h).
#include "duck_env_kernels.h"
#include "generated/duck_model_flat.h"

DUCK_DEFINE_VARIANT(flat, DuckModel_flat)
