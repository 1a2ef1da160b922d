#!/bin/bash
# Can step_kernel run two waves per SIMD? Compiles one scene unit with the production flags, once as
# shipped and once with amdgpu_waves_per_eu(2,2) on step_kernel (the register budget of two waves per
# SIMD: 256 VGPR + AGPR per lane), and prints the compiler's resource usage for both. CPU only.
# usage (repo root): bash tools/occupancy_probe.sh [flat|rough|backlash|rough_backlash]
set -e -o pipefail
V=${1:-flat}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/open_duck_playground_amd/csrc
TMP=$(mktemp -d)
trap 'rm -rf $TMP' EXIT
FLAGS=$(python3 -c "
import sys; sys.path.insert(0, '$ROOT')
from open_duck_playground_amd import native
print(' '.join(native.compile_flags()))")
sed 's/__global__ void __launch_bounds__(TPB) step_kernel/__global__ void __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(2, 2))) step_kernel/' \
  $CSRC/duck_env_kernels.h > $TMP/duck_env_kernels.h
grep -q 'amdgpu_waves_per_eu(2, 2)' $TMP/duck_env_kernels.h
# the unit includes "duck_env_kernels.h" from its own directory first: the capped copy sits next to it
cp $CSRC/variant_$V.hip $TMP/
for mode in shipped two_waves; do
  SRC=$([ $mode = two_waves ] && echo $TMP || echo $CSRC)/variant_$V.hip
  echo "== $V step_kernel, $mode"
  hipcc $FLAGS -Rpass-analysis=kernel-resource-usage -c $SRC -o $TMP/$mode.o 2>&1 \
    | grep -A10 'Function Name: _Z11step_kernel' | grep -E 'VGPRs|AGPRs|Scratch|Occupancy|Spill' | sed 's/.*remark: *//; s/ \[-R.*//'
done
