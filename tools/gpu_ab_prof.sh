#!/bin/bash
# GPU parity (physics + env), same-box A/B, then the stage profile of the candidate.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_physics.py tests/test_gpu_env.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
bash tools/gpu_ab.sh || exit 1
if [ "$1" = "prof" ]; then
  DUCK_LIB=$PWD/open_duck_playground_amd/libduck_prof.so timeout -k 10 200 python tools/stage_prof.py 4096 --random 2>&1 | grep -v amdgpu.ids
fi
