#!/bin/bash
# Stage-cycle profile (-DDUCK_STAGE_PROF build) of the rough scenes (C4 shape at 4096 envs, C5), random actions.
set -o pipefail
mkdir -p gpurun_out
for T in rough_terrain rough_terrain_backlash; do
  DUCK_LIB=$PWD/open_duck_playground_amd/libduck_prof.so timeout -k 10 200 python tools/stage_prof.py 4096 --random --task=$T > gpurun_out/stage_$T.txt 2>&1 || { tail gpurun_out/stage_$T.txt; exit 1; }
done
cat gpurun_out/stage_rough_terrain.txt
