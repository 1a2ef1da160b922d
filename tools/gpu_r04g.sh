#!/bin/bash
# latency-kernel timeline (DUCK_LAT_PROF build) for C2 and C5, then the PPO learner A/B against libduck_A.so
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for C in C2 C5; do
  DUCK_LIB=$PWD/open_duck_playground_amd/libduck_latprof.so timeout -k 10 120 python tools/lat_prof.py --config $C > $OUT/r04_latprof_$C.txt 2>&1 || { tail $OUT/r04_latprof_$C.txt; exit 1; }
  echo "== $C"; grep -v amdgpu.ids $OUT/r04_latprof_$C.txt
done
A=A bash tools/gpu_ppo_ab.sh
