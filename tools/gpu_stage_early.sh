#!/bin/bash
# Flat (C2) stage profile over env-steps 5-24 after reset (the driver's timed window) and 80-99.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/open_duck_playground_amd
for w in 5 80; do
  DUCK_LIB=${PROF_LIB:-$L/libduck_prof.so} timeout -k 10 200 python tools/stage_prof.py 4096 --random --warm=$w --steps=20 > $OUT/early_w$w.txt 2>&1 || { tail $OUT/early_w$w.txt; exit 1; }
done
paste $OUT/early_w5.txt $OUT/early_w80.txt | grep -v amdgpu.ids | cut -c1-150
