#!/bin/bash
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/diag_newton.py rough_terrain_backlash rough_terrain > $OUT/diag_newton_def.log 2>&1 || { tail -30 $OUT/diag_newton_def.log; exit 1; }
DUCK_LIB=$PWD/open_duck_playground_amd/libduck_ilp.so timeout -k 10 300 python -u tools/diag_newton.py \
  rough_terrain_backlash rough_terrain > $OUT/diag_newton_ilp.log 2>&1 || { tail -30 $OUT/diag_newton_ilp.log; exit 1; }
grep -v amdgpu.ids $OUT/diag_newton_def.log $OUT/diag_newton_ilp.log | grep "nsub"
