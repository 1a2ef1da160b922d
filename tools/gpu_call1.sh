#!/bin/bash
# max-ILP build: per-env Newton-step diagnosis, then the parity suite on the shipped library
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
DUCK_LIB=$PWD/open_duck_playground_amd/libduck_ilp.so timeout -k 10 300 python -u tools/diag_newton.py \
  rough_terrain_backlash flat_terrain_backlash > $OUT/diag_newton.log 2>&1 || { tail -30 $OUT/diag_newton.log; exit 1; }
cat $OUT/diag_newton.log | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/call1_tests.log 2>&1 \
  || { tail -30 $OUT/call1_tests.log; exit 1; }
tail -3 $OUT/call1_tests.log
