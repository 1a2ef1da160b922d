#!/bin/bash
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for lib in libduck_dbg libduck_ilp_dbg; do
  DUCK_LIB=$PWD/open_duck_playground_amd/$lib.so timeout -k 10 200 python -u tools/diag_lds.py rough_terrain_backlash 2 > $OUT/diag_lds_$lib.log 2>&1 || { tail -30 $OUT/diag_lds_$lib.log; exit 1; }
  echo "== $lib"; grep -v amdgpu.ids $OUT/diag_lds_$lib.log
done
