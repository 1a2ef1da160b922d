#!/bin/bash
# which stage group's cross-statement contractions make the flat kernels differ (tools/fpc_bisect.py libraries)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for v in all g1 g2 g3 g4 g5 g6 g7 g8 g9 g10; do
  DUCK_LIB=$PWD/open_duck_playground_amd/build/libduck_fpc_$v.so timeout -k 10 120 python -u tools/lat_bitcmp.py C2 > $OUT/r05f_$v.txt 2>&1 || { tail -5 $OUT/r05f_$v.txt; exit 1; }
  echo "$v: $(grep -v amdgpu.ids $OUT/r05f_$v.txt | cut -c1-150)"
done
