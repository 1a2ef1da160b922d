#!/bin/bash
# Rough-terrain stage profiles (-DDUCK_STAGE_PROF) of libduck_Aprof.so and libduck_prof.so, same box.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/open_duck_playground_amd
for v in Aprof prof; do
  DUCK_LIB=$L/libduck_$v.so timeout -k 10 200 python tools/stage_prof.py 4096 --random --task=${TASK:-rough_terrain} > $OUT/sab_$v.txt 2>&1 || { tail $OUT/sab_$v.txt; exit 1; }
  echo "== $v"; grep -E "hfield|sat:|queue:|^collision " $OUT/sab_$v.txt
done
