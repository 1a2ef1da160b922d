#!/bin/bash
# tools/tf_seed_sweep.py for libduck_A.so and the candidate libduck.so, same seeds.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/open_duck_playground_amd
for v in A cand; do
  if [ $v = cand ]; then f=$L/libduck.so; else f=$L/libduck_$v.so; fi
  DUCK_LIB=$f timeout -k 10 400 python tools/tf_seed_sweep.py ${CASE:-rough_dr} ${SEEDS:-7 11 13} > $OUT/tfs_$v.txt 2>&1 || { tail -5 $OUT/tfs_$v.txt; exit 1; }
  echo "== $v"; grep seed $OUT/tfs_$v.txt | cut -c1-400
done
