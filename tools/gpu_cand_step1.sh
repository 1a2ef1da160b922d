#!/bin/bash
# Per-env differences between libduck_A.so and the candidate after each of the first 5 env-steps (C4 shape).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/open_duck_playground_amd
for v in A cand; do
  if [ $v = cand ]; then f=$L/libduck.so; else f=$L/libduck_$v.so; fi
  DUCK_LIB=$f timeout -k 10 200 python tools/lib_bitcmp.py --config ${BCFG:-C4} --envs 4096 --steps 5 --every 1 --out $OUT/s1_$v.npz > $OUT/s1_$v.log 2>&1 || { tail -5 $OUT/s1_$v.log; exit 1; }
done
python tools/lib_bitcmp.py --cmp $OUT/s1_A.npz $OUT/s1_cand.npz --envs-of 4096
