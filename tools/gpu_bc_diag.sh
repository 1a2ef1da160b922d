#!/bin/bash
# Diagnosis for tools/gpu_ab_bitcmp.sh: A vs A determinism and A vs candidate per env-step (C4 at
# 4096 envs), then the rough stage profiles of libduck_Aprof.so and libduck_prof.so.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/open_duck_playground_amd
run() { DUCK_LIB=$L/$1 timeout -k 10 200 python tools/lib_bitcmp.py --config C4 --envs 4096 --steps 12 --every 1 --out $OUT/$2.npz > $OUT/$2.log 2>&1 || { tail -5 $OUT/$2.log; exit 1; }; }
run libduck_A.so dA1 && run libduck_A.so dA2 && run libduck.so dB || exit 1
echo -n "A vs A: "; python tools/lib_bitcmp.py --cmp $OUT/dA1.npz $OUT/dA2.npz
echo -n "A vs cand: "; python tools/lib_bitcmp.py --cmp $OUT/dA1.npz $OUT/dB.npz
rm -f $OUT/dA1.npz $OUT/dA2.npz $OUT/dB.npz
for v in Aprof prof; do
  DUCK_LIB=$L/libduck_$v.so timeout -k 10 200 python tools/stage_prof.py 4096 --random --task=rough_terrain > $OUT/d_stage_$v.txt 2>&1 || { tail $OUT/d_stage_$v.txt; exit 1; }
  echo "== $v"; grep -E "hfield|sat:|queue:|collision" $OUT/d_stage_$v.txt
done
