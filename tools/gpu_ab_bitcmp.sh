#!/bin/bash
# Same-box check of a kernel change that must not change any result: bit-identity of the candidate
# (libduck.so) against libduck_A.so (tools/ab_build.sh) over 100 env-steps of C4 and C5, then the
# C4 / C5 bench A/B, alternating. usage: bash tools/gpu_ab_bitcmp.sh [TAG]
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-bc}
L=$PWD/open_duck_playground_amd
for C in ${CFGS:-C4 C5}; do
  for v in A cand; do
    if [ $v = cand ]; then f=$L/libduck.so; else f=$L/libduck_$v.so; fi
    DUCK_LIB=$f timeout -k 10 200 python tools/lib_bitcmp.py --config $C --steps 100 --out $OUT/${TAG}_${C}_$v.npz > $OUT/${TAG}_${C}_$v.log 2>&1 || { tail -5 $OUT/${TAG}_${C}_$v.log; exit 1; }
  done
  python tools/lib_bitcmp.py --cmp $OUT/${TAG}_${C}_A.npz $OUT/${TAG}_${C}_cand.npz | sed "s/^/$C /"
  rm -f $OUT/${TAG}_${C}_A.npz $OUT/${TAG}_${C}_cand.npz
done
for i in 1 2; do for v in A cand; do for C in ${CFGS:-C4 C5}; do
  if [ $v = cand ]; then f=$L/libduck.so; else f=$L/libduck_$v.so; fi
  DUCK_LIB=$f timeout -k 10 200 python bench.py --cpu-budget 0 --steps 200 --warmup 20 --config $C > $OUT/${TAG}_ab_${v}_${C}_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/${TAG}_ab_${v}_${C}_$i.json'));print('$C $v %.4gM kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
done; done; done
