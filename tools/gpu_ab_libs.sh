#!/bin/bash
# Same-box A/B of libduck_<v>.so variants ($LIBS, default "A opq") on $CFGS (default C2), $REPS
# alternating passes, after a bit-identity check of each variant against the first one on C2
# (tools/lib_bitcmp.py, 30 env-steps).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-abl}
L=$PWD/open_duck_playground_amd
set -- ${LIBS:-A opq}
first=$1
for v in "$@"; do
  DUCK_LIB=$L/libduck_$v.so timeout -k 10 200 python tools/lib_bitcmp.py --config ${BCFG:-C2} --steps 30 --out $OUT/${TAG}_bc_$v.npz > $OUT/${TAG}_bc_$v.log 2>&1 || { tail -5 $OUT/${TAG}_bc_$v.log; exit 1; }
  [ $v = $first ] || { echo -n "$v vs $first: "; python tools/lib_bitcmp.py --cmp $OUT/${TAG}_bc_$first.npz $OUT/${TAG}_bc_$v.npz; }
done
rm -f $OUT/${TAG}_bc_*.npz
for i in $(seq 1 ${REPS:-2}); do for C in ${CFGS:-C2}; do for v in "$@"; do
  DUCK_LIB=$L/libduck_$v.so timeout -k 10 200 python bench.py --cpu-budget 0 --steps ${STEPS:-400} --warmup 20 --config $C > $OUT/${TAG}_${v}_${C}_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/${TAG}_${v}_${C}_$i.json'));print('$C $v %.4gM kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
done; done; done
