#!/bin/bash
# Same-box A/B timing only (no parity suite): bench.py with libduck_<A>.so vs libduck.so, alternating,
# for each config in CFGS. usage: A=A CFGS="C2 C5" bash tools/gpu_ab_quick.sh
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for i in 1 2 3; do
  for C in ${CFGS:-C2}; do
    for v in ${A:-A} cand; do
      if [ $v = cand ]; then unset DUCK_LIB; else export DUCK_LIB=$PWD/open_duck_playground_amd/libduck_$v.so; fi
      timeout -k 10 200 python bench.py --cpu-budget 0 --steps ${STEPS:-400} --config $C --step-mode throughput \
        > $OUT/abq_${C}_$v$i.json 2> $OUT/abq_${C}_$v$i.err || { tail -3 $OUT/abq_${C}_$v$i.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/abq_${C}_$v$i.json'));print('$C $v value %.4gM  kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
    done
  done
done
