#!/bin/bash
# Same-box timing of several library builds (libduck_<v>.so; "cand" = libduck.so), alternating, plus the
# teacher-forced parity suite on each. usage: VARIANTS="a b" bash tools/gpu_ab_multi.sh
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for v in $VARIANTS; do
  if [ $v = cand ]; then unset DUCK_LIB; else export DUCK_LIB=$PWD/open_duck_playground_amd/libduck_$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_teacher_forced.py -x -q -s --timeout 200 --timeout-method thread > $OUT/abm_tf_$v.log 2>&1 \
    && echo "$v parity: $(tail -1 $OUT/abm_tf_$v.log)" || echo "$v parity FAILED: $(grep -E 'Error|assert' $OUT/abm_tf_$v.log | head -2)"
done
for i in 1 2; do
  for v in $VARIANTS; do
    if [ $v = cand ]; then unset DUCK_LIB; else export DUCK_LIB=$PWD/open_duck_playground_amd/libduck_$v.so; fi
    timeout -k 10 200 python bench.py --cpu-budget 0 --steps 400 --config ${CFG:-C2} > $OUT/abm_$v$i.json 2> $OUT/abm_$v$i.err || { tail -3 $OUT/abm_$v$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/abm_$v$i.json'));print('$v value %.4gM  kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
  done
done
