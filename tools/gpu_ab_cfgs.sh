#!/bin/bash
# Same-box A/B over several configurations: libduck_A.so (baseline, tools/ab_build.sh) against
# libduck.so (candidate), alternating, after the teacher-forced + physics parity tests on the
# candidate. usage: CFGS="C2 C4 C5" bash tools/gpu_ab_cfgs.sh
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ -z "$SKIP_TF" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_teacher_forced.py tests/test_gpu_physics.py -x -q -s --timeout 200 --timeout-method thread > $OUT/abc_tf.log 2>&1 \
  || { tail -30 $OUT/abc_tf.log; exit 1; }
tail -1 $OUT/abc_tf.log
fi
for i in 1 2; do
  for C in ${CFGS:-C2 C4 C5}; do
    for v in A cand; do
      if [ $v = cand ]; then unset DUCK_LIB; else export DUCK_LIB=$PWD/open_duck_playground_amd/libduck_A.so; fi
      timeout -k 10 200 python bench.py --cpu-budget 0 --steps ${STEPS:-200} --config $C > $OUT/abc_$C$v$i.json 2> $OUT/abc_$C$v$i.err || { tail -3 $OUT/abc_$C$v$i.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/abc_$C$v$i.json'));print('$C $v %.4gM  kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
    done
  done
done
