#!/bin/bash
# Same-box A/B: bench C2 with libduck_<A>.so (baseline) vs libduck.so (candidate), alternating;
# then the teacher-forced parity suite on the candidate. usage: A=nofloor bash tools/gpu_ab_lib.sh
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_teacher_forced.py tests/test_gpu_physics.py -x -q -s --timeout 200 --timeout-method thread > $OUT/ab_tf.log 2>&1 \
  || { tail -30 $OUT/ab_tf.log; exit 1; }
grep -E "passed|failed|good_frac" $OUT/ab_tf.log | cut -c1-200 | tail -12
for i in 1 2 3; do
  for v in $A cand; do
    if [ $v = cand ]; then unset DUCK_LIB; else export DUCK_LIB=$PWD/open_duck_playground_amd/libduck_$v.so; fi
    timeout -k 10 200 python bench.py --cpu-budget 0 --steps 400 --config ${CFG:-C2} > $OUT/ab_$v$i.json 2> $OUT/ab_$v$i.err || { tail -3 $OUT/ab_$v$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab_$v$i.json'));print('$v value %.4gM  kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
  done
done
