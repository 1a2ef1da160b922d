#!/bin/bash
set -o pipefail
# (usage: build the candidate as open_duck_playground_amd/libduck_B.so -- git archive HEAD into a temp dir, apply
# tools/patches/*.patch, native.build(out=...libduck_B.so) -- then run this on the box: C5 A/B + rough parity)
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/open_duck_playground_amd
for i in 1 2 3; do for v in libduck libduck_B; do
  DUCK_LIB=$L/$v.so timeout -k 10 200 python bench.py --cpu-budget 0 --steps 400 --config C5 > $OUT/abB_$v$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/abB_$v$i.json'));print('C5 $v %.4gM kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
done; done
DUCK_LIB=$L/libduck_B.so timeout -k 10 400 python -u -m pytest tests/test_gpu_teacher_forced.py -k "rough" -x -q -s --timeout 300 --timeout-method thread > $OUT/abB_tf.log 2>&1 || { tail -30 $OUT/abB_tf.log; exit 1; }
grep -E "passed|failed" $OUT/abB_tf.log | tail -2
