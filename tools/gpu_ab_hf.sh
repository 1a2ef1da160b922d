#!/bin/bash
# Height-field contact change on the box: teacher-forced suite + GPU physics tests on the candidate
# (libduck.so), then C4 / C5 same-box A/B against libduck_A.so (tools/ab_build.sh <rev>).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-hf}
timeout -k 10 900 python -u -m pytest tests/test_gpu_teacher_forced.py -v -s --timeout 600 --timeout-method thread > $OUT/${TAG}_tf.log 2>&1
rc=$?; grep -E "rules:|passed|failed" $OUT/${TAG}_tf.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_physics.py -v -s --timeout 300 --timeout-method thread > $OUT/${TAG}_phys.log 2>&1
rc2=$?; grep -E "passed|failed" $OUT/${TAG}_phys.log | tail -3
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
L=$PWD/open_duck_playground_amd
for i in 1 2; do for v in libduck_A libduck; do for C in C4 C5; do
  DUCK_LIB=$L/$v.so timeout -k 10 200 python bench.py --cpu-budget 0 --steps 200 --warmup 20 --config $C > $OUT/${TAG}_ab_${v}_${C}_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/${TAG}_ab_${v}_${C}_$i.json'));print('$C $v %.4gM kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
done; done; done
