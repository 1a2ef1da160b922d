#!/bin/bash
# Height-field work on the box: teacher-forced suite + GPU physics tests on the candidate (libduck.so),
# C4 / C5 same-box A/B over the libraries in $LIBS (libduck_<v>.so, built by tools/ab_build.sh or
# native.build(out=...)), then the stage profile of libduck_prof.so (-DDUCK_STAGE_PROF) if present.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-hf}
timeout -k 10 120 python tools/step_time_curve.py > $OUT/${TAG}_curve.txt 2>&1 || { tail -5 $OUT/${TAG}_curve.txt; exit 1; }
tail -3 $OUT/${TAG}_curve.txt
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-budget 0 > $OUT/${TAG}_drv$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/${TAG}_drv$i.json'));print('driver-style C2 %.4gM ms_per_step %.4f kernel_ms %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
done
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_teacher_forced.py -v -s --timeout 600 --timeout-method thread > $OUT/${TAG}_tf.log 2>&1
  rc=$?; grep -E "rules:|passed|failed" $OUT/${TAG}_tf.log | tail -30
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 400 python -u -m pytest tests/test_gpu_physics.py -v -s --timeout 300 --timeout-method thread > $OUT/${TAG}_phys.log 2>&1
  rc2=$?; grep -E "passed|failed" $OUT/${TAG}_phys.log | tail -3
  [ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
fi
L=$PWD/open_duck_playground_amd
for i in 1 2; do for v in ${LIBS:-A cand}; do for C in ${CFGS:-C4 C5}; do
  if [ $v = cand ]; then f=$L/libduck.so; else f=$L/libduck_$v.so; fi
  DUCK_LIB=$f timeout -k 10 200 python bench.py --cpu-budget 0 --steps 200 --warmup 20 --config $C > $OUT/${TAG}_ab_${v}_${C}_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/${TAG}_ab_${v}_${C}_$i.json'));print('$C $v %.4gM kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
done; done; done
if [ -f $L/libduck_prof.so ]; then
  for T in rough_terrain rough_terrain_backlash; do
    DUCK_LIB=$L/libduck_prof.so timeout -k 10 200 python tools/stage_prof.py 4096 --random --task=$T > $OUT/${TAG}_stage_$T.txt 2>&1 || { tail $OUT/${TAG}_stage_$T.txt; exit 1; }
  done
  cat $OUT/${TAG}_stage_rough_terrain.txt
fi
