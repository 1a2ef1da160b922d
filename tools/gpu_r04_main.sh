#!/bin/bash
# Round-4 evidence in one box call (boxes are scarce): step-time curve + driver-style C2 lines, the
# PPO fused-MLP tests and training throughput, the teacher-forced + physics suites, C4/C5 same-box A/B
# over $LIBS, the rough stage profiles. Each GPU step under its own timeout; stops at the first failure.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r04}
L=$PWD/open_duck_playground_amd
step() { echo "== $1 ($(date +%T))"; }
step curve
timeout -k 10 120 python tools/step_time_curve.py > $OUT/${TAG}_curve.txt 2>&1 || { tail -5 $OUT/${TAG}_curve.txt; exit 1; }
tail -2 $OUT/${TAG}_curve.txt
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-budget 0 > $OUT/${TAG}_drv$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/${TAG}_drv$i.json'));print('driver-style C2 %.4gM ms_per_step %.4f kernel_ms %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
done
if [ -z "$SKIP_PPO" ]; then
  step ppo-tests
  timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -v -s --timeout 300 --timeout-method thread > $OUT/${TAG}_ppo_tests.log 2>&1
  rc=$?; grep -E "PASS|FAIL|passed|failed" $OUT/${TAG}_ppo_tests.log | tail -14
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  step ppo-throughput
  timeout -k 10 300 python tools/ppo_throughput.py --updates 4 > $OUT/${TAG}_ppo_fused.json 2> $OUT/${TAG}_ppo_fused.err || { tail -5 $OUT/${TAG}_ppo_fused.err; exit 1; }
  DUCK_PPO_FUSED_MLP=0 timeout -k 10 300 python tools/ppo_throughput.py --updates 4 > $OUT/${TAG}_ppo_autograd.json 2> $OUT/${TAG}_ppo_autograd.err || { tail -5 $OUT/${TAG}_ppo_autograd.err; exit 1; }
  python -c "
import json
for k in ('fused', 'autograd'):
    d = json.load(open('$OUT/${TAG}_ppo_%s.json' % k)); print(k, '%.3gM env-steps/s' % (d['value'] / 1e6), d['timing'])"
fi
if [ -z "$SKIP_TESTS" ]; then
  step tf
  timeout -k 10 600 python -u -m pytest tests/test_gpu_teacher_forced.py -v -s --timeout 500 --timeout-method thread > $OUT/${TAG}_tf.log 2>&1
  rc=$?; grep -E "rules:|passed|failed" $OUT/${TAG}_tf.log | tail -30
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  step physics
  timeout -k 10 400 python -u -m pytest tests/test_gpu_physics.py -v -s --timeout 300 --timeout-method thread > $OUT/${TAG}_phys.log 2>&1
  rc2=$?; grep -E "passed|failed" $OUT/${TAG}_phys.log | tail -3
  [ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
fi
step ab
for i in 1 2; do for v in ${LIBS:-cand}; do for C in ${CFGS:-C4 C5}; do
  if [ $v = cand ]; then f=$L/libduck.so; else f=$L/libduck_$v.so; fi
  DUCK_LIB=$f timeout -k 10 200 python bench.py --cpu-budget 0 --steps 200 --warmup 20 --config $C > $OUT/${TAG}_ab_${v}_${C}_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/${TAG}_ab_${v}_${C}_$i.json'));print('$C $v %.4gM kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
done; done; done
if [ -f $L/libduck_prof.so ]; then
  step stage
  for T in rough_terrain rough_terrain_backlash; do
    DUCK_LIB=$L/libduck_prof.so timeout -k 10 200 python tools/stage_prof.py 4096 --random --task=$T > $OUT/${TAG}_stage_$T.txt 2>&1 || { tail $OUT/${TAG}_stage_$T.txt; exit 1; }
  done
  head -40 $OUT/${TAG}_stage_rough_terrain.txt
fi
step done
