#!/bin/bash
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for C in C2 C5; do
  DUCK_LIB=$PWD/open_duck_playground_amd/libduck_latprof.so timeout -k 10 120 python tools/lat_prof.py --config $C > $OUT/r04_latprof_$C.txt 2>&1 || { tail $OUT/r04_latprof_$C.txt; exit 1; }
  echo "== $C"; grep -v amdgpu.ids $OUT/r04_latprof_$C.txt
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py -x -q -s --timeout 300 --timeout-method thread \
  -k "latency_mode or step_mode_auto" > $OUT/lat_ab_tests.log 2>&1 || { tail -30 $OUT/lat_ab_tests.log; exit 1; }
grep -E "passed|failed" $OUT/lat_ab_tests.log | tail -2
SIZES="512" CONFIGS="C2 C5" MODES=latency STEPS=100 bash tools/gpu_latency.sh
