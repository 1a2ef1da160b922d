#!/bin/bash
# Round 6 learner A/B: output tile rows BM = 64 (shipped) vs 32 (build/libduck_bm32.so).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
for run in 1 2; do
  for LIBV in shipped bm32; do
    L=""; [ $LIBV = bm32 ] && L=open_duck_playground_amd/build/libduck_bm32.so
    DUCK_LIB=$L $T 300 python tools/ppo_throughput.py --updates 6 > $OUT/r06h_${LIBV}.json 2> $OUT/r06h.err || { tail -20 $OUT/r06h.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/r06h_${LIBV}.json'));print('$run $LIBV', '%.3fM training env-steps/s' % (d['value']/1e6), 'learn %.1f ms/update' % (d['timing']['learn_s']/6e-3))"
  done
done
DUCK_LIB=open_duck_playground_amd/build/libduck_bm32.so $T 300 python -m pytest tests/test_gpu_ppo.py -x -q -k "fused or group or gemm" > $OUT/r06h_tests.log 2>&1 || { tail -30 $OUT/r06h_tests.log; exit 1; }
tail -1 $OUT/r06h_tests.log
