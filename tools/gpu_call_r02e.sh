#!/bin/bash
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v -s --timeout 280 --timeout-method thread > $OUT/multirank.log 2>&1 \
  || { tail -30 $OUT/multirank.log; exit 1; }
grep -E "passed|failed" $OUT/multirank.log
rm -rf $OUT/ppo_c2_long
timeout -k 10 900 python -u -m open_duck_playground_amd.runner --num_timesteps 60000000 --output_dir gpurun_out/ppo_c2_long > $OUT/ppo_c2_long.log 2>&1 \
  || { tail -30 $OUT/ppo_c2_long.log; exit 1; }
grep -E "STEP" $OUT/ppo_c2_long.log
rm -f $OUT/ppo_c2_long/*.pt $OUT/ppo_c2_long/*.onnx
