#!/bin/bash
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sim2sim.py -x -v -s --timeout 200 --timeout-method thread > $OUT/sim2sim.log 2>&1 \
  || { tail -30 $OUT/sim2sim.log; exit 1; }
grep -E "per-period|control loop|passed|failed" $OUT/sim2sim.log
rm -rf $OUT/ppo_c2
timeout -k 10 600 python -u -m open_duck_playground_amd.runner --num_timesteps 9830400 --output_dir gpurun_out/ppo_c2 > $OUT/ppo_c2.log 2>&1 \
  || { tail -30 $OUT/ppo_c2.log; exit 1; }
grep -E "STEP" $OUT/ppo_c2.log
