#!/bin/bash
# learning evidence: the reference runner's CLI for 60 M env-steps on flat terrain (metrics in gpurun_out/ppo60M)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m open_duck_playground_amd.runner --num_timesteps 60000000 --output_dir $OUT/ppo60M > $OUT/ppo60M.log 2>&1 || { tail -20 $OUT/ppo60M.log; exit 1; }
grep -v amdgpu.ids $OUT/ppo60M.log | tail -5
