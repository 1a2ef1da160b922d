#!/bin/bash
# step-time curve after reset (driver-style short runs), PPO kernel profile, latency curve of both kernels
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python tools/step_time_curve.py > $OUT/r04_curve.txt 2>&1 || { tail -5 $OUT/r04_curve.txt; exit 1; }
grep -v amdgpu.ids $OUT/r04_curve.txt
bash tools/gpu_ppo_prof.sh r04 > $OUT/r04_ppo_prof.txt 2>&1 || { tail $OUT/r04_ppo_prof.txt; exit 1; }
head -20 $OUT/r04_ppo_prof.txt
SIZES="256 512 1024 2048 4096 8192" STEPS=40 bash tools/gpu_latency.sh > $OUT/r04_latency.txt 2>&1 || { tail $OUT/r04_latency.txt; exit 1; }
cat $OUT/r04_latency.txt
