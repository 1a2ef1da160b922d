#!/bin/bash
# latency-kernel iteration: parity of the latency kernel vs the throughput kernel, C2/C5 step times at 512
# envs (both kernels), and the throughput kernel against libduck_A.so (same box)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py -x -q -s --timeout 300 --timeout-method thread \
  -k "latency_mode or step_mode_auto" > $OUT/lat_ab_tests.log 2>&1 || { tail -30 $OUT/lat_ab_tests.log; exit 1; }
grep -E "passed|failed" $OUT/lat_ab_tests.log | tail -2
SIZES="512" CONFIGS="C2 C5" STEPS=100 bash tools/gpu_latency.sh || exit 1
A=A CFGS="C2" STEPS=400 bash tools/gpu_ab_quick.sh
