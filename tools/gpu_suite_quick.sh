#!/bin/bash
# The whole -m gpu suite, then C2 / C4 / C5 bench lines (no CPU baseline): one GPU call.
# usage (repo root, on the box): bash tools/gpu_suite_quick.sh TAG
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -1
for C in C2 C4 C5; do
  timeout -k 10 300 python bench.py --config $C --cpu-budget 0 > gpurun_out/bench_${TAG}_$C.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$C.json'));print('$C', round(d['value']/1e6,3), 'M env-steps/s, kernel', round(d['roofline']['kernel_ms'],4), 'ms')"
done
