#!/bin/bash
# One GPU call: the whole -m gpu suite (verbose, per-test timeout), then a C2 bench line.
# usage (from the repo root, on the box): bash tools/gpu_suite.sh TAG
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests_$TAG.log 2>&1 || { tail -40 $OUT/gpu_tests_$TAG.log; exit 1; }
grep -E "passed|failed" $OUT/gpu_tests_$TAG.log | tail -2
timeout -k 10 300 python bench.py --cpu-budget 0 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { cat $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
