#!/bin/bash
# One teacher-forced case (or a -k expression) of the GPU suite, verbose.
# usage (repo root, on the box): bash tools/gpu_tf_case.sh EXPR [TAG]
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_teacher_forced.py -m gpu -x -v -s --timeout 500 \
  --timeout-method thread -k "$1" > gpurun_out/tf_case_${2:-x}.log 2>&1 || { tail -30 gpurun_out/tf_case_${2:-x}.log; exit 1; }
grep -E "outlier|reset:|passed|failed" gpurun_out/tf_case_${2:-x}.log | tail -30
