#!/bin/bash
# Round 5: the paired latency kernel (8 envs per workgroup, each substep's stages over a pair of waves):
# equivalence with the throughput kernel, the surfaced timeout in both latency kernels, AUTO's choice,
# the teacher-forced paired cases; then its step time against the other two kernels.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_env.py::test_latency_timeout_surfaces" \
  "tests/test_gpu_env.py::test_step_mode_auto_selects_by_batch" \
  "tests/test_gpu_env.py::test_latency_mode_matches_throughput_mode" \
  "tests/test_gpu_teacher_forced.py::test_teacher_forced_step_parity" -s > $OUT/r05b_tests.log 2>&1 || { tail -40 $OUT/r05b_tests.log; exit 1; }
grep -E "passed|failed" $OUT/r05b_tests.log | tail -3
CONFIGS="C2 C5" MODES="paired" SIZES="1024 1536 2048" STEPS=100 $T 600 bash tools/gpu_latency.sh > $OUT/r05b_lat.txt 2>&1 || { tail -5 $OUT/r05b_lat.txt; exit 1; }
CONFIGS="C2 C5" MODES="throughput latency" SIZES="2048" STEPS=100 $T 600 bash tools/gpu_latency.sh >> $OUT/r05b_lat.txt 2>&1 || { tail -5 $OUT/r05b_lat.txt; exit 1; }
cat $OUT/r05b_lat.txt
