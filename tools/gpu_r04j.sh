#!/bin/bash
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_r04h.sh || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_teacher_forced.py -x -q -s --timeout 300 --timeout-method thread \
  -k "step_parity and (flat_imitation or rough_backlash_dr or standing) and not autoreset and not throughput" > $OUT/r04j_tf.log 2>&1; rc=$?
grep -E "rules:|passed|failed" $OUT/r04j_tf.log | tail -6
exit $rc
