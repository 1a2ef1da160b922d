#!/bin/bash
# latency kernel diagnosis: per-step differences vs the throughput kernel (tools/diag_lat.py) for
# the four scenes, then teacher-forced parity of the latency kernel against the oracle (two cases)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for C in C2 C3 C4 C5; do
  echo "== $C"; timeout -k 10 120 python tools/diag_lat.py --config $C --envs 512 --steps 6 || exit 1
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_teacher_forced.py -x -v -s --timeout 300 --timeout-method thread \
  -k "step_parity and (flat_imitation or rough_backlash_dr) and not autoreset and not throughput" > $OUT/r04_lat_tf.log 2>&1; rc=$?
grep -E "rules:|good_frac|passed|failed" $OUT/r04_lat_tf.log | tail -12
exit $rc
