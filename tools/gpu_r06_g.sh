#!/bin/bash
# Round 6: the 60 M-step learning curve on the round-6 learner, then the rough + backlash + DR outlier report
# over four seeds (tools/tf_outlier_report.py).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m open_duck_playground_amd.runner --num_timesteps 60000000 --output_dir $OUT/ppo60M > $OUT/ppo60M.log 2>&1 || { tail -20 $OUT/ppo60M.log; exit 1; }
grep -v amdgpu.ids $OUT/ppo60M.log | tail -3
for s in 7 11 13 17; do
  $T 600 python -u tools/tf_outlier_report.py rough_backlash_dr $s > $OUT/r06_tf_report_$s.txt 2>&1 || { tail -20 $OUT/r06_tf_report_$s.txt; exit 1; }
  grep -E "^==|^rules" $OUT/r06_tf_report_$s.txt
done
