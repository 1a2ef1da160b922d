#!/bin/bash
# teacher-forced suite + rough stage profiles + PPO tests, throughput and kernel profile
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo.py -v -s --timeout 200 --timeout-method thread > $OUT/r04c_ppo_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" $OUT/r04c_ppo_tests.log | tail -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/ppo_throughput.py --updates 4 > $OUT/r04c_ppo_fused.json 2> $OUT/r04c_ppo_fused.err || { tail -5 $OUT/r04c_ppo_fused.err; exit 1; }
python -c "
import json
d = json.load(open('$OUT/r04c_ppo_fused.json')); print('fused', '%.3gM env-steps/s' % (d['value'] / 1e6), d['timing'])"
bash tools/gpu_ppo_prof.sh r04c > $OUT/r04c_prof_summary.txt 2>&1; head -3 $OUT/r04c_prof_summary.txt
bash tools/gpu_tf_stage.sh
