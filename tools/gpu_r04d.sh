#!/bin/bash
# rough_dr outlier dump (tools/diag_tf_substep.py), the whole GPU suite without -x, PPO throughput
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/diag_tf_substep.py run rough_dr 6 256 6 1e-3 > $OUT/r04d_diag.txt 2>&1 || { tail $OUT/r04d_diag.txt; exit 1; }
cat $OUT/r04d_diag.txt | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/r04d_tests.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/r04d_tests.log | tail -3; grep -E "^FAILED|rules:" $OUT/r04d_tests.log | head -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/ppo_throughput.py --updates 4 > $OUT/r04d_ppo.json 2> $OUT/r04d_ppo.err || { tail -5 $OUT/r04d_ppo.err; exit 1; }
python -c "
import json
d = json.load(open('$OUT/r04d_ppo.json')); print('ppo', '%.3gM env-steps/s' % (d['value'] / 1e6), d['timing'])"
