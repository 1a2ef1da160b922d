#!/bin/bash
# The fused PPO loss: its parity test and the GPU PPO tests, then training throughput fused vs torch loss.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -x -v --timeout 300 --timeout-method thread > $OUT/ppo_fused_tests.log 2>&1 \
  || { tail -30 $OUT/ppo_fused_tests.log; exit 1; }
grep -E "passed|failed|PASS|FAIL" $OUT/ppo_fused_tests.log | tail -12
for f in 1 0 1; do
  DUCK_PPO_FUSED=$f timeout -k 10 300 python tools/ppo_throughput.py --updates 5 > $OUT/ppo_tp_$f.json 2> $OUT/ppo_tp_$f.err || { tail $OUT/ppo_tp_$f.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ppo_tp_$f.json'));print('fused=$f', '%.3gM env-steps/s' % (d['value']/1e6), d['timing'])"
done
