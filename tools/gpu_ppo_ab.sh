#!/bin/bash
# PPO learner A/B: the fused-learner GPU tests on libduck.so, then training throughput with
# libduck_<A>.so (baseline) and libduck.so alternating (tools/ppo_throughput.py, 8192 envs)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -x -q -s --timeout 300 --timeout-method thread > $OUT/ppo_ab_tests.log 2>&1 \
  || { tail -30 $OUT/ppo_ab_tests.log; exit 1; }
grep -E "passed|failed" $OUT/ppo_ab_tests.log | tail -2
for i in 1 2; do
  for v in ${A:-kc32} cand; do
    if [ $v = cand ]; then unset DUCK_LIB; else export DUCK_LIB=$PWD/open_duck_playground_amd/libduck_$v.so; fi
    timeout -k 10 300 python tools/ppo_throughput.py --updates 4 > $OUT/ppo_ab_$v$i.json 2> $OUT/ppo_ab_$v$i.err || { tail -5 $OUT/ppo_ab_$v$i.err; exit 1; }
    python -c "import json; d = json.load(open('$OUT/ppo_ab_$v$i.json')); print('$v', '%.3gM env-steps/s' % (d['value'] / 1e6), d['timing'])"
  done
done
