#!/bin/bash
# Learner: the weight gradients' row-block target (DUCK_WGRAD_TARGET workgroups per weight gradient) A/B.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
for run in 1 2; do
  for W in 768 384 1536 3072; do
    DUCK_WGRAD_TARGET=$W $T 300 python tools/ppo_throughput.py --updates 6 > $OUT/r06s_$W.json 2> $OUT/r06s.err || { tail -20 $OUT/r06s.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/r06s_$W.json'));print('$run target $W', '%.3fM training env-steps/s' % (d['value']/1e6), 'learn %.1f ms/update' % (d['timing']['learn_s']/6e-3))"
  done
done
