#!/bin/bash
# Round 6 learner A/B: reduction chunk KC = 32 (shipped) vs 64 (build/libduck_kc64.so), tile width 32 / 64.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
for run in 1 2; do
  for LIBV in shipped kc64; do
    for BNM in 32 64; do
      L=""; [ $LIBV = kc64 ] && L=open_duck_playground_amd/build/libduck_kc64.so
      DUCK_LIB=$L DUCK_MLP_BN=$BNM $T 300 python tools/ppo_throughput.py --updates 6 > $OUT/r06f_${LIBV}_$BNM.json 2> $OUT/r06f.err || { tail -20 $OUT/r06f.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/r06f_${LIBV}_$BNM.json'));print('$run $LIBV BN=$BNM', '%.3fM training env-steps/s' % (d['value']/1e6), 'learn %.1f ms/update' % (d['timing']['learn_s']/6e-3))"
    done
  done
done
