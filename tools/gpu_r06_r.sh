#!/bin/bash
# Step-kernel A/B: build/libduck_prev.so (the committed kernels) against build/libduck_new.so (the candidate):
# bit-identity of the state after 50 env-steps (flat, rough, rough + backlash) and same-box bench lines.
set -o pipefail
OUT=gpurun_out/r06r; rm -rf $OUT; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
P=$PWD/open_duck_playground_amd/build/libduck_prev.so; N=$PWD/open_duck_playground_amd/build/libduck_new.so
for task in flat_terrain rough_terrain rough_terrain_backlash; do
  for v in prev new; do
    L=$P; [ $v = new ] && L=$N
    DUCK_LIB=$L $T 200 python tools/ab_state_dump.py $OUT/${task}_$v.npz --task $task > /dev/null 2> $OUT/dump.err || { tail -20 $OUT/dump.err; exit 1; }
  done
  python -c "
import numpy as np
a, b = np.load('$OUT/${task}_prev.npz'), np.load('$OUT/${task}_new.npz')
print('$task', {k: bool((a[k].view(np.uint32) == b[k].view(np.uint32)).all()) for k in a.files})"
done
for run in 1 2; do
  for v in prev new; do
    L=$P; [ $v = new ] && L=$N
    for C in C2 C5 C4; do
      DUCK_LIB=$L $T 200 python bench.py --config $C --cpu-budget 0 > $OUT/${C}_$v.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/${C}_$v.json'));print('$run $v $C', '%.4gM %.4f ms' % (d['value']/1e6, d['roofline']['kernel_ms']))"
    done
  done
done
