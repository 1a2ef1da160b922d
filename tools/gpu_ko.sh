#!/bin/bash
# Knockout timing: bench C2 with libduck.so and with libduck_<variant>.so builds that skip a stage
# (wrong physics; an upper bound on what optimising that stage could gain). Same box, alternating.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
for i in 1 2; do
  for v in base $KO; do
    if [ $v = base ]; then unset DUCK_LIB; else export DUCK_LIB=$PWD/open_duck_playground_amd/libduck_$v.so; fi
    timeout -k 10 200 python bench.py --cpu-budget 0 --steps 400 > $OUT/ko_$v$i.json 2> $OUT/ko_$v$i.err || { tail -3 $OUT/ko_$v$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ko_$v$i.json'));print('$v value %.4gM  kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
  done
done
