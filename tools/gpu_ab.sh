#!/bin/bash
# Same-box A/B: alternate bench runs of libduck_A.so (baseline) and libduck.so (candidate).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export DUCK_LIB=$PWD/open_duck_playground_amd/libduck_A.so; else unset DUCK_LIB; fi
    timeout -k 10 200 python bench.py --cpu-budget 0 --steps 400 > gpurun_out/ab_$v$i.json 2> /dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_$v$i.json'));print('$v value %.4gM  kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
  done
done
