#!/bin/bash
# Same-box A/B/C...: alternate bench runs of libduck_A.so (baseline) and each named candidate library.
# usage: bash tools/gpu_abn.sh libduck_X1.so libduck_X2.so ...
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in libduck_A.so "$@"; do
    export DUCK_LIB=$PWD/open_duck_playground_amd/$v
    timeout -k 10 200 python bench.py --cpu-budget 0 --steps 400 > gpurun_out/abn.json 2> /dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abn.json'));print('$v value %.4gM  kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
  done
done
