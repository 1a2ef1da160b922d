#!/bin/bash
# Quick GPU iteration: parity suite (physics + env), C2 bench without CPU leg, stage cycles.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/quick_tests.log 2>&1 \
  || { tail -30 $OUT/quick_tests.log; exit 1; }
tail -2 $OUT/quick_tests.log
timeout -k 10 200 python bench.py --cpu-budget 0 > $OUT/quick_bench.json 2> $OUT/quick_bench.err || { tail $OUT/quick_bench.json; exit 1; }
python -c "import json;d=json.load(open('$OUT/quick_bench.json'));print('value %.4gM  kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
if [ -f open_duck_playground_amd/libduck_prof.so ]; then
  DUCK_LIB=$PWD/open_duck_playground_amd/libduck_prof.so timeout -k 10 200 python tools/stage_prof.py 4096 --random 2>&1 | grep -v amdgpu.ids
fi
