#!/bin/bash
# paired/latency kernel timelines; the plane collision out of line: latency/throughput bit-compare and C2 A/B
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 400 bash tools/gpu_latprof2.sh || exit 1
DUCK_LIB=$PWD/open_duck_playground_amd/libduck_planenoinline.so $T 300 python -u tools/lat_bitcmp.py C2 C3 > $OUT/r05c_bitcmp.txt 2>&1 || { tail -5 $OUT/r05c_bitcmp.txt; exit 1; }
grep -v amdgpu.ids $OUT/r05c_bitcmp.txt
for i in 1 2; do
  for v in libduck libduck_planenoinline; do
    DUCK_LIB=$PWD/open_duck_playground_amd/$v.so $T 200 python bench.py --steps 400 --warmup 50 --cpu-budget 0 > $OUT/r05c_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/r05c_$v.json'));print('$v', '%.4gM' % (d['value']/1e6), 'kernel_ms %.4f' % d['roofline']['kernel_ms'])"
  done
done
