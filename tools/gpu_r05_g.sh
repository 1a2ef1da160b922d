#!/bin/bash
# G7 narrowed (tools/fpc_bisect.py), then the C2 cost of the pragma (flat-only libraries, same box)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for v in sp cj fc mr g7; do
  DUCK_LIB=$PWD/open_duck_playground_amd/build/libduck_fpc_$v.so timeout -k 10 120 python -u tools/lat_bitcmp.py C2 C3 > $OUT/r05g_$v.txt 2>&1 || { tail -5 $OUT/r05g_$v.txt; exit 1; }
  echo "$v: $(grep -v amdgpu.ids $OUT/r05g_$v.txt | cut -c1-120)"
done
for i in 1 2 3; do for v in none g7; do
  DUCK_LIB=$PWD/open_duck_playground_amd/build/libduck_fpc_$v.so timeout -k 10 200 python bench.py --steps 400 --warmup 50 --cpu-budget 0 > $OUT/r05g_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/r05g_$v.json'));print('C2 $v', '%.4gM' % (d['value']/1e6), 'kernel_ms %.4f' % d['roofline']['kernel_ms'])"
done; done
