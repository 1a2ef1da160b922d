#!/bin/bash
# Marker-free cost of the height-field SAT's sub-stages: builds that run one idempotent sub-stage
# twice (-DDUCK_DOUBLE = 11 pass 2, 12 pass 1, 13 contact point, 14 the lane-parallel screen,
# 15 vertical-edge pairs; libduck_d<k>.so) timed against libduck_A.so on the same box, C4 and C5.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
L=$PWD/open_duck_playground_amd
for i in 1 2; do for v in ${VARS:-A d11 d12 d13 d14 d15}; do for C in C4 C5; do
  DUCK_LIB=$L/libduck_$v.so timeout -k 10 200 python bench.py --cpu-budget 0 --steps 200 --warmup 20 --config $C > $OUT/sd_${v}_${C}_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/sd_${v}_${C}_$i.json'));print('$C $v %.4gM kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
done; done; done
