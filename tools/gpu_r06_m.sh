#!/bin/bash
# Learner GEMM variants against the shipped tiles (libduck.so: 64 x 32 tiles, one LDS buffer, two barriers per
# chunk, 6 workgroups per CU). Variants: build/libduck_<v>.so, e.g. db32a = double-buffered LDS (one barrier per
# chunk) with 32 x 32 tiles (24 KB, 6 per CU). usage: VARIANTS="db32a" bash tools/gpu_r06_m.sh
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
V=${VARIANTS:-db32a}
first=$(echo $V | cut -d' ' -f1)
DUCK_LIB=$PWD/open_duck_playground_amd/build/libduck_$first.so $T 600 python -u -m pytest tests/test_gpu_ppo.py -x -q --timeout 300 --timeout-method thread > $OUT/r06m_tests.log 2>&1 || { tail -40 $OUT/r06m_tests.log; exit 1; }
tail -1 $OUT/r06m_tests.log
for run in 1 2; do
  for LIBV in base $V; do
    L=""; [ $LIBV != base ] && L=$PWD/open_duck_playground_amd/build/libduck_$LIBV.so
    DUCK_LIB=$L $T 300 python tools/ppo_throughput.py --updates 6 > $OUT/r06m_${LIBV}.json 2> $OUT/r06m.err || { tail -20 $OUT/r06m.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/r06m_${LIBV}.json'));print('$run $LIBV', '%.3fM training env-steps/s' % (d['value']/1e6), 'learn %.1f ms/update' % (d['timing']['learn_s']/6e-3))"
  done
done
