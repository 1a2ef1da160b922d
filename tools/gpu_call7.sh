#!/bin/bash
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/diag_newton.py rough_terrain_backlash flat_terrain > $OUT/diag_newton_fix.log 2>&1 || { tail -30 $OUT/diag_newton_fix.log; exit 1; }
grep "nsub" $OUT/diag_newton_fix.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/call7_tests.log 2>&1 \
  || { tail -30 $OUT/call7_tests.log; exit 1; }
tail -2 $OUT/call7_tests.log
for c in C2 C5; do
  timeout -k 10 200 python bench.py --config $c --cpu-budget 0 > $OUT/call7_bench_$c.json 2> $OUT/call7_bench_$c.err || { tail $OUT/call7_bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/call7_bench_$c.json'));print('$c', 'value %.4gM  ms %.4f kernel_ms %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
done
