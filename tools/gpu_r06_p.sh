#!/bin/bash
# The bench lines on the final build with the build-id-matched PMC files in profiles/ (issue roofline and
# counter traffic filled in): C2 steady, C2 in the driver's 20-after-5 form three times, C5.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python bench.py > $OUT/r06p_bench_C2.json 2> $OUT/r06p_bench.err || { tail -20 $OUT/r06p_bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/r06p_bench_C2.json'));print('C2 steady %.4gM %.4f ms' % (d['value']/1e6, d['ms_per_step']), d['issue_roofline'], d['roofline']['traffic'])"
rm -f $OUT/r06p_bench_C2_driver_style.jsonl
for i in 1 2 3; do
  $T 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-budget 0 >> $OUT/r06p_bench_C2_driver_style.jsonl 2> $OUT/r06p_bench.err || { tail -20 $OUT/r06p_bench.err; exit 1; }
done
python -c "import json; print('driver form', [round(json.loads(l)['value']/1e6, 3) for l in open('$OUT/r06p_bench_C2_driver_style.jsonl')])"
$T 300 python bench.py --config C5 --cpu-budget 0 > $OUT/r06p_bench_C5.json 2> $OUT/r06p_bench.err || { tail -20 $OUT/r06p_bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/r06p_bench_C5.json'));print('C5 %.4gM %.4f ms' % (d['value']/1e6, d['ms_per_step']), d['issue_roofline'])"
