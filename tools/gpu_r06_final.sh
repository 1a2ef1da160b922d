#!/bin/bash
# Round 6 final evidence on the final build: the GPU suite, smoke(), the C2 and C5 rocprofv3 evidence
# (kernel trace + stats, FETCH/WRITE_SIZE, SQ passes; tools/gpu_pmc.sh), the bench lines C2 (steady and
# the driver's 20-after-5 form), C3, C4, C5, and bench.py --gpus 2 run directly (weak and --strong, gloo).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r06_final_gpu_tests.log 2>&1 || { tail -60 $OUT/r06_final_gpu_tests.log; exit 1; }
grep -E "passed|failed" $OUT/r06_final_gpu_tests.log | tail -1
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r06_final_smoke.log 2>&1 || { tail -20 $OUT/r06_final_smoke.log; exit 1; }
grep smoke $OUT/r06_final_smoke.log
$T 400 bash tools/gpu_pmc.sh r06 C2 > $OUT/r06_final_pmc_c2.log 2>&1 || { tail -20 $OUT/r06_final_pmc_c2.log; exit 1; }
$T 400 bash tools/gpu_pmc.sh r06 C5 > $OUT/r06_final_pmc_c5.log 2>&1 || { tail -20 $OUT/r06_final_pmc_c5.log; exit 1; }
ls $OUT/pmc_r06
$T 300 python bench.py > $OUT/r06_bench_C2.json 2> $OUT/r06_bench.err || { tail -20 $OUT/r06_bench.err; exit 1; }
cat $OUT/r06_bench_C2.json
for i in 1 2 3; do
  $T 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-budget 0 >> $OUT/r06_bench_C2_driver_style.jsonl 2> $OUT/r06_bench.err || { tail -20 $OUT/r06_bench.err; exit 1; }
done
python -c "import json; print('driver form', [round(json.loads(l)['value']/1e6, 3) for l in open('$OUT/r06_bench_C2_driver_style.jsonl')])"
for C in C3 C4 C5; do
  $T 300 python bench.py --config $C --cpu-budget 0 > $OUT/r06_bench_$C.json 2> $OUT/r06_bench.err || { tail -20 $OUT/r06_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r06_bench_$C.json'));print('$C', '%.4gM env-steps/s %.4f ms' % (d['value']/1e6, d['ms_per_step']))"
done
DUCK_DIST_BACKEND=gloo $T 300 python bench.py --gpus 2 --steps 100 --warmup 10 --cpu-budget 0 > $OUT/r06_bench_direct2.jsonl 2> $OUT/r06_bench.err || { tail -20 $OUT/r06_bench.err; exit 1; }
DUCK_DIST_BACKEND=gloo $T 300 python bench.py --gpus 2 --strong --steps 100 --warmup 10 --cpu-budget 0 >> $OUT/r06_bench_direct2.jsonl 2> $OUT/r06_bench.err || { tail -20 $OUT/r06_bench.err; exit 1; }
cut -c1-400 $OUT/r06_bench_direct2.jsonl
