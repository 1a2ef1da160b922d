#!/bin/bash
# Round 6 call C: the shipped LATENCY_X2 kernel (the latency kernel at two workgroups per CU): the whole
# GPU suite, its step time against the paired kernel at 1,536 / 2,048 envs (C2, C3), the bench lines.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r06c_gpu_tests.log 2>&1 || { tail -60 $OUT/r06c_gpu_tests.log; exit 1; }
grep -E "passed|failed" $OUT/r06c_gpu_tests.log | tail -2
for C in C2 C3; do
  for N in 1536 2048; do
    for M in paired latency_x2; do
      f=$OUT/r06c_w_${C}_${M}_$N
      $T 240 python bench.py --config $C --envs $N --steps 200 --warmup 20 --cpu-budget 0 --step-mode $M > $f.json 2> $f.err || { tail $f.err; exit 1; }
      python -c "import json;d=json.load(open('$f.json'));print('$C', '$M', $N, '%.4gM env-steps/s %.4f ms kernel %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
    done
  done
done
DUCK_DIST_BACKEND=gloo $T 300 python bench.py --gpus 2 --strong --steps 100 --warmup 10 --cpu-budget 0 > $OUT/r06c_bench_strong2.jsonl 2> $OUT/r06c_bench_strong2.err || { tail -30 $OUT/r06c_bench_strong2.err; exit 1; }
cat $OUT/r06c_bench_strong2.jsonl
$T 300 python bench.py --steps 20 --warmup 5 > $OUT/r06c_bench_C2_driver.json 2> $OUT/r06c_bench_C2_driver.err || { tail -30 $OUT/r06c_bench_C2_driver.err; exit 1; }
cat $OUT/r06c_bench_C2_driver.json
