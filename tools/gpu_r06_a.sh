#!/bin/bash
# Round 6 first call: the VALU issue rate against waves per SIMD, the whole GPU suite
# (new: bench.py --gpus 2 run directly, train() raising on the device error word), the direct
# two-rank bench line, the C2 bench line.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
true
true
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r06a_gpu_tests.log 2>&1 || { tail -60 $OUT/r06a_gpu_tests.log; exit 1; }
grep -E "passed|failed" $OUT/r06a_gpu_tests.log | tail -2
DUCK_DIST_BACKEND=gloo $T 300 python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-budget 0 > $OUT/r06a_bench_direct2.jsonl 2> $OUT/r06a_bench_direct2.err || { tail -30 $OUT/r06a_bench_direct2.err; exit 1; }
cat $OUT/r06a_bench_direct2.jsonl
$T 300 python bench.py --steps 200 --warmup 20 > $OUT/r06a_bench_C2.json 2> $OUT/r06a_bench_C2.err || { tail -30 $OUT/r06a_bench_C2.err; exit 1; }
cat $OUT/r06a_bench_C2.json
# two waves per SIMD: the flat latency kernel capped at 256 VGPR + AGPR
# (-DDUCK_LAT_WAVES_PER_EU=2, build/libduck_lat2w.so: 2 VGPRs spilled, 61 KB LDS -> two workgroups per
# CU) against the shipped kernels at the same batch sizes, same box
for N in 1024 2048 4096 8192; do
  for M in throughput paired latency; do
    f=$OUT/r06a_w_${M}_$N
    $T 240 python bench.py --config C2 --envs $N --steps 100 --warmup 10 --cpu-budget 0 --step-mode $M > $f.json 2> $f.err || { tail $f.err; exit 1; }
    python -c "import json;d=json.load(open('$f.json'));print('shipped', '$M', $N, '%.4gM env-steps/s %.4f ms kernel %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
  done
  f=$OUT/r06a_w_lat2w_$N
  DUCK_LIB=open_duck_playground_amd/build/libduck_lat2w.so $T 240 python bench.py --config C2 --envs $N --steps 100 --warmup 10 --cpu-budget 0 --step-mode latency > $f.json 2> $f.err || { tail $f.err; exit 1; }
  python -c "import json;d=json.load(open('$f.json'));print('lat2w  ', 'latency', $N, '%.4gM env-steps/s %.4f ms kernel %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
done
