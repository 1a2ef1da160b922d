#!/bin/bash
# Round 6 first call: the VALU issue rate against waves per SIMD, the whole GPU suite
# (new: bench.py --gpus 2 run directly, train() raising on the device error word), the direct
# two-rank bench line, the C2 bench line.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 60 ./tools/valu_occupancy_probe > $OUT/r06_valu_occupancy_probe.txt 2>&1 || { cat $OUT/r06_valu_occupancy_probe.txt; exit 1; }
cat $OUT/r06_valu_occupancy_probe.txt
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r06a_gpu_tests.log 2>&1 || { tail -60 $OUT/r06a_gpu_tests.log; exit 1; }
grep -E "passed|failed" $OUT/r06a_gpu_tests.log | tail -2
DUCK_DIST_BACKEND=gloo $T 300 python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-budget 0 > $OUT/r06a_bench_direct2.jsonl 2> $OUT/r06a_bench_direct2.err || { tail -30 $OUT/r06a_bench_direct2.err; exit 1; }
cat $OUT/r06a_bench_direct2.jsonl
$T 300 python bench.py --steps 200 --warmup 20 > $OUT/r06a_bench_C2.json 2> $OUT/r06a_bench_C2.err || { tail -30 $OUT/r06a_bench_C2.err; exit 1; }
cat $OUT/r06a_bench_C2.json
