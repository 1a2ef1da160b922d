#!/bin/bash
# Latency-mode check in one GPU call: latency == throughput bit for bit (all four scenes), the
# AUTO selection, then C2 / C5 step times at small batches in both modes and a driver-style C2 line.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r04_lat}
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py -x -v -s --timeout 300 --timeout-method thread \
  -k "latency_mode or step_mode_auto" > $OUT/${TAG}_tests.log 2>&1 || { tail -30 $OUT/${TAG}_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/${TAG}_tests.log | tail -8
SIZES="${SIZES:-512 1024}" CONFIGS="${CONFIGS:-C2 C5}" bash tools/gpu_latency.sh > $OUT/${TAG}_curve.txt 2>&1 || { tail $OUT/${TAG}_curve.txt; exit 1; }
cat $OUT/${TAG}_curve.txt
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-budget 0 > $OUT/${TAG}_drv.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$OUT/${TAG}_drv.json'));print('driver-style C2 %.4gM ms_per_step %.4f kernel_ms %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
