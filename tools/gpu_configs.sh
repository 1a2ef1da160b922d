#!/bin/bash
# bench.py for every BASELINE config (C2..C5), one line each, into gpurun_out/bench_<C>.json
set -o pipefail
mkdir -p gpurun_out
for C in C2 C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $C --cpu-budget 0 > gpurun_out/bench_$C.json 2> gpurun_out/bench_$C.err || { tail gpurun_out/bench_$C.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$C.json'));print('$C', d['config']['envs_per_gpu'], 'envs: %.4gM env-steps/s, kernel %.4f ms' % (d['value']/1e6, d['roofline']['kernel_ms']))"
done
