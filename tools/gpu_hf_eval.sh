#!/bin/bash
# Height-field evidence: kernel vs brute-force prisms (tests + tools/hfield_deviation.py --gpu), C4 / C5 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_physics.py -k "hfield" > gpurun_out/hf2.log 2>&1 || { tail -30 gpurun_out/hf2.log; exit 1; }
grep -E "passed|failed" gpurun_out/hf2.log | tail -1
timeout -k 10 400 python tools/hfield_deviation.py 64 40 --gpu > gpurun_out/hfield_dev_gpu.jsonl || exit 1
cat gpurun_out/hfield_dev_gpu.jsonl
for C in C4 C5; do timeout -k 10 300 python bench.py --config $C --cpu-budget 0 > gpurun_out/bench_r03_$C.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('gpurun_out/bench_r03_$C.json'));print('$C', d['value']/1e6, d['roofline']['kernel_ms'])"; done
