#!/bin/bash
# Per-step latency vs envs per GPU (the floor that decides strong scaling): bench.py lines for
# C2 and C5 at 256 .. 8192 envs into gpurun_out/lat_<C>_<n>.json, one summary line each.
set -o pipefail
mkdir -p gpurun_out
for C in ${CONFIGS:-C2 C5}; do
  for N in ${SIZES:-256 512 1024 2048 3072 4096 6144 8192}; do
    timeout -k 10 240 python bench.py --config $C --envs $N --steps 50 --warmup 10 --cpu-budget 0 \
      > gpurun_out/lat_${C}_$N.json 2> gpurun_out/lat_${C}_$N.err || { tail gpurun_out/lat_${C}_$N.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/lat_${C}_$N.json'));print('$C', $N, 'envs: %.4gM env-steps/s, %.4f ms/step, kernel %.4f ms' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
  done
done
