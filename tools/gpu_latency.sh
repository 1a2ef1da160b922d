#!/bin/bash
# Per-step latency vs envs per GPU (the floor that decides strong scaling): bench.py lines for
# C2 and C5 at 256 .. 8192 envs into gpurun_out/lat_<C>_<mode>_<n>.json, one summary line each,
# for each step kernel in MODES (auto picks the latency kernel at <= 4 envs per CU).
set -o pipefail
mkdir -p gpurun_out
for C in ${CONFIGS:-C2 C5}; do
  for M in ${MODES:-throughput latency}; do
    for N in ${SIZES:-256 512 1024 2048 3072 4096 6144 8192}; do
      f=gpurun_out/lat_${C}_${M}_$N
      timeout -k 10 240 python bench.py --config $C --envs $N --steps ${STEPS:-50} --warmup 10 --cpu-budget 0 \
        --step-mode $M > $f.json 2> $f.err || { tail $f.err; exit 1; }
      python -c "import json;d=json.load(open('$f.json'));print('$C', '$M', $N, 'envs: %.4gM env-steps/s, %.4f ms/step, kernel %.4f ms' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
    done
  done
done
