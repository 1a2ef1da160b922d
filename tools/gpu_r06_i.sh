#!/bin/bash
# Round 6 latency curves (strong scaling): ms per env-step of each step kernel against envs per GPU, C2 and C5.
set -o pipefail
mkdir -p gpurun_out/r06_latency
export TMPDIR=/tmp
for C in C2 C5; do
  MODES="throughput latency paired"; [ $C = C2 ] && MODES="$MODES latency_x2"
  for M in $MODES; do
    for N in 256 512 1024 1536 2048 3072 4096; do
      f=gpurun_out/r06_latency/lat_${C}_${M}_$N
      timeout -k 10 240 python bench.py --config $C --envs $N --steps 100 --warmup 10 --cpu-budget 0 --step-mode $M > $f.json 2> $f.err || { tail $f.err; exit 1; }
      python -c "import json;d=json.load(open('$f.json'));print('$C', '$M', $N, '%.4f ms/step %.4gM env-steps/s' % (d['ms_per_step'], d['value']/1e6))"
    done
  done
done
