#!/bin/bash
# Three back-to-back C2 bench runs (no CPU leg) to gauge run-to-run spread.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --cpu-budget 0 --steps 400 > gpurun_out/b3_$i.json 2> /dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b3_$i.json'));print('value %.4gM  kernel_ms %.4f' % (d['value']/1e6, d['roofline']['kernel_ms']))"
done
