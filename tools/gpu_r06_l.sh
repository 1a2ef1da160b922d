#!/bin/bash
# C4 evidence on the final build (build-id-matched C4 PMC) and the C4 scene's step time at
# 4,096 vs 8,192 envs (is the second round of workgroups at 8,192 a tail cost?).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T="timeout -k 10"
$T 450 bash tools/gpu_pmc.sh r06 C4 > $OUT/r06_pmc_c4.log 2>&1 || { tail -30 $OUT/r06_pmc_c4.log; exit 1; }
tail -25 $OUT/r06_pmc_c4.log
for n in 4096 8192 4096 8192; do
  $T 200 python bench.py --config C4 --envs $n --cpu-budget 0 > $OUT/r06l_c4_$n.json 2> $OUT/r06l.err || { tail -20 $OUT/r06l.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r06l_c4_$n.json'));print('C4 envs $n', '%.4gM env-steps/s %.4f ms' % (d['value']/1e6, d['ms_per_step']))"
done
