#!/bin/bash
# evidence for the current build: GPU suite, C2-C5 bench lines, latency curves of both kernels, PPO
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r04i}
bash tools/gpu_suite.sh $TAG || exit 1
for C in C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $C --cpu-budget 0 > $OUT/bench_${TAG}_$C.json 2>> $OUT/bench_${TAG}.err || exit 1
done
SIZES="256 512 1024 2048 4096" STEPS=60 bash tools/gpu_latency.sh > $OUT/${TAG}_latency.txt 2>&1 || { tail $OUT/${TAG}_latency.txt; exit 1; }
cat $OUT/${TAG}_latency.txt
bash tools/gpu_ppo_prof.sh $TAG > $OUT/${TAG}_ppo_prof.txt 2>&1 || { tail $OUT/${TAG}_ppo_prof.txt; exit 1; }
head -16 $OUT/${TAG}_ppo_prof.txt
