#!/bin/bash
# Round-end evidence in one GPU call: the PMC profile of the C2 bench (tools/gpu_pmc.sh), then the
# default bench line (CPU baseline included) read against that fresh profile, the whole -m gpu suite
# and the C3-C5 lines. usage (repo root, on the box): bash tools/gpu_round_end.sh TAG
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ -z "$SKIP_HEAD" ]; then
bash tools/gpu_pmc.sh $TAG C2 > $OUT/pmc_$TAG.log 2>&1 || { tail -20 $OUT/pmc_$TAG.log; exit 1; }
cp $OUT/pmc_$TAG/${TAG}_pmc_c2.json $OUT/pmc_$TAG/${TAG}_pmc_c2_stats.csv profiles/ || exit 1
mkdir -p $OUT/pmc_keep && cp profiles/${TAG}_pmc_c2.json profiles/${TAG}_pmc_c2_stats.csv $OUT/pmc_keep/ || exit 1
timeout -k 10 400 python bench.py > $OUT/bench_full_$TAG.json 2> $OUT/bench_full_$TAG.err || { tail $OUT/bench_full_$TAG.err; exit 1; }
cat $OUT/bench_full_$TAG.json
fi
bash tools/gpu_suite.sh $TAG || exit 1
for C in C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $C --cpu-budget 0 > $OUT/bench_${TAG}_$C.json 2>> $OUT/bench_full_$TAG.err || exit 1
done
for C in ${PMC_EXTRA:-}; do
  c=$(echo $C | tr 'A-Z' 'a-z')
  bash tools/gpu_pmc.sh $TAG $C > $OUT/pmc_${TAG}_$c.log 2>&1 || { tail -20 $OUT/pmc_${TAG}_$c.log; exit 1; }
  mkdir -p $OUT/pmc_keep && cp $OUT/pmc_$TAG/${TAG}_pmc_$c.json $OUT/pmc_$TAG/${TAG}_pmc_${c}_stats.csv $OUT/pmc_keep/ || exit 1
done
